"""Shared input cases for the CPU and GPU parity tests."""
import numpy as np


def lambert_cases(n=4000, seed=5):
    """Random (p, normal, rius) plus engineered zero directions: at |p| = 1000
    the fp32 sums ((p + n) + rius) - p cancel to exactly 0 when rius ~ -n."""
    rng = np.random.default_rng(seed)
    p = rng.uniform(-20, 20, (n, 3)).astype(np.float32)
    nrm = rng.normal(size=(n, 3))
    nrm = (nrm / np.linalg.norm(nrm, axis=1, keepdims=True)).astype(np.float32)
    rius = rng.uniform(-0.5, 0.5, (n, 3)).astype(np.float32)
    zp = np.array([[0, 1000, 0], [1000, 0, 0], [0, 0, -1000], [512, -512, 1024]], np.float32)
    zn = np.array([[0, 1, 0], [1, 0, 0], [0, 0, -1], [0, -1, 0]], np.float32)
    zr = -zn * np.float32(0.99999994)
    return np.concatenate([p, zp]), np.concatenate([nrm, zn]), np.concatenate([rius, zr]), len(zp)
