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


def grazing_rays(spheres, n, rng, ext_frac=0.05, vert_frac=0.08, xaxis_frac=0.0):
    """Rays whose line passes within 1e-9..1e-2 (relative) of a sphere's
    silhouette, on either side, with origins far down the line; a share of
    near-vertical directions, with xaxis_frac > 0 a share of directions near
    the x axis (the prefilter basis's degenerate direction, rtx_prefilter.h)
    and, with ext_frac > 0, direction lengths outside the prefilter's safe
    range. Returns (n, 6) float32 (origin, direction)."""
    sph = np.asarray(spheres, np.float64)
    pick = rng.integers(0, len(sph), n)
    c, r = sph[pick, :3], sph[pick, 3]
    dirs = rng.normal(size=(n, 3))
    vert = rng.random(n) < vert_frac
    dirs[vert] = np.stack([rng.normal(scale=1e-7, size=vert.sum()), np.sign(rng.normal(size=vert.sum())),
                           rng.normal(scale=1e-7, size=vert.sum())], 1)
    if xaxis_frac > 0:
        xa = (rng.random(n) < xaxis_frac) & ~vert
        eps = 10.0 ** rng.uniform(-9, -3, xa.sum())
        dirs[xa] = np.stack([np.sign(rng.normal(size=xa.sum())), eps * rng.normal(size=xa.sum()),
                             eps * rng.normal(size=xa.sum())], 1)
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    e = np.cross(dirs, rng.normal(size=(n, 3)))
    e /= np.linalg.norm(e, axis=1, keepdims=True)
    delta = np.sign(rng.normal(size=n)) * 10.0 ** rng.uniform(-9, -2, n)
    p = c + (r * (1 + delta))[:, None] * e
    o = p - rng.uniform(-40, 40, n)[:, None] * dirs
    scale = 10.0 ** rng.uniform(-3, 3, n)
    ext = rng.random(n) < ext_frac  # |d| outside the prefilter's safe range: lanes flag every sphere
    scale[ext] = 10.0 ** rng.choice([-7.0, 7.0], ext.sum())
    d = dirs * scale[:, None]
    return np.concatenate([o, d], 1).astype(np.float32)


def camera_rays(frame, n, rng):
    """Primary rays of a DxCSApp camera (get_ray, ShaderCompute.hlsl:118-127)
    at random (s, t) in [0, 1]^2, float32-representable, as (n, 6) float64."""
    org = np.array(frame.origin[:3], np.float64)
    hor, ver, llc = (np.array(v[:3], np.float64) for v in (frame.horizontal, frame.vertical, frame.lower_left))
    st = rng.uniform(0, 1, (n, 2))
    d = llc + st[:, :1] * hor + st[:, 1:] * ver - org
    rays = np.concatenate([np.repeat(org[None], n, 0), d], 1)
    return rays.astype(np.float32).astype(np.float64)


def scene_digest(spheres):
    """sha256 of a scene's float32 (center, radius) array: the large golden
    fixtures name their scene by generator + digest instead of storing it."""
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(spheres, np.float32).tobytes()).hexdigest()
