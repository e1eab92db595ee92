"""The speculative chain's seed jump, checked on the CPU.

The chain RNG's state is one float advanced by `seed += 0.1` twice per hash
call (ShaderCompute.hlsl:30-48). The speculative chain needs
the seed after 2k additions for arbitrary k; raytrace-we-gpu_amd/csrc/
rtx_seed.h computes it binade by binade. tests/seed_check.cpp compares it with
the literal additions (the oracle's sequence) and must find no mismatch; the
GPU side is test_gpu_parity.py::test_seed_advance_matches_literal_steps.
"""
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "seed_check.cpp")


def test_seed_jump_equals_literal_steps(tmp_path):
    exe = str(tmp_path / "seed_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe, SRC], check=True)
    out = subprocess.run([exe, "6000"], capture_output=True, text=True, timeout=120)
    rep = json.loads(out.stdout.strip().splitlines()[-1])
    assert out.returncode == 0 and rep["mismatches"] == 0, out.stderr
    assert rep["checked"] > 10_000_000


def test_oracle_literal_seed_steps():
    """The oracle's fn 14 is the literal loop: n additions of 0.1f."""
    import oracle

    s0 = np.array([0.0, 0.3, 0.7, 123.25], np.float32)
    n = np.array([0, 1, 7, 1000], np.float32)
    got = oracle.math("seed_steps", s0, n)
    want = []
    for s, k in zip(s0, n):
        v = np.float32(s)
        for _ in range(int(k)):
            v = np.float32(v + np.float32(0.1))
        want.append(v)
    assert got.view(np.uint32).tolist() == np.array(want, np.float32).view(np.uint32).tolist()
