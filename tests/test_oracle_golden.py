"""Pin the oracle against the reference's own outputs (CPU only).

The golden vectors (tests/golden/*.json) were produced by the reference's
CPU geometry library compiled from /root/reference (Sphere.cpp,
Hittable_list.cpp, Camera.cpp) via tests/golden/make_golden.py.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from cases import lambert_cases
from golden_cases import case_ids, load_case
from tolerance import check_hits_against_fp64


def _load(name):
    return json.load(open(os.path.join(GOLDEN, name)))


class _W:
    def __init__(self, spheres):
        self.spheres = np.asarray(spheres, np.float32)
        self.mat_types = np.zeros(len(spheres), np.float32)
        self.mat_values = np.zeros((len(spheres), 4), np.float32)


def _cases():
    for name, k in case_ids():
        yield pytest.param(name, k, id=f"{name}-{k}")


def _load_case(oracle, name, k):
    return load_case(name, k, lambda ext, cap: oracle.random_world(ext, cap)[0])


def test_camera_simple_fp64_bit_exact(oracle):
    """Camera(400,225).get_ray (Camera.h:9-26) restated in fp64 == reference, bit for bit."""
    d = _load("camera_simple_400x225.json")
    got = oracle.camera_simple_rays_f64(d["width"], d["height"], np.array(d["uv"]))
    np.testing.assert_array_equal(got, np.array(d["rays"]))


@pytest.mark.parametrize("name,k", list(_cases()))
def test_hit_world_fp64_bit_exact(oracle, name, k):
    """Sphere::hit + Hittable_list::hit restated in fp64 == compiled reference, every field."""
    c = _load_case(oracle, name, k)
    got = oracle.hit_world_f64(c["spheres"].astype(np.float64), c["rays"], c["t_min"], c["t_max"])
    np.testing.assert_array_equal(got, c["expected"])


@pytest.mark.parametrize("name,k", list(_cases()))
def test_hit_world_fp32_twin_within_tolerance(oracle, name, k):
    """The fp32 twin (the GPU's arithmetic) vs the reference's fp64 result,
    within the conditioning-based fp32 bound of tests/tolerance.py (grazing
    rays: ill-conditioned ones may decide differently, the rest may not)."""
    c = _load_case(oracle, name, k)
    got = oracle.hit_world_f32(_W(c["spheres"]), c["rays"].astype(np.float32), c["t_min"], c["t_max"])
    res = check_hits_against_fp64(c["spheres"], c["rays"], got, c["expected"], c["t_min"], c["t_max"],
                                  allow_ill=c["allow_ill"])
    worst = res[0] if c["allow_ill"] else res
    assert worst < 0.5
    if c["allow_ill"]:
        print(f"{name}: {res[1]} ill-conditioned rays decide differently in fp32")


def test_device_math_accuracy(oracle):
    """The twin's sin/cos/pow are accurate restatements of the HLSL intrinsics."""
    x = np.linspace(0, 2 * np.pi, 20001).astype(np.float32)
    np.testing.assert_allclose(oracle.math("sin", x), np.sin(x.astype(np.float64)), atol=3e-7)
    np.testing.assert_allclose(oracle.math("cos", x), np.cos(x.astype(np.float64)), atol=3e-7)
    p = np.linspace(1e-6, 2, 20001).astype(np.float32)
    for y in (1 / 3, 1 / 2.2):
        np.testing.assert_allclose(oracle.math("pow", p, np.full_like(p, y)),
                                   np.power(p.astype(np.float64), np.float32(y)), rtol=2e-6)


def test_c1_oracle_golden_rows(oracle, rtx):
    """Regression pin of the fp32 twin itself: C1 rows committed by
    tests/golden/make_oracle_golden.py (oracle output, not a reference artifact)."""
    gold = np.load(os.path.join(GOLDEN, "c1_oracle_rows.npz"))
    world = rtx.test_world(depth=12, spp=20)
    frame = rtx.camera_simple(400, 225)
    got, _ = oracle.render_rows(world, frame, gold["rows"], nthreads=4)
    np.testing.assert_array_equal(got.view(np.uint32), gold["pixels"].view(np.uint32))


def test_fp32_twin_vs_fp64_image(oracle, rtx):
    """The fp32 twin against the fp64 restatement (Sphere.cpp algebra in
    double, libm transcendentals, same RNG chain) on the C1 image: paths
    that flip hit/miss on an ulp decorrelate, so the check is statistical:
    per-channel means within 1e-3 and PSNR >= 45 dB (measured ~57 dB)."""
    world = rtx.test_world(depth=12, spp=20)
    frame = rtx.camera_simple(400, 225)
    a, _ = oracle.render_rows(world, frame, np.arange(225), nthreads=8)
    b, _ = oracle.render_rows(world, frame, np.arange(225), nthreads=8, precision=64)
    assert np.abs(a[..., :3].mean((0, 1)) - b[..., :3].mean((0, 1))).max() < 1e-3
    mse = float(((a[..., :3] - b[..., :3]) ** 2).mean())
    assert 10 * np.log10(1.0 / mse) >= 45.0


def test_fp32_twin_vs_fp64_c2_rows(oracle, rtx):
    """The north star's tolerance statement at C2: the fp32
    path (the GPU's arithmetic, bit-exact with the GPU) against the fp64
    CPU path (Sphere.cpp/Hittable_list.cpp algebra in double, same RNG
    chain) on the RTIOW final scene (486 spheres), spp 100, depth 50, over 8
    full 1920-pixel rows. Paths that flip on an ulp decorrelate (a glass or
    metal bounce), so the bar is statistical: per-channel means within 1e-3
    and PSNR >= 35 dB. Measured: means within 3.2e-5, PSNR 49.2 dB, 3,126 of
    15,360 pixels differ by more than 1e-5 (their paths diverged somewhere)."""
    world = rtx.random_world(11, depth=50, spp=100)
    frame = rtx.camera_look_at(1920, 1080)
    rows = np.linspace(60, 1020, 8).astype(np.uint32)
    a, _ = oracle.render_rows(world, frame, rows, nthreads=8)
    b, _ = oracle.render_rows(world, frame, rows, nthreads=8, precision=64)
    d = a[..., :3].astype(np.float64) - b[..., :3]
    mean_err = np.abs(a[..., :3].mean((0, 1)) - b[..., :3].mean((0, 1))).max()
    psnr = 10 * np.log10(1.0 / float((d ** 2).mean()))
    divergent = int((np.abs(d).max(-1) > 1e-5).sum())
    print(f"C2 rows: mean err {mean_err:.2e}, PSNR {psnr:.1f} dB, {divergent} of {d.shape[0] * d.shape[1]} "
          f"pixels differ by > 1e-5")
    assert mean_err < 1e-3
    assert psnr >= 35.0
    assert divergent < d.shape[0] * d.shape[1] // 2


def test_oracle_row_order_and_threads_invariant(oracle, rtx):
    world = rtx.random_world(4, depth=20, spp=3)
    frame = rtx.camera_look_at(64, 36, aspect=64 / 36)
    rows = np.arange(36)
    a, sa = oracle.render_rows(world, frame, rows, nthreads=1)
    b, sb = oracle.render_rows(world, frame, rows[::-1].copy(), nthreads=5)
    np.testing.assert_array_equal(a.view(np.uint32), b[::-1].view(np.uint32))
    assert sa == sb


def test_lambert_guard_oracle(oracle):
    """f-4: without the guard a zero diffuse direction normalises to NaN (the
    compute shader, ShaderCompute.hlsl:211-212); with it, to the normal
    (Shader_RT.fx:222-225, near_zero of ShaderCompute.hlsl:70-74)."""
    p, nrm, rius, nz = lambert_cases()
    plain = oracle.lambert_dir(p, nrm, rius, guard=False)
    guard = oracle.lambert_dir(p, nrm, rius, guard=True)
    np.testing.assert_array_equal(plain[:-nz].view(np.uint32), guard[:-nz].view(np.uint32))
    assert np.isnan(plain[-nz:]).all()
    np.testing.assert_array_equal(guard[-nz:], nrm[-nz:])


def test_lambert_guard_frame_flag(oracle, rtx):
    """On ordinary frames the guard never fires: the same image bit for bit."""
    world = rtx.ps_world(depth=25, spp=2)
    f0 = rtx.camera_look_at(48, 27, aspect=48 / 27)
    f1 = rtx.camera_look_at(48, 27, aspect=48 / 27)
    f1.flags = rtx.FRAME_LAMBERT_GUARD
    a, sa = oracle.render_rows(world, f0, np.arange(27))
    b, sb = oracle.render_rows(world, f1, np.arange(27))
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    assert sa == sb


def test_thin_lens_changes_only_when_enabled(oracle, rtx):
    world = rtx.random_world(4, depth=10, spp=2)
    pin = rtx.camera_look_at(32, 18, aspect=32 / 18)
    a, _ = oracle.render_rows(world, pin, np.arange(18))
    b, _ = oracle.render_rows(world, rtx.set_aperture(rtx.camera_look_at(32, 18, aspect=32 / 18), 0.0), np.arange(18))
    c, _ = oracle.render_rows(world, rtx.set_aperture(rtx.camera_look_at(32, 18, aspect=32 / 18), 0.5), np.arange(18))
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    assert (a != c).mean() > 0.1
