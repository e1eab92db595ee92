"""Known-answer tests for the hot path's integer RNG, scene and camera
producers (CPU only). Anchors come from SURVEY.md §4 / §8a, computed from
the reference's code (ShaderCompute.hlsl:23-48, DxCSApp.cpp:39-134)."""
import ctypes as C
import struct

import numpy as np
import pytest

M32 = 0xFFFFFFFF


def base_hash_py(px: int, py: int) -> int:
    """Independent pure-Python restatement of baseHash (ShaderCompute.hlsl:23-28)."""
    qx = (1103515245 * (((px >> 1) ^ py) & M32)) & M32
    qy = (1103515245 * (((py >> 1) ^ px) & M32)) & M32
    h = (1103515245 * ((qx ^ (qy >> 3)) & M32)) & M32
    return h ^ (h >> 16)


KAT = {(0, 0): 0x00000000, (1, 0): 0xEF388D71, (0, 1): 0xC2A258CB,
       (1023, 575): 0x4DE3FA9F, (1919, 1079): 0xF9940006}


@pytest.mark.parametrize("xy,h", list(KAT.items()))
def test_base_hash_kat(oracle, xy, h):
    assert base_hash_py(*xy) == h
    assert oracle.base_hash(*xy) == h


def test_base_hash_random_agree(oracle):
    rng = np.random.default_rng(1)
    for x, y in rng.integers(0, 2**32, size=(2000, 2), dtype=np.uint64):
        assert oracle.base_hash(int(x), int(y)) == base_hash_py(int(x), int(y))


def _f2u(f):
    return struct.unpack("<I", struct.pack("<f", f))[0]


def hash2_py(seed: float):
    """hash2 (ShaderCompute.hlsl:36-41) in numpy fp32."""
    s = np.float32(seed)
    a = s = np.float32(s + np.float32(0.1))
    b = s = np.float32(s + np.float32(0.1))
    n = base_hash_py(_f2u(a), _f2u(b))
    h0 = np.float32(np.float32(n & 0x7FFFFFFF) / np.float32(2147483648.0))
    h1 = np.float32(np.float32(((n * 48271) & M32) & 0x7FFFFFFF) / np.float32(2147483648.0))
    return h0, h1, s


def test_first_pixel_hash2_kat(oracle):
    """Pixel (0,0): seed p = baseHash(0,0)/2^32 = 0; first hash2 = (0.89364517, 0.14578328), seed -> 0.2."""
    h0, h1, s = hash2_py(0.0)
    assert abs(h0 - 0.89364517) < 1e-7 and abs(h1 - 0.14578328) < 1e-7
    assert s == np.float32(0.2)
    got = oracle.math("hash2", np.array([0.0], np.float32))[0]
    assert (got[0], got[1], got[2]) == (h0, h1, s)


def test_hash_functions_match_python(oracle):
    seeds = np.random.default_rng(2).uniform(0, 1, 500).astype(np.float32)
    got = oracle.math("hash2", seeds)
    for i, sd in enumerate(seeds):
        h0, h1, s = hash2_py(float(sd))
        assert (got[i, 0], got[i, 1], got[i, 2]) == (h0, h1, s)


def test_pixel_seed_kat(oracle):
    # p = float(baseHash(1,0)) / 2^32 = 0.93445665
    assert abs(np.float32(oracle.base_hash(1, 0)) / np.float32(2**32) - 0.93445665) < 1e-7


def test_random_world_kat(rtx, oracle):
    """WorldDef::random_world (DxCSApp.cpp:72-134), MSVC rand() unseeded."""
    w = rtx.random_world(9)
    assert w.count == 326
    np.testing.assert_allclose(w.spheres[4], [-8.492773, 0.2, -8.826026, 0.2], atol=1e-6)
    assert w.mat_types[4] == 0.0
    assert np.bincount(w.mat_types.astype(int)).tolist() == [271, 39, 16]
    # fixed spheres
    np.testing.assert_array_equal(w.spheres[:4], [[0, -1000, 0, 1000], [0, 1, 0, 1], [-4, 1, 0, 1], [4, 1, 0, 1]])
    np.testing.assert_array_equal(w.mat_types[:4], [0, 2, 0, 1])
    # metal albedo in [1, 1.5], fuzz 0 (Appendix A quirk 3)
    met = w.mat_values[w.mat_types == 1]
    assert met[1:, :3].min() >= 1.0 and met[1:, :3].max() <= 1.5 and (met[:, 3] == 0).all()
    w11 = rtx.random_world(11)
    assert w11.count == 486
    assert np.bincount(w11.mat_types.astype(int)).tolist() == [394, 63, 29]
    # product producer == independent oracle restatement, bit for bit
    for ext in (9, 11, 30):
        s, m, v = oracle.random_world(ext)
        wp = rtx.random_world(ext)
        np.testing.assert_array_equal(s, wp.spheres)
        np.testing.assert_array_equal(m, wp.mat_types)
        np.testing.assert_array_equal(v, wp.mat_values)


def test_random_world_100k_kat(rtx):
    """C5 stress scene: grid -159..159 gives 101,124 spheres; capped at 100,000."""
    w = rtx.random_world(159)
    assert w.count == 101124
    w5 = rtx.random_world(159, capacity=100000)
    assert w5.count == 100000
    np.testing.assert_array_equal(w5.spheres, w.spheres[:100000])


def test_test_world(rtx, oracle):
    w = rtx.test_world()
    np.testing.assert_array_equal(w.spheres, [[0, -1000.5, -1, 1000], [0, 0, -1, 0.5], [1, 0, -1, 0.5], [-1, 0, -1, 0.5]])
    np.testing.assert_array_equal(w.mat_types, [0, 0, 1, 2])
    s, m, v = oracle.test_world()
    np.testing.assert_array_equal(s, w.spheres)
    np.testing.assert_array_equal(v, w.mat_values)


def test_ps_world(rtx):
    """Shader_RT.fx:300-335: ground, three small Lambert spheres, glass, Lambert, metal."""
    w = rtx.ps_world()
    assert (w.count, w.depth, w.spp) == (7, 25, 1)
    np.testing.assert_array_equal(w.spheres, np.array([
        [0, -1000, 0, 1000], [3, 0.2, 1.5, 0.2], [4.5, 0.2, 1, 0.2], [4.5, 0.2, 2, 0.2],
        [0, 1, 0, 1], [-4, 1, 0, 1], [4, 1, 0, 1]], np.float32))
    np.testing.assert_array_equal(w.mat_types, [0, 0, 0, 0, 2, 0, 1])
    np.testing.assert_array_equal(w.mat_values[:, :3], np.array([
        [0.5, 0.5, 0.5], [0.2, 0.2, 0.8], [0.2, 0.8, 0.2], [0.8, 0.3, 0.2],
        [1, 1, 1], [0.4, 0.2, 0.1], [0.7, 0.6, 0.5]], np.float32))
    assert w.mat_values[4, 3] == np.float32(1.5) and w.mat_values[6, 3] == 0.0


def test_camera_kat(rtx, oracle):
    """PerFrame::ComputeViewVals for camPos (13,2,3) -> 0, vfov 20, 16:9 (DxCSApp.cpp:39-61, 176-179)."""
    f = rtx.camera_look_at(1024, 576)
    np.testing.assert_allclose(f.origin[:3], [13, 2, 3])
    np.testing.assert_allclose(f.horizontal[:3], [1.901837, 0, -8.241292], atol=2e-6)
    np.testing.assert_allclose(f.vertical[:3], [-0.687246, 4.70499, -0.158595], atol=2e-6)
    np.testing.assert_allclose(f.lower_left[:3], [-0.607295, -2.352495, 4.199944], atol=2e-6)
    assert (f.img_w, f.img_h) == (1024.0, 576.0)
    g = rtx.camera_look_at(1920, 1080)
    assert (g.img_w, g.img_h, g.width, g.height) == (1920.0, 1080.0, 1920, 1080)
    assert bytes(oracle.camera_look_at(1920, 1080)) == bytes(g)


def test_camera_simple(rtx):
    f = rtx.camera_simple(400, 225)
    np.testing.assert_allclose(f.horizontal[:3], [2 * 400 / 225, 0, 0], rtol=1e-7)
    np.testing.assert_allclose(f.lower_left[:3], [-400 / 225, -1, -1], rtol=1e-7)


def test_worlddef_adapter(rtx):
    """The reference's exact WorldDef cbuffer bytes (DxCSApp.cpp:64-71) parse back."""
    w = rtx.random_world(9)
    buf = np.zeros(18448 // 4, np.float32)
    buf[0:4] = [w.count, 50, 60, -1]
    buf[4:4 + 4 * w.count] = w.spheres.ravel()
    mt = buf[4 + 4 * 512:4 + 4 * 512 + 4 * 128]
    mt[:w.count] = w.mat_types  # matTypes[i/4][i%4] == flat i
    buf[4 + 4 * 512 + 4 * 128:4 + 4 * 512 + 4 * 128 + 4 * w.count] = w.mat_values.ravel()
    lib = rtx.load_library()
    sph, mtt, mv = np.zeros(2048, np.float32), np.zeros(512, np.float32), np.zeros(2048, np.float32)
    out = rtx.rtx_world()
    f = rtx._fptr
    assert lib.rtx_world_from_worlddef(buf.ctypes.data, buf.nbytes, f(sph), f(mtt), f(mv), C.byref(out)) == 0
    assert (out.count, out.depth, out.spp) == (326, 50, 60)
    np.testing.assert_array_equal(sph[:4 * 326].reshape(-1, 4), w.spheres)
    np.testing.assert_array_equal(mtt[:326], w.mat_types)
    assert lib.rtx_world_from_worlddef(buf.ctypes.data, 100, f(sph), f(mtt), f(mv), C.byref(out)) != 0


def test_perframe_adapter(rtx):
    """PerFrame bytes with viewVals transposed (DxCSApp.cpp:55-60) -> rows."""
    g = rtx.camera_look_at(1024, 576)
    rows = np.array([g.origin[:], g.horizontal[:], g.vertical[:], g.lower_left[:]], np.float32)
    pf = np.zeros(28, np.float32)
    pf[4:8] = [20.0, np.float32(16 / 9), 2.0, 1024.0]
    pf[12:28] = rows.T.ravel()  # XMMatrixTranspose
    out = rtx.rtx_frame()
    assert rtx.load_library().rtx_frame_from_perframe(pf.ctypes.data, pf.nbytes, 1024, 576, C.byref(out)) == 0
    np.testing.assert_array_equal(np.array(out.horizontal[:]), rows[1])
    np.testing.assert_array_equal(np.array(out.lower_left[:]), rows[3])
    assert (out.img_w, out.img_h) == (1024.0, 576.0)
