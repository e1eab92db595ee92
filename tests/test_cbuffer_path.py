"""The reference's own cbuffer bytes, on the
CPU: rtx_app.cpp fills WorldDef (18,448 B, DxCSApp.cpp:64-71, random_world
:72-134) and PerFrame (112 B, :30-37, ComputeViewVals :39-61 with
DxCSApp::Update's focus distance :488) exactly as DxCSApp lays them out, and
the library's adapters (rtx_world_from_worlddef / rtx_frame_from_perframe)
turn them into the scene and frame the render takes. Those must equal the
direct producers' (rtx_scene_random_world, rtx_camera_look_at) bit for bit;
the GPU test renders the frame (test_gpu_parity.py
test_reference_frame_through_cbuffer_bytes)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "raytrace-we-gpu_amd", "lib")


@pytest.fixture(scope="module")
def dumped(tmp_path_factory):
    if not os.path.exists(os.path.join(LIBDIR, "librtx.so")):
        pytest.fail("librtx.so missing: build first")
    d = tmp_path_factory.mktemp("cb")
    exe = str(d / "cbuffer_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"),
                    "-o", exe, os.path.join(ROOT, "tests", "cbuffer_check.cpp"),
                    os.path.join(ROOT, "raytrace-we-gpu_amd", "csrc", "rtx_app.cpp"),
                    "-L", LIBDIR, "-lrtx", "-Wl,-rpath," + LIBDIR], check=True)
    subprocess.run([exe, str(d)], check=True)
    return d


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def test_worlddef_bytes_layout_and_parse(dumped, rtx):
    raw = np.fromfile(dumped / "worlddef.bin", np.float32)
    assert raw.size * 4 == 18448
    ref = rtx.random_world(9, depth=50, spp=60)  # 326 spheres (DxCSApp.cpp:95-97)
    n = ref.count
    np.testing.assert_array_equal(raw[:4], np.float32([n, 50, 60, -1]))  # sceneValues (:133)
    spheres = raw[4:4 + 4 * 512].reshape(512, 4)
    mat_types = raw[4 + 4 * 512:4 + 4 * 512 + 4 * 128]  # matTypes[i/4][i%4] = flat index i
    mat_values = raw[4 + 4 * 512 + 4 * 128:].reshape(512, 4)
    assert (bits(spheres[:n]) == bits(ref.spheres)).all() and not spheres[n:].any()
    assert (bits(mat_types[:n]) == bits(ref.mat_types)).all()
    assert (bits(mat_values[:n]) == bits(ref.mat_values)).all()
    count, depth, spp = map(int, open(dumped / "world.txt").read().split())
    assert (count, depth, spp) == (n, 50, 60)
    parsed = np.fromfile(dumped / "world.f32", np.float32).reshape(n, 9)
    assert (bits(parsed[:, :4]) == bits(ref.spheres)).all()
    assert (bits(parsed[:, 4]) == bits(ref.mat_types)).all()
    assert (bits(parsed[:, 5:]) == bits(ref.mat_values)).all()


def test_perframe_bytes_layout_and_parse(dumped, rtx):
    raw = np.fromfile(dumped / "perframe.bin", np.float32)
    assert raw.size * 4 == 112
    np.testing.assert_array_equal(raw[4:8], np.float32([20.0, 16.0 / 9.0, 2.0, 1024.0]))  # perspectiveVals (:179)
    np.testing.assert_array_equal(raw[8:12], np.float32([1, 1, 1, 1]))                    # currSamples, frame 1
    want = rtx.camera_look_at(1024, 576, aspect=16.0 / 9.0)  # ComputeViewVals, focus |from - at|
    rows = [np.ctypeslib.as_array(getattr(want, r)) for r in ("origin", "horizontal", "vertical", "lower_left")]
    view_t = raw[12:28].reshape(4, 4)  # stored transposed (:60): column i = row i
    for i, r in enumerate(rows):
        assert (bits(view_t[:, i]) == bits(r)).all()
    got = rtx.rtx_frame.from_buffer_copy(open(dumped / "frame.bin", "rb").read())
    for name in ("origin", "horizontal", "vertical", "lower_left"):
        assert (bits(np.ctypeslib.as_array(getattr(got, name))) ==
                bits(np.ctypeslib.as_array(getattr(want, name)))).all(), name
    assert bits(got.img_w) == bits(want.img_w) and bits(got.img_h) == bits(want.img_h)
    assert (got.width, got.height, got.rng_mode, got.frame_index, got.flags) == (1024, 576, 0, 0, 0)
    assert got.lens_u[3] == 0.0  # pinhole, as the reference's shader (aperture unused, :179)
