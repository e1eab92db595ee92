"""Image output contract: rtx_cli's writers (rtx_app.cpp)
round-trip on the CPU. The framebuffer is RGBA32F with row 0 = image bottom
(ShaderCompute.hlsl:306-307 with the display quad's texcoords,
DxCSApp.cpp:297-303): the PFM keeps that order (PFM rows run bottom to top)
and all 32 bits; the PPM is 8-bit, top row first, each channel clamped to
[0, 1] (NaN -> 0) and scaled by 255.999 (Color.h:6-11)."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "raytrace-we-gpu_amd", "lib")


@pytest.fixture(scope="module")
def writer(tmp_path_factory):
    if not os.path.exists(os.path.join(LIBDIR, "librtx.so")):
        pytest.fail("librtx.so missing: build first")
    exe = str(tmp_path_factory.mktemp("iw") / "image_writer_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"),
                    "-o", exe, os.path.join(ROOT, "tests", "image_writer_check.cpp"),
                    os.path.join(ROOT, "raytrace-we-gpu_amd", "csrc", "rtx_app.cpp"),
                    "-L", LIBDIR, "-lrtx", "-Wl,-rpath," + LIBDIR], check=True)
    return exe


def read_pnm(path):
    with open(path, "rb") as f:
        magic = f.readline().strip()
        w, h = map(int, f.readline().split())
        scale = f.readline().strip()
        data = f.read()
    return magic, w, h, scale, data


@pytest.mark.parametrize("w,h", [(7, 5), (1, 1), (64, 3)])
def test_pfm_and_ppm_round_trip(writer, tmp_path, w, h):
    rng = np.random.default_rng(w * 100 + h)
    img = rng.uniform(-0.5, 1.5, (h, w, 4)).astype(np.float32)  # values outside [0, 1] on purpose
    img[..., 3] = 1.0
    img.flat[::11] = np.nan
    img.flat[5::13] = np.float32(1.0)
    img.flat[7::17] = np.float32(0.99999994)
    src = tmp_path / "in.f32"
    img.tofile(src)
    pfm, ppm = tmp_path / "o.pfm", tmp_path / "o.ppm"
    subprocess.run([writer, str(w), str(h), str(src), str(pfm), str(ppm)], check=True)

    magic, pw, ph, scale, data = read_pnm(pfm)
    assert (magic, pw, ph) == (b"PF", w, h) and float(scale) < 0  # little endian
    got = np.frombuffer(data, "<f4").reshape(h, w, 3)  # bottom row first, like the framebuffer
    same = (got.view(np.uint32) == img[..., :3].view(np.uint32)) | (np.isnan(got) & np.isnan(img[..., :3]))
    assert same.all()

    magic, pw, ph, scale, data = read_pnm(ppm)
    assert (magic, pw, ph, scale) == (b"P6", w, h, b"255")
    got8 = np.frombuffer(data, np.uint8).reshape(h, w, 3)
    v = np.nan_to_num(img[::-1, :, :3], nan=0.0)  # top row first
    want = (np.float32(255.999) * np.clip(v, 0.0, 1.0).astype(np.float32)).astype(np.uint8)
    np.testing.assert_array_equal(got8, want)
    assert got8.max() <= 255 and (got8[np.isnan(img[::-1, :, :3])] == 0).all()
