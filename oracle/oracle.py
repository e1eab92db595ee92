"""oracle.py — ctypes wrapper of oracle/lib/liboracle.so.

TEST INFRASTRUCTURE ONLY (see rtx_oracle.h): imported by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker or
the timed CPU baseline — never by the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "liboracle.so")
REF_GOLDEN = os.path.join(HERE, "_ref", "ref_golden")
FN = dict(sqrt=0, div=1, sin=2, cos=3, log2=4, exp2=5, pow=6, basehash=7,
          hash1=8, hash2=9, hash3=10, rius=11, lambert_dir=12, lambert_dir_guard=13)


class or_world(C.Structure):
    _fields_ = [("count", C.c_uint32), ("depth", C.c_uint32), ("spp", C.c_uint32),
                ("reserved", C.c_uint32), ("spheres", C.POINTER(C.c_float)),
                ("mat_types", C.POINTER(C.c_float)), ("mat_values", C.POINTER(C.c_float))]


class or_frame(C.Structure):
    _fields_ = [("origin", C.c_float * 4), ("horizontal", C.c_float * 4),
                ("vertical", C.c_float * 4), ("lower_left", C.c_float * 4),
                ("img_w", C.c_float), ("img_h", C.c_float), ("width", C.c_uint32),
                ("height", C.c_uint32), ("rng_mode", C.c_uint32), ("frame_index", C.c_uint32),
                ("flags", C.c_uint32), ("reserved", C.c_uint32),
                ("lens_u", C.c_float * 4), ("lens_v", C.c_float * 4)]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = C.CDLL(LIB_PATH)
        f, d, u32 = C.POINTER(C.c_float), C.POINTER(C.c_double), C.c_uint32
        L.or_render_rows.argtypes = [C.POINTER(or_world), C.POINTER(or_frame), C.POINTER(u32), u32,
                                     f, C.c_int, C.c_int, C.POINTER(C.c_uint64)]
        L.or_render_rows_linear.argtypes = [C.POINTER(or_world), C.POINTER(or_frame), C.POINTER(u32),
                                            u32, f, C.c_int, C.POINTER(C.c_uint64)]
        L.or_hit_world_f32.argtypes = [C.POINTER(or_world), f, u32, C.c_float, C.c_float, f]
        L.or_hit_world_f64.argtypes = [d, u32, d, u32, C.c_double, C.c_double, d]
        L.or_camera_simple_rays_f64.argtypes = [u32, u32, d, u32, d]
        L.or_math.argtypes = [C.c_int, f, f, u32, f]
        L.or_base_hash.argtypes = [u32, u32]
        L.or_base_hash.restype = u32
        L.or_random_world.argtypes = [C.c_int32, u32, f, f, f, C.POINTER(u32)]
        L.or_test_world.argtypes = [f, f, f, C.POINTER(u32)]
        L.or_camera_look_at.argtypes = [f, f, f, C.c_float, C.c_float, C.c_float, u32, u32,
                                        C.POINTER(or_frame)]
        L.or_camera_simple.argtypes = [u32, u32, C.POINTER(or_frame)]
        _lib = L
    return _lib


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _d(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _world_struct(spheres, mat_types, mat_values, depth, spp):
    keep = [np.ascontiguousarray(spheres, np.float32), np.ascontiguousarray(mat_types, np.float32),
            np.ascontiguousarray(mat_values, np.float32)]
    w = or_world()
    w.count, w.depth, w.spp, w.reserved = keep[0].shape[0], depth, spp, 0
    w.spheres, w.mat_types, w.mat_values = _f(keep[0]), _f(keep[1]), _f(keep[2])
    return w, keep


def frame_from(frame) -> or_frame:
    """Copy an rtx.rtx_frame (identical layout) or an or_frame."""
    f = or_frame()
    C.memmove(C.byref(f), C.byref(frame), C.sizeof(or_frame))
    return f


def render_rows(world, frame, ys: Sequence[int], nthreads: int = 1, precision: int = 32):
    """Render global rows `ys` -> (len(ys), W, 4) float32 and the segment count.
    `world` has .spheres/.mat_types/.mat_values/.depth/.spp (rtx.World)."""
    ys = np.ascontiguousarray(ys, np.uint32)
    f = frame_from(frame)
    w, keep = _world_struct(world.spheres, world.mat_types, world.mat_values, world.depth, world.spp)
    out = np.zeros((ys.size, f.width, 4), np.float32)
    segs = C.c_uint64(0)
    rc = lib().or_render_rows(C.byref(w), C.byref(f), ys.ctypes.data_as(C.POINTER(C.c_uint32)),
                              ys.size, _f(out), nthreads, precision, C.byref(segs))
    if rc != 0:
        raise RuntimeError("or_render_rows failed")
    del keep
    return out, int(segs.value)


def render_rows_linear(world, frame, ys: Sequence[int], nthreads: int = 1):
    """Per-pixel linear sample sums (progressive-accumulation contribution)."""
    ys = np.ascontiguousarray(ys, np.uint32)
    f = frame_from(frame)
    w, keep = _world_struct(world.spheres, world.mat_types, world.mat_values, world.depth, world.spp)
    out = np.zeros((ys.size, f.width, 4), np.float32)
    segs = C.c_uint64(0)
    if lib().or_render_rows_linear(C.byref(w), C.byref(f), ys.ctypes.data_as(C.POINTER(C.c_uint32)),
                                   ys.size, _f(out), nthreads, C.byref(segs)) != 0:
        raise RuntimeError("or_render_rows_linear failed")
    del keep
    return out, int(segs.value)


def hit_world_f32(world, rays, t_min=0.001, t_max=float("inf")):
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
    w, keep = _world_struct(world.spheres, world.mat_types, world.mat_values, 1, 1)
    out = np.zeros((rays.shape[0], 10), np.float32)
    if lib().or_hit_world_f32(C.byref(w), _f(rays), rays.shape[0], t_min, t_max, _f(out)) != 0:
        raise RuntimeError("or_hit_world_f32 failed")
    return out


def hit_world_f64(spheres, rays, t_min=0.001, t_max=float("inf")):
    sph = np.ascontiguousarray(spheres, np.float64).reshape(-1, 4)
    rays = np.ascontiguousarray(rays, np.float64).reshape(-1, 6)
    out = np.zeros((rays.shape[0], 10), np.float64)
    if lib().or_hit_world_f64(_d(sph), sph.shape[0], _d(rays), rays.shape[0], t_min, t_max,
                              _d(out)) != 0:
        raise RuntimeError("or_hit_world_f64 failed")
    return out


def camera_simple_rays_f64(width, height, uv):
    uv = np.ascontiguousarray(uv, np.float64).reshape(-1, 2)
    out = np.zeros((uv.shape[0], 6), np.float64)
    lib().or_camera_simple_rays_f64(width, height, _d(uv), uv.shape[0], _d(out))
    return out


def math(fn: str, in0, in1=None):
    a = np.ascontiguousarray(in0, np.float32)
    b = None if in1 is None else np.ascontiguousarray(in1, np.float32)
    out = np.zeros(3 * a.size, np.float32)
    if lib().or_math(FN[fn], _f(a), _f(b) if b is not None else None, a.size, _f(out)) != 0:
        raise RuntimeError("or_math failed")
    return out.reshape(a.size, 3) if FN[fn] >= FN["hash1"] else out[:a.size]


def lambert_dir(p, nrm, rius, guard: bool):
    """normalize(((p + normal) + rius) - p), optionally near-zero guarded
    (RTX_FN_LAMBERT_DIR[_GUARD]); arrays of shape (n, 3)."""
    a = np.ascontiguousarray(p, np.float32).reshape(-1, 3)
    b = np.ascontiguousarray(np.concatenate([np.reshape(nrm, (-1, 3)), np.reshape(rius, (-1, 3))], 1), np.float32)
    out = np.zeros_like(a)
    fn = FN["lambert_dir_guard" if guard else "lambert_dir"]
    if lib().or_math(fn, _f(a), _f(b), a.shape[0], _f(out)) != 0:
        raise RuntimeError("or_math failed")
    return out


def base_hash(x: int, y: int) -> int:
    return int(lib().or_base_hash(x, y))


def random_world(ext: int, capacity: Optional[int] = None):
    cap = capacity if capacity is not None else 4 + (2 * ext) ** 2
    sph, mt, mv = np.zeros((cap, 4), np.float32), np.zeros(cap, np.float32), np.zeros((cap, 4), np.float32)
    n = C.c_uint32()
    lib().or_random_world(ext, cap, _f(sph), _f(mt), _f(mv), C.byref(n))
    k = n.value
    return sph[:k].copy(), mt[:k].copy(), mv[:k].copy()


def test_world():
    sph, mt, mv = np.zeros((4, 4), np.float32), np.zeros(4, np.float32), np.zeros((4, 4), np.float32)
    n = C.c_uint32()
    lib().or_test_world(_f(sph), _f(mt), _f(mv), C.byref(n))
    return sph, mt, mv


def camera_look_at(width, height, look_from=(13, 2, 3), look_at=(0, 0, 0), vup=(0, 1, 0),
                   vfov=20.0, aspect=16.0 / 9.0, focus_dist=0.0) -> or_frame:
    a = [np.asarray(v, np.float32) for v in (look_from, look_at, vup)]
    f = or_frame()
    lib().or_camera_look_at(_f(a[0]), _f(a[1]), _f(a[2]), vfov, np.float32(aspect), focus_dist,
                            width, height, C.byref(f))
    return f


def camera_simple(width, height) -> or_frame:
    f = or_frame()
    lib().or_camera_simple(width, height, C.byref(f))
    return f


def run_ref_golden(stdin_text: str) -> str:
    """Run the compiled reference driver (oracle/_ref/ref_golden). Only in the
    build container (needs /root/reference at build time)."""
    if not os.path.exists(REF_GOLDEN):
        raise FileNotFoundError(REF_GOLDEN)
    return subprocess.run([REF_GOLDEN], input=stdin_text, capture_output=True, text=True,
                          check=True).stdout
