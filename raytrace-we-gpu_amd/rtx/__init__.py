"""rtx — Python host binding of librtx.so (the MI355X path tracer's C-ABI).

Thin ctypes layer over ``include/rtx.h``; the compute path is the HIP kernel
in ``raytrace-we-gpu_amd/csrc``. There is deliberately no CPU fallback: if
``librtx.so`` is missing, importing the GPU entry points raises.

Host surface mirrors the reference app (CSVersion/DxCSApp.cpp):
  * :func:`random_world` / :func:`test_world`  ~ WorldDef::random_world /
    test_world (DxCSApp.cpp:72-157)
  * :func:`camera_look_at`                    ~ PerFrame::ComputeViewVals
    (DxCSApp.cpp:39-61) + focus distance (:488)
  * :class:`Context`                           ~ CDx11Base + DxCSApp resource
    lifetime (upload_world = WorldDef cbuffer, set_frame = PerFrame cbuffer,
    render_rows = Dispatch, DxCSApp.cpp:524)
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("RTX_LIB", os.path.join(_PKG_DIR, "lib", "librtx.so"))

RTX_OK = 0
RTX_ERR_INCOMPLETE = -5  # a render launch left pixels unwritten (ABI 1.3)
SCHEDULE_ABI = 140  # the rtx_schedule layout this module passes (ABI 1.4.0)
DEBUG_CULLED = 0xFFFFFFFF  # rtx_debug_hit_world_from: the culled scan (include/rtx.h RTX_DEBUG_CULLED)


def DEBUG_CULLED_COOP(q: int) -> int:
    """rtx_debug_hit_world_from: the culled group coop, q rays per wave (RTX_DEBUG_CULLED_COOP)."""
    if not 1 <= q <= 64:
        raise ValueError("q must be in 1..64")
    return 0xFFFFFF00 | q


def DEBUG_CULLED_COOP_LANE(q: int) -> int:
    """rtx_debug_hit_world_from: the culled group coop with the per-lane walk
    (the per-sample kernel's form), q rays per wave (RTX_DEBUG_CULLED_COOP_LANE)."""
    if not 1 <= q <= 64:
        raise ValueError("q must be in 1..64")
    return 0xFFFFFE00 | q
MAT_LAMBERT, MAT_METAL, MAT_DIELECTRIC = 0, 1, 2
RNG_CHAIN, RNG_PER_SAMPLE = 0, 1
SCAN_MODES = {"auto": 0, "linear": 1}  # rtx_set_scan_mode (RTX_SCAN_AUTO / RTX_SCAN_LINEAR)
FN = dict(sqrt=0, div=1, sin=2, cos=3, log2=4, exp2=5, pow=6, basehash=7,
          hash1=8, hash2=9, hash3=10, rius=11, lambert_dir=12, lambert_dir_guard=13)
FRAME_LAMBERT_GUARD = 1  # rtx_frame.flags bit (RTX_FRAME_LAMBERT_GUARD)


class RtxError(RuntimeError):
    pass


class rtx_world(C.Structure):
    _fields_ = [("count", C.c_uint32), ("depth", C.c_uint32), ("spp", C.c_uint32),
                ("reserved", C.c_uint32), ("spheres", C.POINTER(C.c_float)),
                ("mat_types", C.POINTER(C.c_float)), ("mat_values", C.POINTER(C.c_float))]


class rtx_frame(C.Structure):
    _fields_ = [("origin", C.c_float * 4), ("horizontal", C.c_float * 4),
                ("vertical", C.c_float * 4), ("lower_left", C.c_float * 4),
                ("img_w", C.c_float), ("img_h", C.c_float), ("width", C.c_uint32),
                ("height", C.c_uint32), ("rng_mode", C.c_uint32), ("frame_index", C.c_uint32),
                ("flags", C.c_uint32), ("reserved", C.c_uint32),
                ("lens_u", C.c_float * 4), ("lens_v", C.c_float * 4)]


class rtx_schedule(C.Structure):
    """The chain render's schedule (include/rtx.h rtx_schedule)."""
    _fields_ = [("tier1_bar", C.c_float), ("tier1_bar_small", C.c_float), ("tier1_bar_low", C.c_float),
                ("tier2_bar_small", C.c_float), ("tier2_bar_medium", C.c_float), ("tier2_bar", C.c_float),
                ("small_share", C.c_float),
                ("low_share", C.c_float), ("medium_share", C.c_float), ("hot_fraction", C.c_float),
                ("occupancy_small", C.c_float), ("occupancy_low", C.c_float), ("occupancy_normal", C.c_float),
                ("trace_small", C.c_float), ("trace_low", C.c_float), ("trace_medium", C.c_float),
                ("trace_large", C.c_float), ("promote_small", C.c_float), ("promote_low", C.c_float),
                ("promote_medium", C.c_float), ("promote_large", C.c_float), ("promote_big_scene", C.c_float),
                ("trace_solo_bar", C.c_float),
                ("tail_coop_max", C.c_uint32), ("tail_coop_max_large", C.c_uint32), ("tier1_priority", C.c_uint32), ("tier2_priority", C.c_uint32),
                ("hot_priority", C.c_uint32), ("refill_chunk", C.c_uint32), ("trace_group", C.c_uint32),
                ("prepass_cap_split", C.c_uint32), ("prio_bar1", C.c_float), ("prio_bar2", C.c_float),
                ("prio_bar3", C.c_float), ("reserved", C.c_uint32)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_ if name != "reserved"}


class rtx_stats(C.Structure):
    _fields_ = [("kernel_ms", C.c_double), ("launches", C.c_uint64), ("samples", C.c_uint64),
                ("segments", C.c_uint64), ("sphere_tests", C.c_uint64)]


_lib = None


def load_library(path: Optional[str] = None) -> C.CDLL:
    """Load librtx.so (raises RtxError if it was not built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RtxError(f"librtx.so not found at {p}: build it first (python -c "
                       "'import __graft_entry__ as g; g.build()' or make)")
    lib = C.CDLL(p)
    f, u32, i32, vp = C.POINTER(C.c_float), C.c_uint32, C.c_int32, C.c_void_p
    ctx = C.c_void_p
    sig = {
        "rtx_version": (C.c_int, []),
        "rtx_build_info": (C.c_char_p, []),
        "rtx_last_error": (C.c_char_p, []),
        "rtx_device_count": (C.c_int, [C.POINTER(C.c_int)]),
        "rtx_create": (C.c_int, [C.c_int, C.POINTER(ctx)]),
        "rtx_destroy": (None, [ctx]),
        "rtx_set_stream": (C.c_int, [ctx, vp]),
        "rtx_use_own_stream": (C.c_int, [ctx]),
        "rtx_upload_world": (C.c_int, [ctx, C.POINTER(rtx_world)]),
        "rtx_set_scan_mode": (C.c_int, [ctx, C.c_int]),
        "rtx_set_frame": (C.c_int, [ctx, C.POINTER(rtx_frame)]),
        "rtx_render_rows": (C.c_int, [ctx, u32, u32, u32, vp]),
        "rtx_render": (C.c_int, [ctx]),
        "rtx_accumulate": (C.c_int, [ctx, C.c_int]),
        "rtx_accumulated_frames": (u32, [ctx]),
        "rtx_camera_set_aperture": (C.c_int, [C.POINTER(rtx_frame), C.c_float]),
        "rtx_part_rows": (u32, [u32, u32, u32, u32]),
        "rtx_deinterleave_rows": (C.c_int, [ctx, vp, u32, u32, u32, u32, vp]),
        "rtx_sync": (C.c_int, [ctx]),
        "rtx_framebuffer": (vp, [ctx]),
        "rtx_download": (C.c_int, [ctx, f, C.c_size_t]),
        "rtx_alloc": (C.c_int, [ctx, C.c_size_t, C.POINTER(C.c_void_p)]),
        "rtx_free": (C.c_int, [ctx, vp]),
        "rtx_copy_to_host": (C.c_int, [ctx, vp, vp, C.c_size_t]),
        "rtx_copy_to_device": (C.c_int, [ctx, vp, vp, C.c_size_t]),
        "rtx_stats_reset": (C.c_int, [ctx]),
        "rtx_get_stats": (C.c_int, [ctx, C.POINTER(rtx_stats)]),
        "rtx_scene_random_world": (C.c_int, [i32, u32, f, f, f, C.POINTER(u32)]),
        "rtx_scene_test_world": (C.c_int, [f, f, f, C.POINTER(u32)]),
        "rtx_scene_ps_world": (C.c_int, [f, f, f, C.POINTER(u32)]),
        "rtx_camera_look_at": (C.c_int, [f, f, f, C.c_float, C.c_float, C.c_float, C.c_float,
                                         u32, u32, C.POINTER(rtx_frame)]),
        "rtx_camera_simple": (C.c_int, [u32, u32, C.POINTER(rtx_frame)]),
        "rtx_world_from_worlddef": (C.c_int, [vp, C.c_size_t, f, f, f, C.POINTER(rtx_world)]),
        "rtx_frame_from_perframe": (C.c_int, [vp, C.c_size_t, u32, u32, C.POINTER(rtx_frame)]),
        "rtx_schedule_defaults": (C.c_int, [C.POINTER(rtx_schedule)]),
        "rtx_set_schedule": (C.c_int, [ctx, C.POINTER(rtx_schedule)]),
        "rtx_get_schedule": (C.c_int, [ctx, C.POINTER(rtx_schedule)]),
        "rtx_debug_hit_world": (C.c_int, [ctx, f, u32, C.c_float, C.c_float, f]),
        "rtx_debug_hit_world_from": (C.c_int, [ctx, f, u32, C.c_float, C.c_float, u32, f]),
        "rtx_debug_math": (C.c_int, [ctx, C.c_int, f, f, u32, f]),
        "rtx_debug_wave_times": (C.c_int, [ctx, C.c_size_t, C.POINTER(C.c_uint64)]),
        "rtx_debug_pixel_cost": (C.c_int, [ctx, u32, C.POINTER(C.c_uint32)]),
        "rtx_debug_scan_rate": (C.c_int, [ctx, u32, C.POINTER(C.c_float), C.POINTER(C.c_uint64)]),
    }
    # entry points added after 1.0 may be absent from older builds (A/B runs
    # of earlier libraries); calling one then fails with AttributeError
    optional = {"rtx_schedule_defaults", "rtx_set_schedule", "rtx_get_schedule", "rtx_debug_hit_world_from",
                "rtx_build_info", "rtx_debug_scan_rate", "rtx_set_scan_mode"}
    for name, (res, args) in sig.items():
        if name in optional and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _check(rc: int, what: str, lib: Optional[C.CDLL] = None):
    if rc != RTX_OK:
        msg = (lib or load_library()).rtx_last_error().decode(errors="replace")
        raise RtxError(f"{what} failed ({rc}): {msg}")


# ---------------------------------------------------------------------------
# Scene / camera producers (host-side, no GPU)
# ---------------------------------------------------------------------------
@dataclass
class World:
    """Scene ~ WorldDef (DxCSApp.cpp:64-71): spheres [n,4] (center, radius),
    mat_types [n] (0 Lambert, 1 metal, 2 dielectric), mat_values [n,4]."""
    spheres: np.ndarray
    mat_types: np.ndarray
    mat_values: np.ndarray
    depth: int = 50
    spp: int = 60

    @property
    def count(self) -> int:
        return int(self.spheres.shape[0])

    def as_struct(self):
        self.spheres = np.ascontiguousarray(self.spheres, dtype=np.float32)
        self.mat_types = np.ascontiguousarray(self.mat_types, dtype=np.float32)
        self.mat_values = np.ascontiguousarray(self.mat_values, dtype=np.float32)
        w = rtx_world()
        w.count, w.depth, w.spp, w.reserved = self.count, self.depth, self.spp, 0
        w.spheres, w.mat_types, w.mat_values = (_fptr(self.spheres), _fptr(self.mat_types),
                                                _fptr(self.mat_values))
        return w


def random_world(grid_half_extent: int = 9, capacity: Optional[int] = None, depth: int = 50,
                 spp: int = 60) -> World:
    """WorldDef::random_world (DxCSApp.cpp:72-134). 9 -> 326 spheres (the
    reference scene), 11 -> 486 (RTIOW final scene), 159 -> 101,124."""
    cap = capacity if capacity is not None else 4 + (2 * grid_half_extent) ** 2
    sph = np.zeros((cap, 4), np.float32)
    mt = np.zeros(cap, np.float32)
    mv = np.zeros((cap, 4), np.float32)
    n = C.c_uint32()
    _check(load_library().rtx_scene_random_world(grid_half_extent, cap, _fptr(sph), _fptr(mt),
                                                 _fptr(mv), C.byref(n)), "rtx_scene_random_world")
    k = n.value
    return World(sph[:k].copy(), mt[:k].copy(), mv[:k].copy(), depth, spp)


def test_world(depth: int = 50, spp: int = 50) -> World:
    """WorldDef::test_world (DxCSApp.cpp:136-157)."""
    sph = np.zeros((4, 4), np.float32)
    mt = np.zeros(4, np.float32)
    mv = np.zeros((4, 4), np.float32)
    n = C.c_uint32()
    _check(load_library().rtx_scene_test_world(_fptr(sph), _fptr(mt), _fptr(mv), C.byref(n)),
           "rtx_scene_test_world")
    return World(sph, mt, mv, depth, spp)


def ps_world(depth: int = 25, spp: int = 1) -> World:
    """The pixel-shader prototype's 7-sphere scene (Shader_RT.fx:300-335);
    its defaults depth 25, 1 sample (Shader_RT.fx:392, 430)."""
    sph = np.zeros((7, 4), np.float32)
    mt = np.zeros(7, np.float32)
    mv = np.zeros((7, 4), np.float32)
    n = C.c_uint32()
    _check(load_library().rtx_scene_ps_world(_fptr(sph), _fptr(mt), _fptr(mv), C.byref(n)),
           "rtx_scene_ps_world")
    return World(sph, mt, mv, depth, spp)


def camera_look_at(width: int, height: int, look_from=(13.0, 2.0, 3.0), look_at=(0.0, 0.0, 0.0),
                   vup=(0.0, 1.0, 0.0), vfov: float = 20.0, aspect: float = 16.0 / 9.0,
                   aperture: float = 2.0, focus_dist: float = 0.0) -> rtx_frame:
    """PerFrame::ComputeViewVals with DxCSApp's defaults (DxCSApp.cpp:176-179)."""
    f = rtx_frame()
    a = [np.asarray(v, np.float32) for v in (look_from, look_at, vup)]
    _check(load_library().rtx_camera_look_at(_fptr(a[0]), _fptr(a[1]), _fptr(a[2]), vfov,
                                             np.float32(aspect), aperture, focus_dist, width,
                                             height, C.byref(f)), "rtx_camera_look_at")
    return f


def set_aperture(frame: rtx_frame, aperture: float) -> rtx_frame:
    """Thin-lens defocus: lens radius = aperture / 2."""
    _check(load_library().rtx_camera_set_aperture(C.byref(frame), aperture), "rtx_camera_set_aperture")
    return frame


def camera_simple(width: int, height: int) -> rtx_frame:
    """Camera(width, height) of the CPU library (Camera.h:9-21)."""
    f = rtx_frame()
    _check(load_library().rtx_camera_simple(width, height, C.byref(f)), "rtx_camera_simple")
    return f


def part_rows(height: int, tile_rows: int, part: int, nparts: int) -> int:
    return int(load_library().rtx_part_rows(height, tile_rows, part, nparts))


def part_row_ids(height: int, tile_rows: int, part: int, nparts: int) -> np.ndarray:
    """Global rows owned by `part` (interleaved tiles), ascending."""
    y = np.arange(height, dtype=np.int64)
    return y[(y // tile_rows) % nparts == part].astype(np.uint32)


def _require_schedule_abi(lib: C.CDLL):
    """rtx_schedule grew in 1.2.0 (promote_big_scene, refill_chunk), 1.3.0
    (trace_solo_bar, trace_group) and 1.4.0 (prio_bar1..3): a library of
    another major.minor (older or newer) would read this module's struct at
    the wrong offsets, so it must match exactly (patch levels may differ)."""
    v = int(lib.rtx_version())
    if v // 10 != SCHEDULE_ABI // 10 or not hasattr(lib, "rtx_set_schedule"):
        raise RtxError(f"library ABI {v} does not match the rtx_schedule layout {SCHEDULE_ABI} this binding "
                       "passes (major.minor must be equal)")


def schedule_defaults() -> rtx_schedule:
    """The library's default schedule (no GPU)."""
    lib = load_library()
    _require_schedule_abi(lib)
    sch = rtx_schedule()
    _check(lib.rtx_schedule_defaults(C.byref(sch)), "rtx_schedule_defaults")
    return sch


def build_info(lib: Optional[C.CDLL] = None) -> dict:
    """rtx_build_info of the loaded library: {"src_sha16": ..., "arch": ...}
    (empty for libraries older than ABI 1.3)."""
    lib = lib or load_library()
    if not hasattr(lib, "rtx_build_info"):
        return {}
    return dict(kv.split("=", 1) for kv in lib.rtx_build_info().decode().split())


def device_count() -> int:
    n = C.c_int(0)
    rc = load_library().rtx_device_count(C.byref(n))
    return n.value if rc == RTX_OK else 0


# ---------------------------------------------------------------------------
# GPU context
# ---------------------------------------------------------------------------
class Context:
    """One HIP device's renderer (~ CDx11Base::Initialize .. Terminate)."""

    def __init__(self, device: int = 0, stream: Optional[int] = None,
                 lib: Optional[C.CDLL] = None):
        self._lib = lib or load_library()
        h = C.c_void_p()
        _check(self._lib.rtx_create(device, C.byref(h)), "rtx_create", self._lib)
        self._h = h
        self.device = device
        self.frame: Optional[rtx_frame] = None
        self.world: Optional[World] = None
        if stream is not None:
            self.set_stream(stream)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.rtx_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream: Optional[int]):
        """Launch on `stream` (a hipStream_t handle; 0 = HIP's null stream,
        i.e. torch's default stream); None = the context's own stream."""
        if stream is None:
            _check(self._lib.rtx_use_own_stream(self._h), "rtx_use_own_stream", self._lib)
        else:
            _check(self._lib.rtx_set_stream(self._h, C.c_void_p(stream)), "rtx_set_stream", self._lib)

    def set_scan_mode(self, mode: str):
        """"auto" (layer grid / culled scan) or "linear" (every block of every
        segment, Hittable_list order): rtx_set_scan_mode, applied by the next
        upload_world."""
        _check(self._lib.rtx_set_scan_mode(self._h, SCAN_MODES[mode]), "rtx_set_scan_mode", self._lib)

    def upload_world(self, world: World):
        w = world.as_struct()
        _check(self._lib.rtx_upload_world(self._h, C.byref(w)), "rtx_upload_world", self._lib)
        self.world = world

    def set_frame(self, frame: rtx_frame):
        _check(self._lib.rtx_set_frame(self._h, C.byref(frame)), "rtx_set_frame", self._lib)
        self.frame = frame

    def render_rows(self, tile_rows: int, part: int, nparts: int, d_out: Optional[int] = None):
        _check(self._lib.rtx_render_rows(self._h, tile_rows, part, nparts,
                                         C.c_void_p(d_out or 0)), "rtx_render_rows", self._lib)

    def render(self):
        _check(self._lib.rtx_render(self._h), "rtx_render", self._lib)

    def accumulate(self, reset: bool = False) -> int:
        """Progressive accumulation; returns frames accumulated."""
        _check(self._lib.rtx_accumulate(self._h, 1 if reset else 0), "rtx_accumulate", self._lib)
        return int(self._lib.rtx_accumulated_frames(self._h))

    def deinterleave(self, d_gathered: int, width: int, height: int, tile_rows: int, nparts: int,
                     d_image: int):
        _check(self._lib.rtx_deinterleave_rows(self._h, C.c_void_p(d_gathered), width, height,
                                               tile_rows, nparts, C.c_void_p(d_image)),
               "rtx_deinterleave_rows", self._lib)

    def sync(self):
        _check(self._lib.rtx_sync(self._h), "rtx_sync", self._lib)

    def framebuffer_ptr(self) -> int:
        return int(self._lib.rtx_framebuffer(self._h) or 0)

    def download(self) -> np.ndarray:
        f = self.frame
        out = np.empty((f.height, f.width, 4), np.float32)
        _check(self._lib.rtx_download(self._h, _fptr(out), out.nbytes), "rtx_download", self._lib)
        return out

    def render_image(self) -> np.ndarray:
        self.render()
        return self.download()

    def alloc(self, shape, dtype=np.float32) -> "DeviceArray":
        return DeviceArray(self, shape, dtype)

    def stats_reset(self):
        _check(self._lib.rtx_stats_reset(self._h), "rtx_stats_reset", self._lib)

    def stats(self) -> rtx_stats:
        s = rtx_stats()
        _check(self._lib.rtx_get_stats(self._h, C.byref(s)), "rtx_get_stats", self._lib)
        return s

    def set_schedule(self, schedule: Optional[rtx_schedule] = None, **fields):
        """Install a schedule (rtx_set_schedule): `schedule`, or the current
        one with `fields` replaced; no arguments = the defaults."""
        _require_schedule_abi(self._lib)
        if schedule is None and not fields:
            _check(self._lib.rtx_set_schedule(self._h, None), "rtx_set_schedule", self._lib)
            return
        sch = schedule if schedule is not None else self.get_schedule()
        for k, v in fields.items():
            if k not in dict(rtx_schedule._fields_):
                raise RtxError(f"unknown schedule field {k}")
            setattr(sch, k, v)
        _check(self._lib.rtx_set_schedule(self._h, C.byref(sch)), "rtx_set_schedule", self._lib)

    def get_schedule(self) -> rtx_schedule:
        _require_schedule_abi(self._lib)
        sch = rtx_schedule()
        _check(self._lib.rtx_get_schedule(self._h, C.byref(sch)), "rtx_get_schedule", self._lib)
        return sch

    def debug_hit_world(self, rays: np.ndarray, t_min: float = 0.001,
                        t_max: float = float("inf"), start_block: Optional[int] = None) -> np.ndarray:
        """hit_world on the GPU (rtx_debug_hit_world); start_block: the scan
        starts at that 8-sphere block and wraps round (rtx_debug_hit_world_from);
        DEBUG_CULLED: the culled scan (worlds of more than 1,024 spheres)."""
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
        out = np.zeros((rays.shape[0], 10), np.float32)
        if start_block is None:
            _check(self._lib.rtx_debug_hit_world(self._h, _fptr(rays), rays.shape[0], t_min, t_max,
                                                 _fptr(out)), "rtx_debug_hit_world", self._lib)
        else:
            _check(self._lib.rtx_debug_hit_world_from(self._h, _fptr(rays), rays.shape[0], t_min, t_max,
                                                      start_block, _fptr(out)), "rtx_debug_hit_world_from",
                   self._lib)
        return out

    def arm_wave_times(self, max_waves: int):
        _check(self._lib.rtx_debug_wave_times(self._h, max_waves, None), "rtx_debug_wave_times", self._lib)

    def wave_times(self, max_waves: int) -> np.ndarray:
        out = np.zeros((max_waves, 2), np.uint64)
        _check(self._lib.rtx_debug_wave_times(self._h, max_waves, out.ctypes.data_as(C.POINTER(C.c_uint64))),
               "rtx_debug_wave_times", self._lib)
        return out

    def debug_scan_rate(self, reps: int) -> tuple:
        """hit_world alone at the render's occupancy (rtx_debug_scan_rate):
        (launch ms, wave-segments)."""
        ms, ws = C.c_float(0.0), C.c_uint64(0)
        _check(self._lib.rtx_debug_scan_rate(self._h, reps, C.byref(ms), C.byref(ws)), "rtx_debug_scan_rate", self._lib)
        return float(ms.value), int(ws.value)

    def debug_pixel_cost(self, spp: int = 0) -> np.ndarray:
        """Per-pixel ray-segment counts of the current frame, (H, W) uint32."""
        f = self.frame
        out = np.zeros((f.height, f.width), np.uint32)
        _check(self._lib.rtx_debug_pixel_cost(self._h, spp, out.ctypes.data_as(C.POINTER(C.c_uint32))),
               "rtx_debug_pixel_cost", self._lib)
        return out

    def debug_math(self, fn: str, in0: np.ndarray, in1: Optional[np.ndarray] = None) -> np.ndarray:
        a = np.ascontiguousarray(in0, np.float32)
        b = None if in1 is None else np.ascontiguousarray(in1, np.float32)
        out = np.zeros(3 * a.size, np.float32)
        _check(self._lib.rtx_debug_math(self._h, FN[fn], _fptr(a),
                                        _fptr(b) if b is not None else None, a.size, _fptr(out)),
               "rtx_debug_math", self._lib)
        return out.reshape(a.size, 3) if FN[fn] >= FN["hash1"] else out[:a.size]

    def debug_lambert_dir(self, p: np.ndarray, nrm: np.ndarray, rius: np.ndarray, guard: bool) -> np.ndarray:
        """The kernel's diffuse direction, normalize(((p + normal) + rius) - p),
        optionally near-zero guarded (RTX_FN_LAMBERT_DIR[_GUARD]); (n, 3) arrays."""
        a = np.ascontiguousarray(p, np.float32).reshape(-1, 3)
        b = np.ascontiguousarray(np.concatenate([np.reshape(nrm, (-1, 3)), np.reshape(rius, (-1, 3))], 1),
                                 np.float32)
        out = np.zeros_like(a)
        fn = FN["lambert_dir_guard" if guard else "lambert_dir"]
        _check(self._lib.rtx_debug_math(self._h, fn, _fptr(a), _fptr(b), a.shape[0], _fptr(out)),
               "rtx_debug_math", self._lib)
        return out


class DeviceArray:
    """Device buffer owned by a Context (rtx_alloc/rtx_free), no torch needed."""

    def __init__(self, ctx: Context, shape, dtype=np.float32):
        self.ctx, self.shape, self.dtype = ctx, tuple(shape), np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        p = C.c_void_p()
        _check(ctx._lib.rtx_alloc(ctx._h, self.nbytes, C.byref(p)), "rtx_alloc", ctx._lib)
        self.ptr = int(p.value)

    def numpy(self) -> np.ndarray:
        out = np.empty(self.shape, self.dtype)
        _check(self.ctx._lib.rtx_copy_to_host(self.ctx._h, out.ctypes.data, C.c_void_p(self.ptr),
                                              self.nbytes), "rtx_copy_to_host", self.ctx._lib)
        return out

    def upload(self, a: np.ndarray):
        a = np.ascontiguousarray(a, self.dtype)
        assert a.nbytes == self.nbytes
        _check(self.ctx._lib.rtx_copy_to_device(self.ctx._h, C.c_void_p(self.ptr), a.ctypes.data,
                                                self.nbytes), "rtx_copy_to_device", self.ctx._lib)

    def free(self):
        if self.ptr and self.ctx._h:
            _check(self.ctx._lib.rtx_free(self.ctx._h, C.c_void_p(self.ptr)), "rtx_free", self.ctx._lib)
        self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
