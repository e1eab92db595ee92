"""C-ABI surface and host logic (CPU only, no GPU compute calls)."""
import ctypes as C
import os
import re
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    """Every RTX_API function declared in include/*.h."""
    names = set()
    for h in os.listdir(os.path.join(ROOT, "include")):
        if not h.endswith(".h"):
            continue
        text = open(os.path.join(ROOT, "include", h)).read()
        for m in re.finditer(r"RTX_API\s+[^;(]*?\b(rtx_\w+)\s*\(", text):
            names.add(m.group(1))
    return sorted(names)


def test_header_declares_boundary():
    names = declared_symbols()
    for must in ("rtx_create", "rtx_destroy", "rtx_upload_world", "rtx_set_frame", "rtx_render_rows",
                 "rtx_sync", "rtx_download", "rtx_last_error", "rtx_deinterleave_rows"):
        assert must in names
    assert len(names) >= 25


def test_library_exports_every_declared_symbol(rtx):
    lib = rtx.load_library()
    missing = [n for n in declared_symbols() if not hasattr(lib, n)]
    assert not missing, f"librtx.so lacks {missing}"
    out = subprocess.run(["nm", "-D", "--defined-only", rtx.LIB_PATH], capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert set(declared_symbols()) <= exported
    # nothing but the C-ABI leaks out (no C++ mangled product symbols)
    assert not [s for s in exported if s.startswith("_ZN3rtx")]


def test_library_built_for_gfx950(rtx):
    """The embedded HIP fat binary carries a gfx950 (MI355X) code object."""
    blob = open(rtx.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_version_and_error_paths(rtx):
    lib = rtx.load_library()
    assert lib.rtx_version() == 145
    # null arguments are rejected without touching the GPU
    assert lib.rtx_upload_world(None, None) == -1
    assert b"null" in lib.rtx_last_error()
    assert lib.rtx_set_frame(None, None) == -1
    assert lib.rtx_render_rows(None, 1, 0, 1, None) == -1
    assert lib.rtx_sync(None) == -1
    assert lib.rtx_get_stats(None, None) == -1
    f = rtx.rtx_frame()
    assert lib.rtx_camera_look_at(None, None, None, 20.0, 1.0, 0.0, 0.0, 4, 4, C.byref(f)) == -1


@pytest.mark.parametrize("H,T,R", [(1080, 5, 8), (1080, 5, 1), (117, 8, 3), (117, 64, 5),
                                   (10, 3, 8), (1, 1, 2), (2160, 8, 8), (1081, 5, 8)])
def test_part_rows_matches_definition(rtx, H, T, R):
    total = 0
    for p in range(R):
        ids = rtx.part_row_ids(H, T, p, R)
        assert rtx.part_rows(H, T, p, R) == len(ids)
        total += len(ids)
    assert total == H
    # part 0 is the largest part (used to size equal gather buffers)
    assert rtx.part_rows(H, T, 0, R) == max(rtx.part_rows(H, T, p, R) for p in range(R))
    assert rtx.part_rows(H, T, R, R) == 0 and rtx.part_rows(H, 0, 0, R) == 0


def deinterleave_np(gathered, H, T, R):
    """Numpy statement of rtx_deinterleave_rows (rtx_kernels.hip k_deinterleave)."""
    W = gathered.shape[2]
    img = np.empty((H, W) + gathered.shape[3:], gathered.dtype)
    for y in range(H):
        tile = y // T
        img[y] = gathered[tile % R, (tile // R) * T + (y - tile * T)]
    return img


@pytest.mark.parametrize("H,T,R", [(1080, 5, 8), (117, 8, 3), (31, 4, 5)])
def test_deinterleave_inverts_partition(rtx, H, T, R):
    W = 3
    img = np.random.default_rng(H).normal(size=(H, W)).astype(np.float32)
    maxr = rtx.part_rows(H, T, 0, R)
    g = np.zeros((R, maxr, W), np.float32)
    for p in range(R):
        ids = rtx.part_row_ids(H, T, p, R)
        g[p, :len(ids)] = img[ids]
    np.testing.assert_array_equal(deinterleave_np(g, H, T, R), img)


def test_schedule_defaults_and_validation(rtx):
    """rtx_schedule (the chain render's schedule): the library's
    defaults are the measured constants, and rtx_set_schedule validates every
    field before a context exists (a null ctx is refused first)."""
    d = rtx.schedule_defaults()
    assert d.tier1_bar == pytest.approx(1.7) and d.tier1_bar_small == pytest.approx(1.6)
    assert d.tier1_bar_low == pytest.approx(1.8) and d.tier2_bar_small == pytest.approx(2.0)
    assert d.tier2_bar_medium == pytest.approx(1e30) and d.small_share == pytest.approx(1.2)
    assert d.low_share == pytest.approx(2.5) and d.medium_share == pytest.approx(3.5)
    assert d.hot_fraction == pytest.approx(0.2) and d.tail_coop_max == 32 and d.tail_coop_max_large == 8
    assert d.refill_chunk == 64
    assert d.tier2_bar == pytest.approx(1e30)
    assert (d.tier1_priority, d.tier2_priority, d.hot_priority) == (3, 2, 3)
    assert (d.trace_small, d.trace_low, d.trace_medium, d.trace_large) == pytest.approx((0.35, 0.3, 0.15, 0.0))
    assert (d.promote_small, d.promote_low, d.promote_medium, d.promote_large) == (400.0, 500.0, 400.0, 400.0)
    assert d.promote_big_scene == 60.0
    assert (d.trace_group, d.trace_solo_bar, d.prepass_cap_split) == (4, pytest.approx(6.0), 0)
    assert (d.prio_bar1, d.prio_bar2, d.prio_bar3) == pytest.approx((0.5, 1.0, 1.5))
    assert d.occupancy_small == d.occupancy_low == d.occupancy_normal == 1.0
    lib = rtx.load_library()
    assert lib.rtx_set_schedule(None, C.byref(d)) == -1
    assert lib.rtx_get_schedule(None, C.byref(d)) == -1
    assert lib.rtx_schedule_defaults(None) == -1


def test_library_reads_no_environment(rtx):
    """The product library takes no tuning from the environment (the
    schedule is an explicit C-ABI call): no getenv/secure_getenv import."""
    out = subprocess.run(["nm", "-D", "--undefined-only", rtx.LIB_PATH], capture_output=True, text=True).stdout
    assert "getenv" not in out, [l for l in out.splitlines() if "getenv" in l]


def test_ctypes_mirror_matches_header_layout(rtx, tmp_path):
    """The Python mirror's structs (rtx/__init__.py) have the sizes and field
    offsets that include/rtx.h gives them under the C compiler, so a field
    added to the header (ABI 1.2.0: promote_big_scene, refill_chunk) cannot
    silently shift the mirror."""
    import rtx as R
    structs = {"rtx_world": R.rtx_world, "rtx_frame": R.rtx_frame, "rtx_schedule": R.rtx_schedule,
               "rtx_stats": R.rtx_stats}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "rtx.h"', 'int main(void) {']
    for name, cls in structs.items():
        lines.append(f'  printf("{name} size %zu\\n", sizeof({name}));')
        for field, _ in cls._fields_:
            lines.append(f'  printf("{name} {field} %zu\\n", offsetof({name}, {field}));')
    lines += ['  return 0;', '}']
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = {}
    for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        *key, val = line.split()
        got[tuple(key)] = int(val)
    for name, cls in structs.items():
        assert got[(name, "size")] == C.sizeof(cls), name
        for field, _ in cls._fields_:
            assert got[(name, field)] == getattr(cls, field).offset, (name, field)


def test_schedule_calls_refuse_another_abi(rtx):
    """rtx_schedule grew in ABI 1.2.0, 1.3.0 and 1.4.0: the binding refuses to
    pass its layout to a library of another major.minor, older or newer (it
    would read the fields at the wrong offsets), instead of installing a
    wrong schedule; a different patch level is accepted."""
    class Lib:
        def __init__(self, v):
            self.v = v

        def rtx_version(self):
            return self.v

        def rtx_set_schedule(self, *a):
            raise AssertionError("must not be called")

    for v in (130, 150, 200):
        with pytest.raises(rtx.RtxError, match="does not match"):
            rtx._require_schedule_abi(Lib(v))
    rtx._require_schedule_abi(Lib(rtx.SCHEDULE_ABI + 1))  # a patch level
    rtx._require_schedule_abi(rtx.load_library())  # the in-tree library passes


def test_library_built_from_this_tree(rtx):
    """Build provenance: the library's embedded source hash (rtx_build_info,
    Makefile SRC_SHA) equals the hash of the tree's sources, i.e. the loaded
    librtx.so was compiled from exactly these files."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from src_sha import src_sha16
    info = rtx.build_info()
    assert info.get("arch") == "gfx950"
    assert info.get("src_sha16") == src_sha16(), "librtx.so is stale: rebuild (make)"
    assert info.get("variant") == "product", info
