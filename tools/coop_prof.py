#!/usr/bin/env python3
"""Clock split of tier-1 group-coop segments (one ray per wave, 64 lanes;
diagnostic, needs the RTX_DIAG_COOP build lib/variants/librtx_cprof.so):
shader clocks per segment in ray exchange + line setup, scan + resolve,
reduction, shade, and the loop between segments. Rendered on one rank's
share of the C2 frame, where tier 1 is populated.

    python tools/coop_prof.py LIB [--parts 8] [--part 0]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytrace-we-gpu_amd"))
import numpy as np  # noqa: E402
import rtx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("lib")
ap.add_argument("--parts", type=int, nargs="*", default=[8, 2])
ap.add_argument("--part", type=int, default=0)
a = ap.parse_args()

W, H, T = 1920, 1080, 5
world = rtx.random_world(11, depth=50, spp=100)
frame = rtx.camera_look_at(W, H, aspect=W / H)
ctx = rtx.Context(0, lib=rtx.load_library(a.lib))
ctx.upload_world(world)
ctx.set_frame(frame)
buf = ctx.alloc((H, W, 4))
names = ["setup", "scan_resolve", "reduce", "shade", "loop"]
for R in a.parts:
    p = a.part % R
    ctx.render_rows(T, p, R, buf.ptr)
    ctx.sync()
    ctx.arm_wave_times(8)
    ctx.stats_reset()
    ctx.render_rows(T, p, R, buf.ptr)
    ctx.sync()
    st = ctx.stats()
    v = ctx.wave_times(8).reshape(-1).astype(np.float64)
    segs = max(v[5], 1.0)
    rep = {"lib": os.path.basename(a.lib), "parts": R, "part": p,
           "kernel_ms": round(st.kernel_ms / max(1, st.launches), 3), "segments": int(v[5])}
    for k, n in enumerate(names):
        rep[n + "_clk"] = round(v[k] / segs, 1)
    rep["total_clk"] = round(v[:5].sum() / segs, 1)
    print(json.dumps(rep), flush=True)
buf.free()
ctx.close()
