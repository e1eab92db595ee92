#!/usr/bin/env python3
"""Strong-scaling rehearsal on ONE device: the per-rank work of an R-GPU
frame is rtx_render_rows(tile_rows, part, R) (interleaved row tiles), so
timing every part of an R-way split on one MI355X gives each rank's kernel
time and the critical path max_p(t_p) the R-GPU frame is bounded by
(before the gather). Efficiency = t(1) / (R * max_p t_p).

    python tools/part_scaling.py [--parts 1 2 4 8] [--frames 2] [lib.so ...]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytrace-we-gpu_amd"))
import rtx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--parts", type=int, nargs="*", default=[1, 2, 4, 8])
ap.add_argument("--frames", type=int, default=2)
ap.add_argument("--tile-rows", type=int, default=5)
ap.add_argument("--spp", type=int, default=100)
ap.add_argument("--rng", choices=["chain", "per-sample"], default="chain")
ap.add_argument("--grid", type=int, default=11, help="random_world grid half extent (159 + --max-spheres 100000: C5)")
ap.add_argument("--max-spheres", type=int, default=0)
ap.add_argument("libs", nargs="*")
a = ap.parse_args()

W, H = 1920, 1080
world = rtx.random_world(a.grid, capacity=a.max_spheres or None, depth=50, spp=a.spp)
frame = rtx.camera_look_at(W, H, aspect=W / H)
frame.rng_mode = 1 if a.rng == "per-sample" else 0
for path in a.libs or [None]:
    lib = rtx.load_library(path) if path else None
    ctx = rtx.Context(0, lib=lib)
    ctx.upload_world(world)
    ctx.set_frame(frame)
    buf = ctx.alloc((H, W, 4))
    t1 = None
    for R in a.parts:
        times, segs = [], []
        for p in range(R):
            ctx.render_rows(a.tile_rows, p, R, buf.ptr)  # warm
            ctx.sync()
            ctx.stats_reset()
            for _ in range(a.frames):
                ctx.render_rows(a.tile_rows, p, R, buf.ptr)
            st = ctx.stats()
            times.append(st.kernel_ms / st.launches)
            segs.append(st.segments // st.launches)
        crit = max(times)
        if R == 1:
            t1 = crit
        rep = {"lib": os.path.basename(path) if path else "default", "rng": a.rng, "parts": R,
               "part_ms": [round(t, 3) for t in times], "critical_ms": round(crit, 3),
               "mean_ms": round(sum(times) / R, 3), "part_segments": segs}
        if t1:
            rep["efficiency"] = round(t1 / (R * crit), 4)
        print(json.dumps(rep), flush=True)
    buf.free()
    ctx.close()
