#!/usr/bin/env python3
"""Sweep the chain render's schedule (rtx_set_schedule, include/rtx.h
rtx_schedule) on one device: for each setting, the critical part time of an
R-way row split of C2 (as tools/part_scaling.py). A setting is a comma list
of short names (a1 tier1_bar, a1s tier1_bar_small, a1l tier1_bar_low, a2s
tier2_bar_small, a2m tier2_bar_medium, rho small_share, rhol low_share, rho2
medium_share, prio hot_fraction, occs/occl/occn occupancy_small/low/normal,
coop tail_coop_max) or full field names, applied on top of the defaults.

    python tools/heavy_sweep.py --parts 8 --set "a1s=4,a2s=2" --set "a1s=3,a2s=1" ...
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytrace-we-gpu_amd"))
import rtx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--parts", type=int, nargs="*", default=[8])
ap.add_argument("--frames", type=int, default=2)
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--set", action="append", default=[])
ap.add_argument("--sets", default="", help="settings separated by ';' ('default' = no change)")
ap.add_argument("--grid", type=int, default=11, help="random_world grid half extent (159 + --max-spheres 100000: C5)")
ap.add_argument("--max-spheres", type=int, default=0)
ap.add_argument("--spp", type=int, default=100)
ap.add_argument("--lib", default=None, help="librtx build to load (default: the product library)")
a = ap.parse_args()

from heavy_sweep_fields import schedule_of  # noqa: E402


W, H, T = 1920, 1080, 5
world = rtx.random_world(a.grid, capacity=a.max_spheres or None, depth=50, spp=a.spp)
frame = rtx.camera_look_at(W, H, aspect=W / H)
ctx = rtx.Context(0, lib=rtx.load_library(a.lib) if a.lib else None)
ctx.upload_world(world)
ctx.set_frame(frame)
buf = ctx.alloc((H, W, 4))
sets = a.set + [("" if x.strip() == "default" else x.strip()) for x in a.sets.split(";") if x.strip()]
sets = sets or [""]
for r in range(a.rounds):
    for s in sets:
        ctx.set_schedule()
        if s:
            ctx.set_schedule(**schedule_of(s))
        for R in a.parts:
            times = []
            for p in range(R):
                ctx.render_rows(T, p, R, buf.ptr)
                ctx.sync()
                ctx.stats_reset()
                for _ in range(a.frames):
                    ctx.render_rows(T, p, R, buf.ptr)
                st = ctx.stats()
                times.append(st.kernel_ms / st.launches)
            print(json.dumps({"set": s or "default", "round": r, "parts": R, "critical_ms": round(max(times), 3),
                              "mean_ms": round(sum(times) / R, 3), "part_ms": [round(t, 3) for t in times]}),
                  flush=True)
buf.free()
ctx.close()
