#!/usr/bin/env python3
"""hit_world alone at the render's occupancy (rtx_debug_scan_rate) for
several library builds, interleaved in one process: ns per wave-segment
(64 ray segments' prefiltered scan + resolve) on the C2 scene, so scan
variants can be compared without the rest of the render.

    python tools/scan_probe.py [--reps 200] [--rounds 3] lib.so ...
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytrace-we-gpu_amd"))
import rtx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=200)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("libs", nargs="+")
a = ap.parse_args()
world = rtx.random_world(11, depth=50, spp=100)
frame = rtx.camera_look_at(1920, 1080, aspect=1920 / 1080)
ctxs = {}
for p in a.libs:
    c = rtx.Context(0, lib=rtx.load_library(p))
    c.upload_world(world)
    c.set_frame(frame)
    c.debug_scan_rate(8)  # warm
    ctxs[os.path.basename(p)] = c
best = {}
for r in range(a.rounds):
    for n, c in ctxs.items():
        ms, ws = c.debug_scan_rate(a.reps)
        ns = ms * 1e6 / ws
        best[n] = min(best.get(n, 1e30), ns)
        print(json.dumps({"lib": n, "round": r, "probe_ms": round(ms, 3), "wave_segments": ws,
                          "ns_per_wave_segment": round(ns, 3)}), flush=True)
print(json.dumps({"summary_min_ns_per_wave_segment": {k: round(v, 3) for k, v in best.items()}}))
