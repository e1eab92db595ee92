#!/usr/bin/env python3
"""Per-wave start/end timeline of one frame or one part of a row split
(diagnostic): how many waves are resident over time, and how long the tail
is. Uses rtx_debug_wave_times.
    python tools/wave_timeline.py [--rng chain|per-sample] [--parts R] [--part p] [lib.so]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytrace-we-gpu_amd"))
import numpy as np  # noqa: E402
import rtx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rng", choices=["chain", "per-sample"], default="chain")
ap.add_argument("--parts", type=int, default=1)
ap.add_argument("--part", type=int, default=0)
ap.add_argument("--grid", type=int, default=11)
ap.add_argument("--cap", type=int, default=0)
ap.add_argument("--spp", type=int, default=100)
ap.add_argument("lib", nargs="?")
a = ap.parse_args()
lib = rtx.load_library(a.lib) if a.lib else None
W_, H_, T_ = 1920, 1080, 5
world = rtx.random_world(a.grid, capacity=a.cap or None, depth=50, spp=a.spp)
frame = rtx.camera_look_at(W_, H_)
frame.rng_mode = 1 if a.rng == "per-sample" else 0
ctx = rtx.Context(0, lib=lib)
ctx.upload_world(world)
ctx.set_frame(frame)
buf = ctx.alloc((H_, W_, 4))
W = (W_ * H_ + 63) // 64  # upper bound on waves (any block size)
ctx.render_rows(T_, a.part, a.parts, buf.ptr)  # warm
ctx.sync()
ctx.arm_wave_times(2 * W)  # k_render_ps also writes (clocks, segments) per wave in the upper half
ctx.render_rows(T_, a.part, a.parts, buf.ptr)
ctx.sync()
tt = ctx.wave_times(2 * W).astype(np.int64)
t, extra = tt[:W], tt[W:]
live = t[:, 0] > 0
t, extra = t[live], extra[live]
t0 = t[:, 0].min()
s, e = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0  # microseconds
dur = e - s
T = e.max()
grid = np.linspace(0, T, 200)
resident = np.array([((s <= g) & (e > g)).sum() for g in grid])
out = {"lib": a.lib or "default", "rng": a.rng, "parts": a.parts, "part": a.part, "waves": int(len(t)),
       "kernel_us": float(T), "wave_us_mean": float(dur.mean()),
       "wave_us_p50": float(np.median(dur)), "wave_us_p99": float(np.percentile(dur, 99)),
       "wave_us_max": float(dur.max()), "end_us_p1": float(np.percentile(e, 1)),
       "end_us_p50": float(np.median(e)), "mean_resident": float(resident.mean()),
       "peak_resident": int(resident.max()),
       "resident_frac_of_peak_over_time": [round(float(x), 3) for x in resident[::10] / resident.max()],
       "last_start_us": float(s.max()), "busy_integral_frac": float(dur.sum() / (resident.max() * T))}
if a.rng == "per-sample" and extra[:, 0].any():
    clk = extra[:, 0] / np.maximum(dur, 1e-3)  # shader clocks per microsecond = MHz
    segs = extra[:, 1]
    out.update({"clock_mhz_p50": float(np.median(clk)), "clock_mhz_min": float(clk.min()),
                "wave_segments_mean": float(segs.mean()), "wave_segments_max": int(segs.max()),
                "us_per_wave_iteration": float(np.median(dur / np.maximum(segs / 64.0, 1)))})
print(json.dumps(out))
buf.free()
