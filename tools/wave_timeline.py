#!/usr/bin/env python3
"""Per-wave start/end timeline of one C2 frame (diagnostic): how many waves
are resident over time, and how long the tail is. Uses rtx_debug_wave_times.
    python tools/wave_timeline.py [variant-lib-path]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytrace-we-gpu_amd"))
import numpy as np  # noqa: E402
import rtx  # noqa: E402

lib = rtx.load_library(sys.argv[1]) if len(sys.argv) > 1 else None
world = rtx.random_world(11, depth=50, spp=100)
frame = rtx.camera_look_at(1920, 1080)
ctx = rtx.Context(0, lib=lib)
ctx.upload_world(world)
ctx.set_frame(frame)
W = (1920 * 1080 + 63) // 64  # upper bound on waves (any block size)
ctx.arm_wave_times(W)
ctx.render()
ctx.sync()
t = ctx.wave_times(W).astype(np.int64)
t = t[(t[:, 0] > 0)]
t0 = t[:, 0].min()
s, e = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0  # microseconds
dur = e - s
T = e.max()
grid = np.linspace(0, T, 200)
resident = np.array([((s <= g) & (e > g)).sum() for g in grid])
out = {"lib": sys.argv[1] if len(sys.argv) > 1 else "default", "waves": int(len(t)), "kernel_us": float(T), "wave_us_mean": float(dur.mean()),
       "wave_us_p50": float(np.median(dur)), "wave_us_p99": float(np.percentile(dur, 99)),
       "wave_us_max": float(dur.max()), "mean_resident": float(resident.mean()),
       "peak_resident": int(resident.max()),
       "resident_frac_of_peak_over_time": [round(float(x), 3) for x in resident[::10] / resident.max()],
       "last_start_us": float(s.max()), "busy_integral_frac": float(dur.sum() / (resident.max() * T))}
print(json.dumps(out))
