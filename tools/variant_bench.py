#!/usr/bin/env python3
"""A/B timing of kernel variants (raytrace-we-gpu_amd/lib/variants/*.so) in
ONE process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24).
Every variant's frame must be bit-identical to the first one's.

    python tools/variant_bench.py [--rounds 3] [--frames 2] [--spp 100] [variant ...]
"""
import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytrace-we-gpu_amd"))
import numpy as np  # noqa: E402
import rtx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--frames", type=int, default=2)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=100)
ap.add_argument("--grid", type=int, default=11)
ap.add_argument("--max-spheres", type=int, default=0)
ap.add_argument("--rng", choices=["chain", "per-sample"], default="chain")
ap.add_argument("names", nargs="*")
a = ap.parse_args()

vdir = os.path.join(ROOT, "raytrace-we-gpu_amd", "lib", "variants")
paths = sorted(glob.glob(os.path.join(vdir, "librtx_*.so")))
if a.names:
    paths = [os.path.join(vdir, f"librtx_{n}.so") for n in a.names]
world = rtx.random_world(a.grid, capacity=a.max_spheres or None, depth=50, spp=a.spp)
frame = rtx.camera_look_at(a.width, a.height, aspect=a.width / a.height)
frame.rng_mode = 1 if a.rng == "per-sample" else 0
ctxs = {}
for p in paths:
    name = os.path.basename(p)[len("librtx_"):-3]
    lib = rtx.load_library(p)
    c = rtx.Context(0, lib=lib)
    c.upload_world(world)
    c.set_frame(frame)
    ctxs[name] = c
ref = None
times = {n: [] for n in ctxs}
for r in range(a.rounds):
    for n, c in ctxs.items():
        c.render()
        c.sync()  # warm
        c.stats_reset()
        t0 = time.perf_counter()
        for _ in range(a.frames):
            c.render()
        c.sync()
        wall = (time.perf_counter() - t0) / a.frames
        st = c.stats()
        times[n].append(st.kernel_ms / st.launches)
        if r == 0:
            img = c.download()
            if ref is None:
                ref = img
            same = (img.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(img) & np.isnan(ref))
            if not same.all() and "diag" not in n and "nostore" not in n:
                print(json.dumps({"variant": n, "ERROR": f"{(~same).sum()} values differ from first variant"}))
        print(json.dumps({"variant": n, "round": r, "kernel_ms": round(times[n][-1], 3),
                          "wall_ms": round(wall * 1e3, 3),
                          "msamples_s": round(a.width * a.height * a.spp / (times[n][-1] * 1e-3) / 1e6, 1),
                          "tests_per_s": st.sphere_tests / st.launches / (times[n][-1] * 1e-3),
                          "segments_per_frame": st.segments // max(1, st.launches)}), flush=True)
summary = {n: {"median_ms": round(float(np.median(t)), 3), "min_ms": round(float(min(t)), 3)} for n, t in times.items()}
print(json.dumps({"summary": summary}))
