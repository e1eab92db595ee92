#!/usr/bin/env python3
"""Per-section clock split of the render kernel (diagnostic).

Needs a variant built with -DRTX_DIAG_PROF=1 (Makefile: prof, prof_merge):
each wave sums core-clock deltas per section of its loop and adds them into
the wave_times buffer. Clocks of interleaved waves overlap, so the split is
a share of wave residency, not of the GPU.

    python tools/section_prof.py raytrace-we-gpu_amd/lib/variants/librtx_prof.so
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytrace-we-gpu_amd"))
import rtx  # noqa: E402

libs = sys.argv[1:] or [os.path.join(ROOT, "raytrace-we-gpu_amd/lib/variants/librtx_prof.so")]
# C2 by default; RTX_SPROF_GRID / _CAP / _SPP select another scene (C5: 159, 100000, 16)
world = rtx.random_world(int(os.environ.get("RTX_SPROF_GRID", "11")),
                         capacity=int(os.environ.get("RTX_SPROF_CAP", "0")) or None, depth=50,
                         spp=int(os.environ.get("RTX_SPROF_SPP", "100")))
frame = rtx.camera_look_at(1920, 1080, aspect=1920 / 1080)
for path in libs:
    c = rtx.Context(0, lib=rtx.load_library(path))
    c.upload_world(world)
    c.set_frame(frame)
    c.render()
    c.sync()
    c.arm_wave_times(8)
    c.stats_reset()
    c.render()
    c.sync()
    st = c.stats()
    v = c.wave_times(8).reshape(-1).astype(np.float64)
    names = ["refill", "hit_world", "shade", "tail", "iters", "tail_iters", "active_lanes"]
    clocks = v[:4].sum()
    rep = {"lib": os.path.basename(path), "kernel_ms": st.kernel_ms / max(st.launches, 1),
           "segments": st.segments}
    for k in range(4):
        rep[names[k] + "_share"] = round(v[k] / clocks, 4)
    rep["iters"] = int(v[4])
    rep["tail_iters"] = int(v[5])
    rep["lane_util"] = round(v[6] / (64 * v[4]), 4)
    rep["clocks_per_iter_hit_world"] = round(v[1] / max(v[4] - v[5], 1), 1)
    rep["clocks_per_iter_shade"] = round(v[2] / max(v[4] - v[5], 1), 1)
    rep["clocks_per_tail_iter"] = round(v[3] / max(v[5], 1), 1)
    seg_iters = max(v[4] - v[5], 1)
    rep["batches_per_iter"] = round(v[8] / seg_iters, 2)
    rep["recorded_frac"] = round(v[9] / max(v[8], 1), 4)
    rep["resolve_iters_per_iter"] = round(v[10] / seg_iters, 3)
    rep["fallback_lanes"] = int(v[11])
    rep["lanes_with_candidates_per_iter"] = round(v[12] / seg_iters, 2)
    # candidate spheres per wave-iteration: the resolve's rounds are their max over the lanes
    # (resolve_iters_per_iter); / 64 their mean per lane — the rounds a wave-wide compaction would take
    rep["candidates_per_iter"] = round(v[13] / seg_iters, 2)
    rep["compacted_rounds_per_iter"] = round(v[13] / seg_iters / 64.0, 3)
    # culled scan: blocks whose bound some lane's line passed (they are scanned; the others skipped)
    rep["cull_pass_blocks_per_iter"] = round(v[14] / seg_iters, 2)
    print(json.dumps(rep), flush=True)
