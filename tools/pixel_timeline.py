#!/usr/bin/env python3
"""Per-pixel timeline of one rank's share of the C2 frame (diagnostic; needs
the RTX_DIAG_PIXEL build, lib/variants/librtx_ptime.so). For every pixel of
rtx_render_rows(T, part, R): its start time and queue (0 lane mode, 1 tier-1
heavy, 2 tier-2 heavy, 3 promoted), its end time, and its segment count
(rtx_debug_pixel_cost). Shows what ends the part: which pixels finish last,
how they were traced and their time per segment.

    python tools/pixel_timeline.py LIB [--parts 2 8] [--which 0]
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
ap.add_argument("--parts", type=int, nargs="*", default=[1, 2, 8])
ap.add_argument("--which", type=int, default=0, help="part index to trace (mod R)")
ap.add_argument("--tile-rows", type=int, default=5)
ap.add_argument("--set", default="", help="schedule fields (tools/heavy_sweep.py syntax), e.g. a1=1.5,coop=32")
ap.add_argument("--grid", type=int, default=11, help="random_world grid (159 with --cap 100000: C5)")
ap.add_argument("--cap", type=int, default=0)
ap.add_argument("--spp", type=int, default=100)
a = ap.parse_args()

W, H, T = 1920, 1080, a.tile_rows
world = rtx.random_world(a.grid, capacity=a.cap or None, depth=50, spp=a.spp)
frame = rtx.camera_look_at(W, H, aspect=W / H)
ctx = rtx.Context(0, lib=rtx.load_library(a.lib))
if a.set:
    from heavy_sweep_fields import schedule_of
    ctx.set_schedule(**schedule_of(a.set))
ctx.upload_world(world)
ctx.set_frame(frame)
cost = ctx.debug_pixel_cost().astype(np.int64)  # (H, W) segments per pixel
buf = ctx.alloc((H, W, 4))
for R in a.parts:
    p = a.which % R
    rows = rtx.part_row_ids(H, T, p, R)
    npix = len(rows) * W
    seg = cost[rows].ravel()
    ctx.arm_wave_times(npix)
    ctx.render_rows(T, p, R, buf.ptr)
    ctx.sync()
    ctx.stats_reset()
    ctx.render_rows(T, p, R, buf.ptr)
    ctx.sync()
    st = ctx.stats()
    t = ctx.wave_times(npix).astype(np.int64)
    start, mode, end = t[:, 0] >> 2, t[:, 0] & 3, t[:, 1]
    ok = start > 0
    t0 = start[ok].min()
    s_us, e_us = (start - t0) / 100.0, (end - t0) / 100.0
    dur = e_us - s_us
    ups = np.where(seg > 0, dur / np.maximum(seg, 1), 0.0)
    span = float(e_us[ok].max())

    def rec(i):
        return {"start_us": round(float(s_us[i]), 1), "end_us": round(float(e_us[i]), 1), "mode": int(mode[i]),
                "segments": int(seg[i]), "us_per_segment": round(float(ups[i]), 3)}

    last = np.argsort(-e_us)[:12]
    heavy = np.argsort(-seg)[:12]
    modes = {}
    for m in (0, 1, 2, 3):  # 3: promoted (start = the promotion)
        sel = ok & (mode == m)
        if sel.any():
            modes[str(m)] = {"pixels": int(sel.sum()), "segments_mean": round(float(seg[sel].mean()), 1),
                             "us_per_segment_p50": round(float(np.median(ups[sel])), 3),
                             "us_per_segment_max": round(float(ups[sel].max()), 3),
                             "start_us_max": round(float(s_us[sel].max()), 1),
                             "end_us_max": round(float(e_us[sel].max()), 1)}
    # over time (1 ms bins): pixels in flight per mode and their segment rate
    # (segments per us, each pixel at its own mean rate): how the share's
    # throughput falls off towards its end
    prof = []
    rate = np.where(ok & (dur > 0), seg / np.maximum(dur, 1e-3), 0.0)
    for tc in np.arange(0.5e3, span, 1e3):
        on = ok & (s_us <= tc) & (e_us > tc)
        prof.append({"t_ms": round(float(tc) / 1e3, 1),
                     "active": {str(m): int((on & (mode == m)).sum()) for m in (0, 1, 2, 3)},
                     "seg_per_us": {str(m): round(float(rate[on & (mode == m)].sum()), 1) for m in (0, 1, 2, 3)}})
    late = ok & (e_us > 0.9 * span)
    out = {"set": a.set or "default", "parts": R, "part": p, "pixels": npix, "kernel_ms": round(st.kernel_ms / max(1, st.launches), 3),
           "span_us": round(span, 1), "segments_total": int(seg.sum()), "segments_max": int(seg.max()),
           "modes": modes, "profile": prof, "last_finishing": [rec(i) for i in last], "heaviest": [rec(i) for i in heavy],
           "late10pct": {"pixels": int(late.sum()), "segments_mean": round(float(seg[late].mean()), 1) if late.any() else 0,
                         "start_us_mean": round(float(s_us[late].mean()), 1) if late.any() else 0}}
    print(json.dumps(out), flush=True)
buf.free()
ctx.close()
