#!/usr/bin/env python3
"""Per-pixel cost study for the scheduling of the C2 frame (diagnostic).

Measures every pixel's ray-segment count at full spp and at the 1-spp
pre-pass (rtx_debug_pixel_cost), then reports the cost distribution, how
well the smoothed pre-pass key ranks pixels, and the makespan of a
lane-level list schedule (R lanes pull pixels in queue order; a pixel takes
its segment count) for several orders, relative to the perfect-balance
bound sum/R. The frame cannot end before its most expensive pixel does.

    python tools/cost_analysis.py [--lanes 393216] [--out gpurun_out/cost.npz]
"""
import argparse
import heapq
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytrace-we-gpu_amd"))
import rtx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=100)
ap.add_argument("--grid", type=int, default=11)
ap.add_argument("--lanes", type=int, default=6144 * 64)
ap.add_argument("--out", default="")
ap.add_argument("--from-npz", default="", help="analyse a saved cost.npz (no GPU)")
ap.add_argument("--dump-only", action="store_true", help="save the npz and stop")
a = ap.parse_args()

if a.from_npz:
    d = np.load(a.from_npz)
    full, one = d["full"].astype(np.int64), d["one"].astype(np.int64)
else:
    world = rtx.random_world(a.grid, depth=50, spp=a.spp)
    frame = rtx.camera_look_at(a.width, a.height, aspect=a.width / a.height)
    c = rtx.Context(0)
    c.upload_world(world)
    c.set_frame(frame)
    full = c.debug_pixel_cost(0).astype(np.int64)
    one = c.debug_pixel_cost(1).astype(np.int64)
    two = c.debug_pixel_cost(2).astype(np.int64)  # the scheduled path's 2-spp pre-pass
if a.out:
    np.savez_compressed(a.out, full=full.astype(np.uint32), one=one.astype(np.uint32),
                        **({} if a.from_npz else {"two": two.astype(np.uint32)}))
if a.dump_only:
    sys.exit(0)


def smooth(x, r):
    p = np.pad(x, r, mode="edge")
    h, w = x.shape
    return sum(p[r + dy:r + dy + h, r + dx:r + dx + w] for dy in range(-r, r + 1) for dx in range(-r, r + 1))


def makespan(costs_in_order, lanes):
    n = costs_in_order.size
    if n <= lanes:
        return int(costs_in_order.max())
    heap = [(int(t), i) for i, t in enumerate(costs_in_order[:lanes])]
    heapq.heapify(heap)
    for t in costs_in_order[lanes:]:
        s, i = heapq.heappop(heap)
        heapq.heappush(heap, (s + int(t), i))
    return max(h[0] for h in heap)


flat = full.ravel()
total = int(flat.sum())
R = a.lanes
bound = float(max(total / R, flat.max()))
rep = {"pixels": int(flat.size), "segments": total, "mean": float(flat.mean()),
       "p50": float(np.percentile(flat, 50)), "p99": float(np.percentile(flat, 99)),
       "p999": float(np.percentile(flat, 99.9)), "max": int(flat.max()),
       "sum_over_lanes": total / R, "lower_bound": bound}
orders = {"linear": np.arange(flat.size), "true_lpt": np.argsort(-flat, kind="stable")}
for r in (0, 1, 2):
    key = smooth(one, r).ravel()
    orders[f"key_r{r}"] = np.argsort(-np.minimum(key, 255), kind="stable")
    rep[f"spearman_r{r}"] = float(np.corrcoef(np.argsort(np.argsort(key)), np.argsort(np.argsort(flat)))[0, 1])
for name, o in orders.items():
    m = makespan(flat[o], R)
    rep[f"makespan_{name}"] = int(m)
    rep[f"makespan_{name}_over_bound"] = round(m / bound, 4)
print(json.dumps(rep))
