#!/usr/bin/env python3
"""Offline check of the scheduling pre-pass's cost key (rtx_kernels.hip
cost_key) against the chains it predicts, from tools/cost_maps.py's maps.
For the R-way share of part 0 (row tiles of 5), each candidate key orders the
share's pixels; greedy list scheduling of that order onto `lanes` identical
lanes (every lane takes the next pixel when it frees up, as k_render's
persistent lanes do) gives a makespan in segments; the lower bound is
max(total / lanes, heaviest pixel). Keys: the 3x3 window of the k-spp costs
(the product's, k = 2), the pixel's own k-spp cost, and their max.

    python tools/key_quality.py COST_MAPS.npz [--lanes 213000]
"""
import argparse
import heapq
import json

import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("maps")
ap.add_argument("--parts", type=int, nargs="*", default=[1, 2, 4, 8])
ap.add_argument("--lanes", type=int, nargs="*", default=[327680, 278528, 229376, 212992])
a = ap.parse_args()
M = np.load(a.maps)
H, W, T = 1080, 1920, 5


def rows_of(R, p=0):
    return [y for y in range(H) if (y // T) % R == p]


def win3(c):
    p = np.pad(c, 1, mode="edge")
    return sum(p[1 + dy:1 + dy + c.shape[0], 1 + dx:1 + dx + c.shape[1]] for dy in (-1, 0, 1) for dx in (-1, 0, 1))


def makespan(order_cost, lanes):
    if len(order_cost) <= lanes:
        return float(order_cost.max())
    h = [0.0] * lanes
    for c in order_cost:
        t = heapq.heappop(h)
        heapq.heappush(h, t + float(c))
    return max(h)


for R, lanes in zip(a.parts, a.lanes):
    rows = rows_of(R)
    true = M["spp100"][rows].astype(np.float64)
    out = {"parts": R, "pixels": true.size, "lanes": lanes,
           "bound": round(max(true.sum() / lanes, true.max()), 1)}
    for k in (1, 2, 4, 8):
        c = M[f"spp{k}"][rows].astype(np.float64)
        keys = {f"win{k}": win3(c) / 9.0, f"own{k}": c}
        keys[f"max{k}"] = np.maximum(keys[f"win{k}"], keys[f"own{k}"])
        for name, key in keys.items():
            order = np.argsort(-key.ravel(), kind="stable")
            ms = makespan(true.ravel()[order], lanes)
            rho = np.corrcoef(np.argsort(np.argsort(key.ravel())), np.argsort(np.argsort(true.ravel())))[0, 1]
            out[name] = {"makespan": round(ms, 1), "spearman": round(float(rho), 3)}
    out["oracle"] = round(makespan(np.sort(true.ravel())[::-1], lanes), 1)
    print(json.dumps(out), flush=True)
