#!/usr/bin/env python3
"""Offline pass rates of block-bound culling on sampled rays (analysis only).

Input: an .npz from tools/ray_sample.py (real lane-mode wave iterations of a
render). For each record (one wave iteration, 64 lanes) it computes, per
block of spheres, whether ANY live lane's ray line passes within the
block's bounding sphere — the fraction of blocks a wave-level block test
(ballot) would still have to scan — for the stored sphere order and for a
Morton (x, z) order of the small spheres, block sizes 8 / 16, the infinite
line (what the scan's prefilter tests) and the half-line (t >= -R). The
per-sphere "recorded" fraction (some lane's line within a sphere) is the
calibration against section_prof's recorded_frac.

    python tools/block_cull_sim.py rays.npz [max_records]
"""
import json
import sys

import numpy as np

z = np.load(sys.argv[1])
maxr = int(sys.argv[2]) if len(sys.argv) > 2 else 400
o, d, live = z["o"].astype(np.float64), z["d"].astype(np.float64), z["live"]
S = z["spheres"].astype(np.float64)
C, R = S[:, :3], S[:, 3]
n = len(S)
rng = np.random.default_rng(0)
recs = np.arange(len(o)) if len(o) <= maxr else np.sort(rng.choice(len(o), maxr, replace=False))


def morton_order():
    small = np.nonzero(R < 100)[0]
    big = np.nonzero(R >= 100)[0]
    lo = C[small][:, [0, 2]].min(0)
    q = np.floor((C[small][:, [0, 2]] - lo) / np.maximum(np.ptp(C[small][:, [0, 2]], 0) / 1023, 1e-9)).astype(np.int64)
    key = np.zeros(len(small), np.int64)
    for b in range(10):
        key |= ((q[:, 0] >> b) & 1) << (2 * b) | ((q[:, 1] >> b) & 1) << (2 * b + 1)
    return np.concatenate([big, small[np.argsort(key, kind="stable")]])


def bounds(order, bs):
    cs, rs = [], []
    for b in range(0, n, bs):
        ii = order[b:b + bs]
        if (R[ii] >= 100).any():
            c = C[ii][R[ii].argmax()]
        else:
            c = 0.5 * (C[ii].min(0) + C[ii].max(0))
        cs.append(c)
        rs.append((np.linalg.norm(C[ii] - c, axis=1) + R[ii]).max())
    return np.array(cs), np.array(rs)


def pass_mask(oo, dd, cb, rb, half):
    dn = dd / np.linalg.norm(dd, axis=1)[:, None]
    res = np.zeros((len(oo), len(cb)), bool)
    for k in range(0, len(cb), 4096):
        oc = cb[None, k:k + 4096] - oo[:, None]
        pr = (oc * dn[:, None]).sum(2)
        dp2 = (oc * oc).sum(2) - pr ** 2
        m = dp2 <= rb[None, k:k + 4096] ** 2
        if half:
            m &= pr >= -rb[None, k:k + 4096]
        res[:, k:k + 4096] = m
    return res


orders = {"stored": np.arange(n), "morton": morton_order()}
out = {"records": int(len(recs)), "spheres": n}
acc = {}
for r in recs:
    lv = live[r]
    oo, dd = o[r][lv], d[r][lv]
    if len(oo) == 0:
        continue
    for nm, od in orders.items():
        for half in (False, True):
            sph = pass_mask(oo, dd, C[od], R[od], half)
            nb = (n + 7) // 8
            padded = np.zeros((len(oo), nb * 8), bool)
            padded[:, :n] = sph
            acc.setdefault(f"{nm}/{'half' if half else 'line'}/recorded8", []).append(
                padded.reshape(len(oo), nb, 8).any(2).any(0).mean())
            for bs in (8, 16, 64):
                cb, rb = bounds(od, bs)
                pm = pass_mask(oo, dd, cb, rb, half)
                acc.setdefault(f"{nm}/{'half' if half else 'line'}/bound{bs}_wave", []).append(pm.any(0).mean())
                acc.setdefault(f"{nm}/{'half' if half else 'line'}/bound{bs}_lane", []).append(pm.mean())
for k in sorted(acc):
    out[k] = round(float(np.mean(acc[k])), 4)
print(json.dumps(out))
