#!/usr/bin/env python3
"""Offline estimate (analysis only, CPU): how many 8-entry records a wave
tests per ray segment at C5 with the culled scan's wave-uniform walk (the
union of what its 64 lanes' lines pass: scan_culled) against a per-lane
walk (the wave's loop runs as long as its busiest lane), with and without a
far cut at each lane's hit. Paths are traced in numpy on the C5 scene
(random_world(159), 100,000 spheres) with approximate materials; the tree is
a Morton (x, z) order of the flat layer with plain bounding spheres (no
stretch, no rounding margins), so only the ratios mean anything.

    python tools/traversal_sim.py [pixels]

Round 6 (256 pixels, 685 segments): union 836 records per wave-segment,
per-lane max 246 (far cut 209), per-lane mean 86 (59). The per-lane walk
built on this (vector loads of each lane's own record) measured 180 ms
against 129 ms for the union scan (profiles/S6i_ab_c5_lane_walk.jsonl):
the wave-uniform walk's records come through the scalar cache, the
per-lane walk's through the vector memory path, 64 addresses a load.
"""
import sys, json
import numpy as np
sys.path.insert(0, "/root/repo/raytrace-we-gpu_amd")
import rtx

rng = np.random.default_rng(1)
w = rtx.random_world(159, capacity=100000)
S = w.spheres.astype(np.float64)
MT = w.mat_types.astype(np.int64)
MV = w.mat_values.astype(np.float64)
n = len(S)
C, R = S[:, :3], S[:, 3]
print("spheres", n)

# ---- paths: camera rays + bounces (geometry statistics only) ----
W_, H_ = 1920, 1080
lf, la, vup = np.array([13., 2., 3.]), np.zeros(3), np.array([0., 1., 0.])
th = np.radians(20.0); hh = np.tan(th / 2); ww = W_ / H_ * hh
wv = (lf - la) / np.linalg.norm(lf - la); uv = np.cross(vup, wv); uv /= np.linalg.norm(uv); vv = np.cross(wv, uv)
llc = lf - ww * uv - hh * vv - wv


def hit_all(o, d, tmin=1e-3):
    # o, d: (k,3) -> t (k,), idx (k,)
    oc = o[:, None, :] - C[None]
    a = (d * d).sum(1)[:, None]
    hb = (oc * d[:, None, :]).sum(2)
    cc = (oc * oc).sum(2) - R[None] ** 2
    disc = hb * hb - a * cc
    sq = np.sqrt(np.maximum(disc, 0))
    rn = (-hb - sq) / a
    rf = (-hb + sq) / a
    t = np.where(rn >= tmin, rn, rf)
    t = np.where((disc >= 0) & (t >= tmin), t, np.inf)
    i = t.argmin(1)
    return t[np.arange(len(o)), i], i


def rand_unit(k):
    v = rng.normal(size=(k, 3))
    return v / np.linalg.norm(v, axis=1)[:, None]


def sample_segments(npix):
    px = rng.uniform(0, W_, npix); py = rng.uniform(0, H_, npix)
    o = np.repeat(lf[None], npix, 0)
    d = llc[None] + (px / W_)[:, None] * 2 * ww * uv[None] + (py / H_)[:, None] * 2 * hh * vv[None] - lf[None]
    segs = [[] for _ in range(npix)]
    alive = np.arange(npix)
    for depth in range(50):
        if len(alive) == 0:
            break
        oo, dd = o[alive], d[alive]
        t, i = [], []
        for k in range(0, len(alive), 32):
            tt, ii = hit_all(oo[k:k + 32], dd[k:k + 32])
            t.append(tt); i.append(ii)
        t = np.concatenate(t); i = np.concatenate(i)
        for j, p in enumerate(alive):
            segs[p].append((oo[j].copy(), dd[j].copy(), t[j]))
        hit = np.isfinite(t)
        alive, oo, dd, t, i = alive[hit], oo[hit], dd[hit], t[hit], i[hit]
        p = oo + t[:, None] * dd
        nrm = (p - C[i]) / R[i][:, None]
        dn = dd / np.linalg.norm(dd, axis=1)[:, None]
        nd = np.empty_like(dd)
        m0, m1, m2 = MT[i] == 0, MT[i] == 1, MT[i] == 2
        nd[m0] = nrm[m0] + rand_unit(m0.sum())
        refl = dn - 2 * (dn * nrm).sum(1)[:, None] * nrm
        nd[m1] = refl[m1] + MV[i][m1, 3:4] * rand_unit(m1.sum()) * rng.uniform(0, 1, (m1.sum(), 1)) ** (1 / 3)
        if m2.any():
            ir = MV[i][m2, 3]
            front = (dn[m2] * nrm[m2]).sum(1) < 0
            nn = np.where(front[:, None], nrm[m2], -nrm[m2])
            eta = np.where(front, 1 / ir, ir)
            cos = np.minimum((-dn[m2] * nn).sum(1), 1)
            sin = np.sqrt(1 - cos * cos)
            tir = eta * sin > 1
            r0 = ((1 - eta) / (1 + eta)) ** 2
            sch = r0 + (1 - r0) * (1 - cos) ** 5
            rf = tir | (sch > rng.uniform(0, 1, len(cos)))
            rperp = eta[:, None] * (dn[m2] + cos[:, None] * nn)
            rpar = -np.sqrt(np.abs(1 - (rperp * rperp).sum(1)))[:, None] * nn
            rr = dn[m2] - 2 * (dn[m2] * nn).sum(1)[:, None] * nn
            nd[m2] = np.where(rf[:, None], rr, rperp + rpar)
        keep = ~(m1 & ((nd * nrm).sum(1) <= 0))
        o = np.zeros((npix, 3)); d = np.zeros((npix, 3))
        o[alive] = p; d[alive] = nd
        alive = alive[keep]
    return segs


# ---- layout: non-flat first, flat in Morton (x, z) order; blocks 8, groups 64, super 512, hyper 4096 ----
flat = np.nonzero(np.abs(C[:, 1] - 0.2) < 1e-6)[0]
big = np.setdiff1d(np.arange(n), flat)
q = np.floor(C[flat][:, [0, 2]] - C[flat][:, [0, 2]].min(0)).astype(np.int64)
key = np.zeros(len(flat), np.int64)
for b in range(10):
    key |= ((q[:, 0] >> b) & 1) << (2 * b) | ((q[:, 1] >> b) & 1) << (2 * b + 1)
order = np.concatenate([big, -np.ones(4096 - len(big), np.int64), flat[np.argsort(key, kind="stable")]])


def level_bounds(child_c, child_r, valid):
    m = len(child_c)
    k = (m + 7) // 8
    cs = np.zeros((k, 3)); rs = np.full(k, -1.0)
    for j in range(k):
        sl = slice(8 * j, min(8 * j + 8, m))
        v = valid[sl]
        if not v.any():
            continue
        cc, rr = child_c[sl][v], child_r[sl][v]
        c = 0.5 * (cc - rr[:, None]).min(0) + 0.5 * (cc + rr[:, None]).max(0)
        cs[j] = c; rs[j] = (np.linalg.norm(cc - c, axis=1) + rr).max()
    return cs, rs, rs >= 0


pad = (-len(order)) % 4096
order = np.concatenate([order, -np.ones(pad, np.int64)])
valid0 = order >= 0
c0 = np.where(valid0[:, None], C[np.maximum(order, 0)], 0); r0 = np.where(valid0, R[np.maximum(order, 0)], -1)
L = [(c0, r0, valid0)]
for lev in range(4):
    L.append(level_bounds(*L[-1]))
print("levels", [len(x[0]) for x in L])  # spheres, blocks, groups, supers, hypers


def passes(o, d, cs, rs, valid, tcut=np.inf):
    dn = d / np.linalg.norm(d)
    oc = cs - o
    pr = oc @ dn
    tc = np.maximum(pr, 0)
    dist2 = ((o + tc[:, None] * dn - cs) ** 2).sum(1)
    ok = valid & (dist2 <= rs * rs)
    # entry along the ray (distance units) <= tcut
    ent = pr - np.sqrt(np.maximum(rs * rs - np.maximum((oc * oc).sum(1) - pr * pr, 0), 0))
    return ok & (ent <= tcut)


def lane_counts(o, d, tcut):
    # passes per level (children of passed parents only): returns sets per level
    sets = []
    cur = np.nonzero(passes(o, d, *L[4], tcut))[0]  # hyper bounds passed (top records always tested)
    sets.append(cur)
    for lev in (3, 2, 1):
        ch = (cur[:, None] * 8 + np.arange(8)[None]).ravel()
        ch = ch[ch < len(L[lev][0])]
        cs, rs, v = L[lev]
        pm = passes(o, d, cs[ch], rs[ch], v[ch], tcut)
        cur = ch[pm]
        sets.append(cur)
    return sets  # hyper, super, group, block passed


nhg_records = (len(L[4][0]) + 7) // 8
segs = sample_segments(int(sys.argv[1]) if len(sys.argv) > 1 else 1024)
allseg = [s for p in segs for s in p]
print("segments", len(allseg), "per pixel", len(allseg) / len(segs))
res = {"union": [], "lane_max": [], "lane_far_max": [], "lane_mean": [], "lane_far_mean": []}
idx = rng.permutation(len(allseg))
nw = len(idx) // 64
for wv_ in range(nw):
    lanes = [allseg[k] for k in idx[64 * wv_:64 * wv_ + 64]]
    U = [set(), set(), set(), set()]
    per, perf = [], []
    for (o, d, t) in lanes:
        s = lane_counts(o, d, np.inf)
        for lv in range(4):
            U[lv].update(s[lv].tolist())
        per.append(sum(len(x) for x in s[:3]) + len(s[3]))  # records below top + blocks
        tf = t * np.linalg.norm(d) if np.isfinite(t) else np.inf
        sf = lane_counts(o, d, tf + 1e-3)
        perf.append(sum(len(x) for x in sf))
    res["union"].append(nhg_records + sum(len(u) for u in U))
    res["lane_max"].append(nhg_records + max(per))
    res["lane_far_max"].append(nhg_records + max(perf))
    res["lane_mean"].append(nhg_records + np.mean(per))
    res["lane_far_mean"].append(nhg_records + np.mean(perf))
out = {k: float(np.mean(v)) for k, v in res.items()}
out["waves"] = nw
out["top_records"] = nhg_records
print(json.dumps(out))
