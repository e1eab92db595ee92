"""Stated fp32 tolerance for ray-sphere hits against the fp64 reference.

The reference's CPU geometry is double precision (Sphere.cpp); the GPU path
(like the reference's own HLSL shader) evaluates the same quadratic in fp32.
The root t = (-hb - sqrt(hb^2 - a*c)) / a loses precision where c = |oc|^2 -
r^2 cancels (the r = 1000 ground sphere) and where disc is small (grazing
rays). The tolerance is the first-order fp32 error bound of that formula
with an 8-ulp safety factor:

    |dt| <= 8 * 2^-23 * ( (|oc|^2 * a + hb^2) / (a * sqrt(disc)) + |t| )
    |dp| <= |dt| * |d| + 8 * 2^-23 * (|o| + |t d|)
    |dn| <= |dp| / r + 8 * 2^-23

with hit/miss, front_face and the winning sphere index required to be
identical. On the committed golden vectors the observed error is at most
~12 % of this bound.

Ill-conditioned rays are the exception: where a sphere's fp64 discriminant
is within the fp32 rounding of zero (|disc| <= 8 eps (hb^2 + a |oc|^2):
a line grazing the silhouette), or two candidate roots of different spheres
(or a root and t_min) agree to 1e-5, fp32 and fp64 can legitimately decide
hit/miss or the winner differently. `ill_conditioned` marks those rays; the
check skips the identity requirement for them (and reports how many there
were), while the GPU must still equal the fp32 twin bit for bit.
"""
import numpy as np

EPS = 2.0 ** -23
K = 8.0


def hit_bounds(spheres, rays, expected):
    """Per-ray bounds (dt, dp, dn) for hit rays of `expected` (fp64 rows)."""
    e = np.asarray(expected, np.float64)
    sph = np.asarray(spheres, np.float64)
    rays = np.asarray(rays, np.float64)
    idx = np.where(e[:, 0] == 1, e[:, 9], 0).astype(int)
    r = sph[idx, 3]
    o, d = rays[:, :3], rays[:, 3:]
    oc = o - sph[idx, :3]
    a = (d * d).sum(1)
    hb = (oc * d).sum(1)
    cc = (oc * oc).sum(1) - r * r
    disc = np.maximum(hb * hb - a * cc, 1e-300)
    t = np.abs(e[:, 1])
    dt = K * EPS * (((oc * oc).sum(1) * a + hb * hb) / (a * np.sqrt(disc)) + t)
    dn_len = np.linalg.norm(d, axis=1)
    dp = dt * dn_len + K * EPS * (np.linalg.norm(o, axis=1) + t * dn_len)
    dn = dp / np.abs(r) + K * EPS
    return dt, dp, dn


def ill_conditioned(spheres, rays, t_min=0.001, t_max=np.inf, chunk=8):
    """Boolean mask of rays whose fp32 decision may differ from fp64 (see the
    module docstring)."""
    sph = np.asarray(spheres, np.float64)
    rays = np.asarray(rays, np.float64)
    out = np.zeros(len(rays), bool)
    c, r = sph[:, :3], sph[:, 3]
    for k in range(0, len(rays), chunk):
        o, d = rays[k:k + chunk, None, :3], rays[k:k + chunk, None, 3:]
        oc = o - c[None]
        a = (d * d).sum(-1)
        hb = (oc * d).sum(-1)
        oc2 = (oc * oc).sum(-1)
        disc = hb * hb - a * (oc2 - r * r)
        scale = 8 * EPS * (hb * hb + a * oc2)
        graze = np.abs(disc) <= scale
        sq = np.sqrt(np.maximum(disc, 0.0))
        rn, rf = (-hb - sq) / a, (-hb + sq) / a
        cand = np.where(rn >= t_min, rn, np.where(rf >= t_min, rf, np.inf))
        cand = np.where((disc >= 0) & (cand <= t_max), cand, np.inf)
        near_tmin = (disc >= 0) & ((np.abs(rn - t_min) <= 1e-5 * np.maximum(t_min, np.abs(rn))) |
                                   (np.abs(rf - t_min) <= 1e-5 * np.maximum(t_min, np.abs(rf))))
        two = np.sort(cand, axis=1)[:, :2] if cand.shape[1] > 1 else np.concatenate([cand, np.full_like(cand, np.inf)], 1)
        with np.errstate(invalid="ignore"):  # inf - inf where no sphere is hit
            tie = np.isfinite(two[:, 1]) & (two[:, 1] - two[:, 0] <= 1e-5 * np.abs(two[:, 1]))
        out[k:k + chunk] = graze.any(1) | near_tmin.any(1) | tie
    return out


def check_hits_against_fp64(spheres, rays, got, expected, t_min=0.001, t_max=np.inf, allow_ill=False):
    """Assert fp32 hit records `got` match fp64 `expected` within the bound.
    allow_ill: rays flagged by ill_conditioned() need not agree on
    hit/miss/winner. Returns (largest observed error / bound ratio, number of
    exempt rays that disagree) if allow_ill, else the ratio."""
    got = np.asarray(got, np.float64)
    e = np.asarray(expected, np.float64)
    assert got.shape == e.shape
    ill = ill_conditioned(spheres, rays, t_min, t_max) if allow_ill else np.zeros(len(e), bool)
    differ = (got[:, 0] != e[:, 0]) | (got[:, 9] != e[:, 9])
    well = ~ill
    np.testing.assert_array_equal(got[well, 0], e[well, 0], err_msg="hit/miss differs on a well-conditioned ray")
    np.testing.assert_array_equal(got[well, 9], e[well, 9], err_msg="winning sphere index differs")
    e = e.copy()
    e[differ] = got[differ]  # exempt disagreements (ill-conditioned only) take no part below
    m = (e[:, 0] == 1) & ~differ
    np.testing.assert_array_equal(got[m, 8], e[m, 8], err_msg="front_face differs")
    dt, dp, dn = hit_bounds(spheres, rays, e)
    et = np.abs(got[m, 1] - e[m, 1])
    ep = np.abs(got[m, 2:5] - e[m, 2:5]).max(1)
    en = np.abs(got[m, 5:8] - e[m, 5:8]).max(1)
    worst = 0.0
    for name, err, bnd in (("t", et, dt[m]), ("p", ep, dp[m]), ("normal", en, dn[m])):
        ratio = err / bnd
        bad = np.nonzero(ratio > 1.0)[0]
        assert bad.size == 0, f"{name} outside fp32 tolerance at rays {bad[:10]}: ratio {ratio[bad[:10]]}"
        worst = max(worst, float(ratio.max(initial=0.0)))
    return (worst, int(differ.sum())) if allow_ill else worst
