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


def check_hits_against_fp64(spheres, rays, got, expected):
    """Assert fp32 hit records `got` match fp64 `expected` within the bound.
    Returns the largest observed error / bound ratio."""
    got = np.asarray(got, np.float64)
    e = np.asarray(expected, np.float64)
    assert got.shape == e.shape
    np.testing.assert_array_equal(got[:, 0], e[:, 0], err_msg="hit/miss differs")
    np.testing.assert_array_equal(got[:, 9], e[:, 9], err_msg="winning sphere index differs")
    m = e[:, 0] == 1
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
    return worst
