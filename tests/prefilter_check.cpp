// prefilter_check.cpp — CPU check of the exactness claim of the scan's
// prefilter (raytrace-we-gpu_amd/csrc/rtx_prefilter.h): over many
// adversarial ray/sphere pairs — near-tangent lines (relative distance
// 1e-9 .. 1e-1 from the silhouette), tiny and huge directions, rays near
// the x axis (the basis's degenerate direction) and near the y axis, far origins, centre magnitudes 1e-2 .. 1e4, radii 1e-3 .. 1e3 —
// whenever the reference's fp32 discriminant is >= 0 or NaN
// (ShaderCompute.hlsl:158-166; the op order of oracle/rtx_oracle.c
// hit_world32), the prefilter must flag the sphere — in both op orders the
// scan uses (line_test_q, and line_test_q_flat for flat blocks), with the
// line basis's hardware rsq/sqrt modelled as exact or one ulp off either way.
// Prints one JSON line; exit status 1 if any reference candidate is missed.
// Build: g++ -O2 -std=c++17 -ffp-contract=off -mfma prefilter_check.cpp
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "../raytrace-we-gpu_amd/csrc/rtx_prefilter.h"

static unsigned long long g_s = 0x9e3779b97f4a7c15ull;
static double uni() {
    g_s ^= g_s << 13;
    g_s ^= g_s >> 7;
    g_s ^= g_s << 17;
    return (double)(g_s >> 11) * (1.0 / 9007199254740992.0);
}
static double sym() { return 2.0 * uni() - 1.0; }
static void unit(double v[3]) {
    do {
        v[0] = sym(), v[1] = sym(), v[2] = sym();
    } while (v[0] * v[0] + v[1] * v[1] + v[2] * v[2] < 1e-6);
    const double n = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    v[0] /= n, v[1] /= n, v[2] /= n;
}

// hit_world32's discriminant (oracle/rtx_oracle.c), reference op order.
static float ref_disc(const float o[3], const float d[3], const float c[3], float negr2, float a) {
    const float ocx = o[0] - c[0], ocy = o[1] - c[1], ocz = o[2] - c[2];
    const float hb = fmaf(ocz, d[2], fmaf(ocy, d[1], ocx * d[0]));
    const float cc = fmaf(ocz, ocz, fmaf(ocy, ocy, fmaf(ocx, ocx, negr2)));
    return fmaf(hb, hb, -(a * cc));
}

// The culled scan's block bounds (rtx_prefilter.h cull_bound): a block of 8
// spheres (a cluster of extent 1e-2..1e2 x the largest radius around a centre
// of magnitude 1e-2..1e4, radii 1/8..1 x r, a third of the blocks flat: one
// centre height, bounded and tested in the space stretched along y by
// kCullSy), a near-tangent line to one of them; whenever the reference's
// disc of that sphere is >= 0 (or NaN), the block test must pass
// (line_test_q, and for flat blocks also line_test_q_flat, on the bound
// against thr * kCullThrScale, or thr' * kCullThrScaleSy for the stretched ray).
// The reference's acceptance of sphere c (hit_world32's roots, best = +inf).
static bool ref_accepts(const float o[3], const float d[3], const float c[3], float negr2, float a, float t_min) {
    const float ocx = o[0] - c[0], ocy = o[1] - c[1], ocz = o[2] - c[2];
    const float hb = fmaf(ocz, d[2], fmaf(ocy, d[1], ocx * d[0]));
    const float disc = ref_disc(o, d, c, negr2, a);
    if (disc < 0.0f) return false;
    const float inv_a = 1.0f / a, sq = std::sqrt(disc);
    const float rn = (-hb - sq) * inv_a;
    if (!(rn < t_min || INFINITY < rn)) return true;
    const float rf = (-hb + sq) * inv_a;
    return !(rf < t_min || INFINITY < rf);
}

// Half-space part (rtx_prefilter.h HalfTest): whenever the reference accepts
// the sphere (a root >= t_min, t_min 0 or 1e-3), the bound must pass both
// tests. A fifth of the rays start on (or just inside or outside) the sphere,
// half of those leaving it straight away from the bound's centre (the tight
// case of the half test: the hit is at t ~ 0, the bound behind the origin).
static void block_cases(long n, long &ref_pos, long &missed, double &max_used, long &acc_pos, long &half_missed,
                        long &half_culled, double &half_max_used) {
    for (long k = 0; k < n; ++k) {
        double cd[3], dir[3], e[3], t[3];
        unit(cd);
        const double cs = std::pow(10.0, -2.0 + 6.0 * uni());
        const double r = std::pow(10.0, -3.0 + 5.0 * uni());
        const double ext = r * std::pow(10.0, -2.0 + 4.0 * uni());
        const bool flat = uni() < 0.33;
        float sph[8][4];
        for (int i = 0; i < 8; ++i) {
            double off[3];
            unit(off);
            const double m = ext * uni();
            for (int j = 0; j < 3; ++j) sph[i][j] = (float)(cs * cd[j] + m * off[j]);
            if (flat) sph[i][1] = (float)(cs * cd[1]);
            sph[i][3] = (float)(r * (0.125 + 0.875 * uni()));
        }
        const int j0 = (int)(uni() * 8.0) & 7;
        const float *c = sph[j0];
        const double rr = c[3];
        unit(dir);
        if (uni() < 0.05) {  // near the x axis
            const double eps = std::pow(10.0, -8.0 + 6.0 * uni());
            dir[1] = eps * sym(), dir[2] = eps * sym(), dir[0] = uni() < 0.5 ? -1.0 : 1.0;
        }
        const float *sp[8];
        for (int i = 0; i < 8; ++i) sp[i] = sph[i];
        // flat blocks are bounded and tested in the space stretched along y
        const float sy = flat ? rtx::kCullSy : 1.0f;
        const rtx::CullBound b = rtx::cull_bound(sp, 8, flat, sph[0][1], sy);
        // half the lines graze the sphere on its side away from the bound's
        // centre (the tightest case for the bound), the others at random
        const double away[3] = {c[0] - (double)b.cx, c[1] - (double)b.cy / sy, c[2] - (double)b.cz};
        const double al = std::sqrt(away[0] * away[0] + away[1] * away[1] + away[2] * away[2]);
        if (uni() < 0.5 && al > 0.0) {
            for (int i = 0; i < 3; ++i) t[i] = away[i] / al;
        } else {
            unit(t);
        }
        const double td = t[0] * dir[0] + t[1] * dir[1] + t[2] * dir[2];
        const double dn = dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2];
        for (int i = 0; i < 3; ++i) e[i] = t[i] - td / dn * dir[i];
        const double en = std::sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
        if (en < 1e-9) continue;
        for (int i = 0; i < 3; ++i) e[i] /= en;
        const double delta = std::pow(10.0, -9.0 + 8.0 * uni()) * (uni() < 0.5 ? -1.0 : 1.0);
        const double dist = uni() < 0.8 ? rr * (1.0 + delta) : 3.0 * rr * uni();
        const double along = sym() * std::pow(10.0, -1.0 + 4.0 * uni()) * std::fmax(ext + rr, 1.0);
        const double dlen = std::pow(10.0, -3.0 + 6.0 * uni());
        float o[3], d[3];
        for (int i = 0; i < 3; ++i) {
            o[i] = (float)(c[i] + dist * e[i] - along * dir[i]);
            d[i] = (float)(dlen * dir[i]);
        }
        if (uni() < 0.2) {  // the origin on the sphere
            double nv[3];
            const bool tight = uni() < 0.5 && al > 0.0;
            if (tight) {
                for (int i = 0; i < 3; ++i) nv[i] = away[i] / al;
            } else {
                unit(nv);
            }
            const double delta = uni() < 0.7 ? std::pow(10.0, -9.0 + 7.0 * uni()) * (uni() < 0.5 ? -1.0 : 1.0)
                                             : -uni();
            double dv[3];
            if (tight) {
                double pt[3];
                unit(pt);
                const double tilt = uni() < 0.5 ? 0.0 : std::pow(10.0, -6.0 + 5.0 * uni());
                for (int i = 0; i < 3; ++i) dv[i] = nv[i] + tilt * pt[i];
            } else {
                unit(dv);
            }
            for (int i = 0; i < 3; ++i) {
                o[i] = (float)(c[i] + rr * (1.0 + delta) * nv[i]);
                d[i] = (float)(dlen * dv[i]);
            }
        }
        const float r2 = c[3] * c[3];
        const float a = fmaf(d[2], d[2], fmaf(d[1], d[1], d[0] * d[0]));
        double sm = 0.0;
        for (int i = 0; i < 8; ++i)
            sm = std::fmax(sm, std::sqrt((double)sph[i][0] * sph[i][0] + (double)sph[i][1] * sph[i][1] +
                                         (double)sph[i][2] * sph[i][2]) + sph[i][3]);
        float smag = (float)sm;
        if ((double)smag < sm) smag = std::nextafter(smag, INFINITY);
        for (int j = 0; j < 3; ++j) rtx::pf_host_ulp[j] = (int)(uni() * 3.0) - 1;
        const rtx::LineTest T = rtx::line_test_setup(o[0], o[1], o[2], d[0], d[1], d[2], a, smag);
        // the stretched ray (the kernel's own ops: sy * o.y, sy * d.y, a from them, smag * sy)
        const float d1s = sy * d[1];
        const float as = fmaf(d[2], d[2], fmaf(d1s, d1s, d[0] * d[0]));
        const rtx::LineTest Ts = rtx::line_test_setup(o[0], sy * o[1], o[2], d[0], d1s, d[2], as, smag * sy);
        const float thr_b = flat ? Ts.thr * rtx::kCullThrScaleSy : T.thr * rtx::kCullThrScale;
        // flat: both op orders (lane mode: the 5-op flat test; the group coop: the 7-op one)
        const float q = flat ? std::fmin(rtx::line_test_q_flat(Ts, rtx::line_test_flat(Ts, b.cy), b.cx, b.cz, b.R),
                                         rtx::line_test_q(Ts, b.cx, b.cy, b.cz, b.R))
                             : rtx::line_test_q(T, b.cx, b.cy, b.cz, b.R);
        const bool ref = !(ref_disc(o, d, c, -r2, a) < 0.0f);
        ref_pos += ref;
        if (ref && q < thr_b) {
            if (++missed <= 5)
                std::fprintf(stderr, "BLOCK MISS c=(%.9g %.9g %.9g) r=%.9g o=(%.9g %.9g %.9g) d=(%.9g %.9g %.9g) q=%.9g thr_b=%.9g\n",
                             c[0], c[1], c[2], c[3], o[0], o[1], o[2], d[0], d[1], d[2], q, thr_b);
        }
        if (ref && T.thr != -INFINITY && thr_b != -INFINITY) {
            // the line's estimated dperp_b^2 against the bound's inflated R_b - thr_b
            const double used = ((double)b.R - q) / ((double)b.R - thr_b);
            if (used > max_used) max_used = used;
        }
        // the half test, in the bound's space (stretched for flat blocks), both op orders for flat
        const float t_min = uni() < 0.5 ? 0.0f : 1e-3f;
        const rtx::HalfTest H = flat ? rtx::half_test_setup(o[0], sy * o[1], o[2], d[0], d1s, d[2], as, thr_b, t_min)
                                     : rtx::half_test_setup(o[0], o[1], o[2], d[0], d[1], d[2], a, thr_b, t_min);
        const float pw = rtx::half_test_pw(H, b.cx, b.cy, b.cz);
        bool hp = rtx::half_test_pass(pw, rtx::half_test_q2(H, pw, b.R));
        if (flat) {
            const float pwf = rtx::half_test_pw_flat(H, rtx::half_test_kw(H, b.cy), b.cx, b.cz);
            hp = hp && rtx::half_test_pass(pwf, rtx::half_test_q2(H, pwf, b.R));
        }
        const bool acc = ref_accepts(o, d, c, -r2, a, t_min);
        acc_pos += acc;
        half_culled += ref && !acc && !hp;
        if (acc && !hp) {
            if (++half_missed <= 5)
                std::fprintf(stderr, "HALF MISS c=(%.9g %.9g %.9g) r=%.9g o=(%.9g %.9g %.9g) d=(%.9g %.9g %.9g) pw=%.9g "
                             "flat=%d\n", c[0], c[1], c[2], c[3], o[0], o[1], o[2], d[0], d[1], d[2], pw, (int)flat);
        }
        if (acc && pw < 0.0f && H.tha != INFINITY) {
            // pw^2 against K = R_b a - 2 thr_b a: the geometric part is 1 / (1 + k) of it
            const double used = (double)pw * pw / ((double)b.R * H.a + (double)H.tha);
            if (used > half_max_used) half_max_used = used;
        }
    }
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? std::atol(argv[1]) : 2000000;
    long ref_pos = 0, flagged = 0, missed = 0, unsafe = 0, false_pos = 0;
    long s_acc = 0, s_half_missed = 0, s_half_culled = 0;
    double max_used = -1e300, s_half_used = -1e300;
    for (long k = 0; k < n; ++k) {
        double cd[3], dir[3], e[3];
        unit(cd);
        const double cs = std::pow(10.0, -2.0 + 6.0 * uni());
        const double r = std::pow(10.0, -3.0 + 6.0 * uni());
        unit(dir);
        const double pv = uni();
        if (pv < 0.04) {  // near the x axis: v = (0, dz, -dy)/|(dy, dz)| degenerates
            const double eps = std::pow(10.0, -8.0 + 6.0 * uni());
            dir[1] = eps * sym(), dir[2] = eps * sym(), dir[0] = uni() < 0.5 ? -1.0 : 1.0;
        } else if (pv < 0.06) {  // near-vertical
            const double eps = std::pow(10.0, -8.0 + 6.0 * uni());
            dir[0] = eps * sym(), dir[2] = eps * sym(), dir[1] = uni() < 0.5 ? -1.0 : 1.0;
        } else if (pv < 0.09) {  // axis-aligned
            const int ax = (int)(uni() * 3.0) % 3;
            dir[0] = dir[1] = dir[2] = 0.0;
            dir[ax] = uni() < 0.5 ? -1.0 : 1.0;
        }
        // e: unit vector perpendicular to dir
        double t[3];
        unit(t);
        const double td = t[0] * dir[0] + t[1] * dir[1] + t[2] * dir[2];
        const double dn = dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2];
        for (int i = 0; i < 3; ++i) e[i] = t[i] - td / dn * dir[i];
        const double en = std::sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
        if (en < 1e-9) continue;
        for (int i = 0; i < 3; ++i) e[i] /= en;
        // line at distance r (1 + delta) from the centre (delta from 1e-9 to 0.1, either side),
        // or anywhere inside 3r for a fifth of the cases
        double dist;
        if (uni() < 0.8) {
            const double delta = std::pow(10.0, -9.0 + 8.0 * uni()) * (uni() < 0.5 ? -1.0 : 1.0);
            dist = r * (1.0 + delta);
        } else {
            dist = 3.0 * r * uni();
        }
        const double along = sym() * std::pow(10.0, -1.0 + 4.0 * uni()) * std::fmax(r, 1.0);
        const double dlen = std::pow(10.0, -3.0 + 6.0 * uni());
        float c[3], o[3], d[3];
        for (int i = 0; i < 3; ++i) {
            c[i] = (float)(cs * cd[i]);
            o[i] = (float)(cs * cd[i] + dist * e[i] - along * dir[i]);
            d[i] = (float)(dlen * dir[i]);
        }
        if (uni() < 0.2) {  // the origin on (or just inside or outside) the sphere, a third leaving it radially
            double nv[3], dv[3];
            unit(nv);
            const double delta = uni() < 0.7 ? std::pow(10.0, -9.0 + 7.0 * uni()) * (uni() < 0.5 ? -1.0 : 1.0)
                                             : -uni();
            if (uni() < 0.33) {
                double pt[3];
                unit(pt);
                const double tilt = uni() < 0.5 ? 0.0 : std::pow(10.0, -6.0 + 5.0 * uni());
                for (int i = 0; i < 3; ++i) dv[i] = nv[i] + tilt * pt[i];
            } else {
                unit(dv);
            }
            for (int i = 0; i < 3; ++i) {
                o[i] = (float)(cs * cd[i] + r * (1.0 + delta) * nv[i]);
                d[i] = (float)(dlen * dv[i]);
            }
        }
        const float rf = (float)r;
        const float r2 = rf * rf;
        const float a = fmaf(d[2], d[2], fmaf(d[1], d[1], d[0] * d[0]));
        const double sm = std::sqrt((double)c[0] * c[0] + (double)c[1] * c[1] + (double)c[2] * c[2]) + rf;
        float smag = (float)sm;
        if ((double)smag < sm) smag = std::nextafter(smag, INFINITY);
        // the basis's 1-ulp hardware rsq/sqrt: exact, or one ulp either way
        for (int j = 0; j < 3; ++j) rtx::pf_host_ulp[j] = (int)(uni() * 3.0) - 1;
        const rtx::LineTest T = rtx::line_test_setup(o[0], o[1], o[2], d[0], d[1], d[2], a, smag);
        const float R = rtx::prefilter_R(c[0], c[1], c[2], r2);
        const float q = rtx::line_test_q(T, c[0], c[1], c[2], R);
        // the flat-block order (the cy terms first), as the scan runs it on flat blocks
        const float qf = rtx::line_test_q_flat(T, rtx::line_test_flat(T, c[1]), c[0], c[2], R);
        const float disc = ref_disc(o, d, c, -r2, a);
        const bool ref = !(disc < 0.0f);
        const bool flag = !(q < T.thr) && !(qf < T.thr);
        ref_pos += ref;
        flagged += flag;
        false_pos += flag && !ref;
        if (T.thr == -INFINITY) ++unsafe;
        if (ref && !flag) {
            if (++missed <= 5)
                std::fprintf(stderr, "MISS c=(%.9g %.9g %.9g) r=%.9g o=(%.9g %.9g %.9g) d=(%.9g %.9g %.9g) disc=%.9g q=%.9g thr=%.9g\n",
                             c[0], c[1], c[2], rf, o[0], o[1], o[2], d[0], d[1], d[2], disc, q, T.thr);
        }
        if (ref && T.thr != -INFINITY) {
            // share of the margin the rounding errors used: (estimated dperp^2 - r^2) / (R - thr - r^2)
            const double used = (((double)R - std::fmin(q, qf)) - r2) / ((double)R - T.thr - r2);
            if (used > max_used) max_used = used;
        }
        // the sphere-level half test of the culled scan (the bounds' H: thr * kCullThrScale), both orders
        const float t_min = uni() < 0.5 ? 0.0f : 1e-3f;
        const rtx::HalfTest H =
            rtx::half_test_setup(o[0], o[1], o[2], d[0], d[1], d[2], a, T.thr * rtx::kCullThrScale, t_min);
        const float pw = rtx::half_test_pw(H, c[0], c[1], c[2]);
        const float pwf = rtx::half_test_pw_flat(H, rtx::half_test_kw(H, c[1]), c[0], c[2]);
        const bool hp = rtx::half_test_pass(pw, rtx::half_test_q2(H, pw, R)) &&
                        rtx::half_test_pass(pwf, rtx::half_test_q2(H, pwf, R));
        const bool acc = ref_accepts(o, d, c, -r2, a, t_min);
        s_acc += acc;
        s_half_culled += ref && !acc && !hp;
        if (acc && !hp && ++s_half_missed <= 5)
            std::fprintf(stderr, "SPHERE HALF MISS c=(%.9g %.9g %.9g) r=%.9g o=(%.9g %.9g %.9g) d=(%.9g %.9g %.9g) "
                         "pw=%.9g\n", c[0], c[1], c[2], rf, o[0], o[1], o[2], d[0], d[1], d[2], pw);
        if (acc && std::fmin(pw, pwf) < 0.0f && H.tha != INFINITY) {
            const double pm = std::fmin(pw, pwf);
            const double used = pm * pm / ((double)R * H.a + (double)H.tha);
            if (used > s_half_used) s_half_used = used;
        }
    }
    long b_ref = 0, b_missed = 0, h_acc = 0, h_missed = 0, h_culled = 0;
    double b_used = -1e300, h_used = -1e300;
    block_cases(n / 2, b_ref, b_missed, b_used, h_acc, h_missed, h_culled, h_used);
    std::printf("{\"cases\": %ld, \"reference_candidates\": %ld, \"flagged\": %ld, \"false_positives\": %ld, "
                "\"unsafe_lanes\": %ld, \"missed\": %ld, \"max_margin_used\": %.6g, \"block_cases\": %ld, "
                "\"block_reference_candidates\": %ld, \"block_missed\": %ld, \"block_max_used\": %.9g, "
                "\"block_reference_accepted\": %ld, \"half_missed\": %ld, \"half_culled\": %ld, "
                "\"half_max_used\": %.9g, \"sphere_reference_accepted\": %ld, \"sphere_half_missed\": %ld, "
                "\"sphere_half_culled\": %ld, \"sphere_half_max_used\": %.9g}\n",
                n, ref_pos, flagged, false_pos, unsafe, missed, max_used, n / 2, b_ref, b_missed, b_used, h_acc,
                h_missed, h_culled, h_used, s_acc, s_half_missed, s_half_culled, s_half_used);
    return missed || b_missed || h_missed || s_half_missed ? 1 : 0;
}
