// rtx_prefilter.h — the conservative line-distance prefilter of hit_world's
// scan (DESIGN.md §3 "prefilter"), shared by the HIP kernel and the CPU
// margin checker (tests/prefilter_check.cpp).
//
// The reference rejects sphere i when disc = hb^2 - a*cc < 0
// (ShaderCompute.hlsl:163-166 / Sphere.cpp:11-13). In exact arithmetic
// disc / a = r^2 - dperp^2, dperp = distance from the sphere centre to the
// ray's LINE. The kernel's scan does not evaluate the reference's disc
// (11 fp32 ops per sphere); it evaluates
//     Q = R_i - (c.u - o.u)^2 - (c.v - o.v)^2          (7 fp32 ops)
// with (u, v) an orthonormal basis of the plane perpendicular to d, v
// chosen with v.x = 0 (v = (0, dz, -dy) / |(dy, dz)|, u = d/|d| x v), and
// flags the sphere as a candidate when Q >= thr. R_i = r^2 + margin(c, r)
// and thr = -margin(o) are inflated so that
//     reference disc >= 0 (or NaN)  ==>  Q >= thr,
// i.e. the prefilter never drops a sphere the reference would test further.
// A flagged sphere is resolved with the reference's own op sequence
// (rtx_kernels.hip, resolve_one), which rejects false positives, so the
// scan's answer is bit-identical to the reference's.
// Why v.x = 0: on a "flat" block (all 8 centres at one height cy, as every
// small sphere of the RTIOW scenes at y = 0.2) the cy terms of both
// projections are per-ray constants, so c.u - o.u is 2 fma (cx, cz) and
// c.v - o.v ONE fma (cz only): 5 fp32 ops per test instead of 6 with the
// round-2 basis (u.y = 0), whose two projections both kept cx and cz.
//
// Error bound (u = unit roundoff 2^-24, S = |c| + |o|). The
// basis is the round-2 one with the x and y axes exchanged, so the
// term-by-term bound is the same:
//   reference disc rounding, divided by a:    13|oc|^2 + 7r^2
//   oc = fl(o - c) perturbation:               2|oc|^2
//   basis (u, v) error (<= 10u, 4u per vector): 23|oc|^2
//   c.u - o.u, c.v - o.v chains (6u S, 4u S):  15 S^2
//   final two fma:                              4r^2
//   total <= u (53 S^2 + 11 r^2) <= u (106|c|^2 + 106|o|^2 + 11 r^2)
// The basis is built with the 1-ulp hardware reciprocal square root
// (v_rsq_f32: 1/|(dy, dz)| and 1/|d|), not IEEE sqrt and division: it only
// has to be close to orthonormal, its error is in the bound above, and it
// saves ~55 VALU instructions per ray segment.
// The margins below are 1.6e-5 (= 268u) per |c|^2 and |o|^2 and 2e-6
// (= 33u) per r^2, i.e. >= 2.5x that bound, plus an absolute 1e-24 that
// covers subnormal rounding in the region the per-lane `safe` test admits
// (a in [2^-40, 2^40], ray not within ~2^-20 rad of the x axis, no fp32
// overflow). Lanes outside that region get u = v = 0 and thr = -inf: every
// sphere is flagged and the lane ends on the exact sequential path.
#pragma once

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define RTX_HD __host__ __device__ __forceinline__
#else
#define RTX_HD static inline
#endif

namespace rtx {

constexpr float kPreMarginO = 1.6e-5f;  // per |o|^2 (ray side, thr)
constexpr double kPreMarginC = 1.6e-5;  // per |c|^2 (sphere side, R_i)
constexpr double kPreMarginR = 2e-6;    // per r^2   (sphere side, R_i)
constexpr float kPreFloor = 1e-24f;

struct LineTest {
    float ux, uy, uz;  // u = d/|d| x v = (-(dy^2 + dz^2), dx*dy, dx*dz) / (|d| |(dy, dz)|)
    float vy, vz;      // v = (0, dz, -dy) / |(dy, dz)|   (v.x = 0)
    float nou, nov;    // -(o.u), -(o.v)
    float thr;         // flag the sphere when Q >= thr
};

// Sphere side, at upload, in double, rounded UP to fp32. r2 is the
// reference's fl(r*r) (the value the exact scan negates into its soa).
inline float prefilter_R(float cx, float cy, float cz, float r2) {
    const double c2 = (double)cx * cx + (double)cy * cy + (double)cz * cz;
    const double R = (double)r2 + kPreMarginC * c2 + kPreMarginR * (double)r2 + (double)kPreFloor;
    float f = (float)R;
    if ((double)f < R) f = nextafterf(f, INFINITY);
    return f;
}

// The two hardware approximations of the basis: v_rsq_f32 and v_sqrt_f32
// (1 ulp). The host build (tests/prefilter_check.cpp) models them as the
// correctly rounded value moved by pf_host_ulp[k] ulps (-1, 0, +1), set per
// case by the checker.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ float pf_rsq(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ float pf_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
#else
inline int pf_host_ulp[3] = {0, 0, 0};
inline float pf_nudge(float v, int k) {
    return k > 0 ? nextafterf(v, INFINITY) : k < 0 ? nextafterf(v, -INFINITY) : v;
}
inline float pf_rsq_k(float x, int k) { return pf_nudge((float)(1.0 / sqrt((double)x)), pf_host_ulp[k]); }
inline float pf_sqrt(float x) { return pf_nudge((float)sqrt((double)x), pf_host_ulp[2]); }
#endif

// Ray side, once per segment. `a` is the reference's |d|^2 (fma form),
// `smag` an upper bound of |c| + r over the scene (rtx_upload_world).
RTX_HD LineTest line_test_setup(float ox, float oy, float oz, float dx, float dy, float dz, float a,
                                float smag) {
    LineTest T;
    const float m2 = fmaf(dy, dy, dz * dz);
    const float o2 = fmaf(ox, ox, fmaf(oy, oy, oz * oz));
    // a in [2^-40, 2^40]; d not within ~2^-20 rad of the x axis; S = smag +
    // |o| with S^2 and a*S^2 <= 1e36 (no fp32 overflow in disc or Q).
    // NaN or infinite inputs fail these tests.
    const float so = smag + pf_sqrt(o2);  // only bounds the magnitudes (1e36 vs fp32's 3.4e38)
    const float so2 = so * so;
    const bool safe = a >= 9.094947e-13f && a <= 1.0995116e12f && m2 >= a * 9.094947e-13f &&
                      so2 <= 1e36f && a * so2 <= 1e36f;
    if (!safe) {
        T.ux = T.uy = T.uz = T.vy = T.vz = T.nou = T.nov = 0.0f;
        T.thr = -INFINITY;
        return T;
    }
#if defined(__HIP_DEVICE_COMPILE__)
    const float inv_m = pf_rsq(m2);  // m2 >= 2^-80 and a >= 2^-40 here: normal inputs
    const float w = pf_rsq(a) * inv_m;
#else
    const float inv_m = pf_rsq_k(m2, 0);
    const float w = pf_rsq_k(a, 1) * inv_m;
#endif
    T.vy = dz * inv_m;
    T.vz = -dy * inv_m;
    T.ux = -(m2 * w);
    T.uy = (dx * dy) * w;
    T.uz = (dx * dz) * w;
    T.nou = -fmaf(oz, T.uz, fmaf(oy, T.uy, ox * T.ux));
    T.nov = -fmaf(oz, T.vz, oy * T.vy);
    T.thr = -fmaf(o2, kPreMarginO, kPreFloor);
    return T;
}

// Q for one sphere; the kernel runs the same op sequence on sphere pairs
// (v_pk_fma_f32), i.e. the same IEEE fma per element.
RTX_HD float line_test_q(const LineTest &T, float cx, float cy, float cz, float R) {
    const float pu = fmaf(cx, T.ux, fmaf(cy, T.uy, fmaf(cz, T.uz, T.nou)));
    const float pv = fmaf(cy, T.vy, fmaf(cz, T.vz, T.nov));
    return fmaf(-pv, pv, fmaf(-pu, pu, R));
}

// Flat blocks: all 8 spheres of a block share one centre height cy. The cy
// terms of c.u and c.v are then per-ray values, ku = fl(cy*uy - o.u) and
// kv = fl(cy*vy - o.v), computed once per segment, and a test costs 5 fp32
// ops (c.u: 2 fma, c.v: 1 fma, Q: 2 fma) instead of 7. Both projections are
// still fma chains over the same terms (cy first instead of second), so the
// chains' rounding bounds (6u S, 4u S) and the margins above are unchanged;
// tests/prefilter_check.cpp checks both orders.
struct LineFlat {
    float ku, kv;
};
RTX_HD LineFlat line_test_flat(const LineTest &T, float cy) {
    LineFlat K;
    K.ku = fmaf(cy, T.uy, T.nou);
    K.kv = fmaf(cy, T.vy, T.nov);
    return K;
}
RTX_HD float line_test_q_flat(const LineTest &T, const LineFlat &K, float cx, float cz, float R) {
    const float pu = fmaf(cx, T.ux, fmaf(cz, T.uz, K.ku));
    const float pv = fmaf(cz, T.vz, K.kv);
    return fmaf(-pv, pv, fmaf(-pu, pu, R));
}

// Block bounds of the culled scan (DESIGN.md §3 "culled scan"). The lane-
// mode scan of small scenes visits 8-sphere blocks of a spatially ordered
// copy of the scene and first tests, per lane, each block's bounding sphere
// (C_b, R_b) with the same 7/5-op test as a sphere: a block no lane's line
// passes is skipped. Exactness needs: reference disc_i >= 0 for a sphere i
// of the block  ==>  the block test passes. Derivation (u = 2^-24, exact
// reals unless fl()):
//   reference disc_i >= 0  ==>  dperp_i^2 <= r_i^2 + u (13|oc_i|^2 + 7 r_i^2)
//                          <= A_i + B,  A_i = r_i^2 (1 + 8u) + 27u |c_i|^2,
//                                        B = 26u |o|^2         (|oc|^2 <= 2|o|^2 + 2|c|^2)
//   dperp_b <= |c_i - C_b| + dperp_i <= rho + sqrt(B),  rho = max_i (|c_i - C_b| + sqrt(A_i))
//   dperp_b^2 <= (1 + k) rho^2 + (1 + 1/k) B            (any k > 0; k = 1/32)
// The block test is the sphere test on (C_b, R_b), whose own rounding the
// sphere margins cover (above: u (53 S^2 + 11 R), S = |C_b| + |o|), so
//   R_b   = fl_up((1 + k) rho^2 (1 + kPreMarginR) + kPreMarginC |C_b|^2 + kPreFloor)
//   thr_b = -(kPreMarginO + (1 + 1/k) 26u) |o|^2 - kPreFloor  >=  thr * kCullThrScale
// (kPreMarginO + 33 * 26u = 6.71e-5 <= 1.6e-5 * 4.25 = 6.8e-5; thr = -inf
// stays -inf). tests/prefilter_check.cpp checks the claim on adversarial
// near-tangent rays through random blocks.
constexpr float kCullThrScale = 4.25f;
constexpr double kCullK = 1.0 / 32.0;
// Flat bounds (every sphere at height flat_cy: the scene's thin layer) are
// tested in a space stretched along y by kCullSy: the ray (o, d) becomes
// (ox, s oy, oz), (dx, s dy, dz) (exact in fp32: s is a power of two), the
// bound's centre (cx, s cy, cz). A sphere of radius r becomes an ellipsoid
// inside the sphere of radius s r, and a point p of the line at distance
// dperp_i from c_i maps to a point of the stretched line at distance <=
// s dperp_i from the stretched centre, so the derivation above holds with
// |c_i - C_b| measured in the stretched space, sqrt(A_i) and sqrt(B) scaled
// by s, and |o| <= |o'|: rho' = max_i (|A c_i - C'_b| + s sqrt(A_i)),
// thr'_b = -(kPreMarginO + (1 + 1/k) 26u s^2) |o'|^2 - kPreFloor, which is
// >= thr' * kCullThrScaleSy (s = 8: 1.6e-5 + 33 * 26u * 64 = 3.289e-3 <= 1.6e-5 * 206).
// The layer's bounds become nearly spheres (the layer is ~0.4 thick, a
// block 2 x 4 cells wide), and a line passing above a patch no longer passes
// its bound: at C5 (s = 4) a wave's lines pass 2.0 % of the flat block bounds
// instead of 4.6 % (tools/block_cull_sim.py on the sampled rays). s = 8 since
// the half test (below): C5 138.7 -> 129.5 ms (2 and 16
// slower; 4 was best without it).
#ifndef RTX_CULL_SY  // the stretch (a power of two: the scaling is exact)
#define RTX_CULL_SY 8
#endif
constexpr float kCullSy = (float)RTX_CULL_SY;
static_assert(RTX_CULL_SY >= 1 && (RTX_CULL_SY & (RTX_CULL_SY - 1)) == 0, "the stretch is a power of two");
// 1 + (1 + 1/k) 26u sy^2 / kPreMarginO, rounded up (206 at sy = 8, 53 at 4)
constexpr float kCullThrScaleSy =
    (float)(int)(2.0 + (1.0 + 1.0 / kCullK) * 26.0 * 5.9604644775390625e-08 * RTX_CULL_SY * RTX_CULL_SY / 1.6e-5);

// Half-space part of the bound test. The line test above passes bounds the
// ray's LINE passes, also those wholly behind the origin. The reference
// accepts sphere i only at a root c >= t_min >= 0 (ShaderCompute.hlsl:
// 160-166; oracle hit_world32), and then some point p = o + t d, t >= 0,
// lies within sqrt(A_i + B) (1 + u) of c_i:
//   near root accepted  ==>  fl(-hb - sq) >= 0  ==>  hb_c <= 0, and
//     dot(c - o, d) >= -5u |c - o| |d|: the line's closest point (if t0 >= 0)
//     or o itself (t0 in [-5u|c-o|/|d|, 0)) is within dperp_i (1 + u);
//   far root accepted with hb_c > 0  ==>  disc_c >= hb_c^2 (1 - 2u)  ==>
//     |o - c|^2 <= r^2 (1 + 16u): o itself, inside sqrt(A_i) (1 + 2u);
// dperp_i^2 <= A_i + B as above. So |p - C_b| <= rho + sqrt(B) (1 + 2u) and
//   pw = dot(C_b - o, d) = dot(C_b - p, d) + t a >= -(rho + sqrt(B)(1+2u)) |d|.
// The kernel's pw_c = fl(C.d - o.d) is within e|d|, e = 4.2u (|C_b| + |o|),
// and pw_c^2 <= ((1+k) rho^2 + (1+1/k)(1.1 B + 11 e^2)) a whenever pw_c < 0;
// K = fl(fma(R_b, a, fl(-2 thr_b a))) exceeds that: R_b holds (1+k) rho^2
// (1 + 2e-6) and 1.6e-5 |C_b|^2, and -2 thr_b >= 2 (6.71e-5 |o|^2) covers
// (1 + 1/k) 1.1 B = 5.6e-5 |o|^2 (stretched, s = 8: 2 * 3.30e-3 |o'|^2 against
// 33 * 1.1 * 64 * 26u = 3.6e-3 |o'|^2, the proof carrying over as for the
// line test: S p = S o + t S d is a point of the stretched ray). A bound
// fails the half test iff pw_c < 0 and fl(fma(-pw_c, pw_c, K)) < 0; NaN
// passes; thr_b = -inf (a lane outside the safe range) and t_min < 0 make
// K = +inf: every bound passes. Checked with the line test by
// tests/prefilter_check.cpp (block cases: reference acceptance at t_min 0
// and 1e-3, origins on and inside the sphere, spheres behind the origin).
struct HalfTest {
    float dx, dy, dz, nod, a, tha;
};
RTX_HD HalfTest half_test_setup(float ox, float oy, float oz, float dx, float dy, float dz, float a, float thr_b,
                                float t_min) {
    HalfTest H;
    H.dx = dx, H.dy = dy, H.dz = dz, H.a = a;
    H.nod = -fmaf(oz, dz, fmaf(oy, dy, ox * dx));
    const float th = (-2.0f * thr_b) * a;
    H.tha = t_min >= 0.0f ? th : INFINITY;
    return H;
}
// the 7-op order (c.d first), and the flat order (cy's term per ray: kw)
RTX_HD float half_test_pw(const HalfTest &H, float cx, float cy, float cz) {
    return fmaf(cx, H.dx, fmaf(cy, H.dy, fmaf(cz, H.dz, H.nod)));
}
RTX_HD float half_test_kw(const HalfTest &H, float cy) { return fmaf(cy, H.dy, H.nod); }
RTX_HD float half_test_pw_flat(const HalfTest &H, float kw, float cx, float cz) {
    return fmaf(cx, H.dx, fmaf(cz, H.dz, kw));
}
RTX_HD float half_test_q2(const HalfTest &H, float pw, float R) { return fmaf(-pw, pw, fmaf(R, H.a, H.tha)); }
RTX_HD bool half_test_pass(float pw, float q2) { return !(pw < 0.0f && q2 < 0.0f); }

struct CullBound {
    float cx, cy, cz, R;
};
#ifndef RTX_CULL_CENTRE_ITERS  // centre search steps of cull_bound (0: the box centre)
#define RTX_CULL_CENTRE_ITERS 64
#endif
// Spheres (cx, cy, cz, r)[m] as uploaded; flat: every centre has height
// flat_cy (the bound's centre takes it exactly, so the 5-op test applies).
// sy: the stretch along y (1, or kCullSy for a flat bound: then the centre
// returned is in the stretched space, cy = sy * flat_cy).
inline CullBound cull_bound(const float *const *sph, int m, bool flat, float flat_cy, float sy = 1.0f) {
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = 0; i < m; ++i)
        for (int k = 0; k < 3; ++k) {
            lo[k] = fmin(lo[k], (double)sph[i][k]);
            hi[k] = fmax(hi[k], (double)sph[i][k]);
        }
    CullBound b;
    b.cx = (float)(0.5 * (lo[0] + hi[0]));
    b.cy = flat ? sy * flat_cy : (float)(sy * 0.5 * (lo[1] + hi[1]));
    b.cz = (float)(0.5 * (lo[2] + hi[2]));
    const double u = 5.9604644775390625e-08;
#if RTX_CULL_CENTRE_ITERS > 0
    {
        // A tighter centre than the box's (the proof holds for any centre:
        // rho is measured from the one chosen): Badoiu-Clarkson steps towards
        // the farthest sphere surface, keeping the best; a flat bound's centre
        // keeps its height (the 5-op test's per-ray cy term).
        double c[3] = {b.cx, b.cy, b.cz}, best[3] = {c[0], c[1], c[2]}, best_rho = INFINITY;
        for (int it = 1; it <= RTX_CULL_CENTRE_ITERS; ++it) {
            double far = -1.0, fv[3] = {0, 0, 0};
            for (int i = 0; i < m; ++i) {
                const double v[3] = {sph[i][0] - c[0], sy * (double)sph[i][1] - c[1], sph[i][2] - c[2]};
                const double dd = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
                const double e = dd + sy * (double)sph[i][3];
                if (e > far) {
                    far = e;
                    const double k = dd > 0.0 ? e / dd : 0.0;
                    fv[0] = v[0] * k, fv[1] = v[1] * k, fv[2] = v[2] * k;
                }
            }
            if (far < best_rho) best_rho = far, best[0] = c[0], best[1] = c[1], best[2] = c[2];
            const double step = 1.0 / (it + 1);
            c[0] += fv[0] * step;
            if (!flat) c[1] += fv[1] * step;
            c[2] += fv[2] * step;
        }
        b.cx = (float)best[0];
        b.cy = flat ? b.cy : (float)best[1];
        b.cz = (float)best[2];
    }
#endif
    double rho = 0.0;
    for (int i = 0; i < m; ++i) {
        const double dx = (double)sph[i][0] - b.cx, dy = (double)sy * sph[i][1] - b.cy, dz = (double)sph[i][2] - b.cz;
        const double r = sph[i][3];
        const double c2 = (double)sph[i][0] * sph[i][0] + (double)sph[i][1] * sph[i][1] + (double)sph[i][2] * sph[i][2];
        const double A = r * r * (1.0 + 8.0 * u) + 27.0 * u * c2;
        // (double rounding of these few ops is ~1e-16 relative: the 1e-12 covers it)
        rho = fmax(rho, (sqrt(dx * dx + dy * dy + dz * dz) + (double)sy * sqrt(A)) * (1.0 + 1e-12));
    }
    const double cb2 = (double)b.cx * b.cx + (double)b.cy * b.cy + (double)b.cz * b.cz;
    const double R = (1.0 + kCullK) * rho * rho * (1.0 + kPreMarginR) + kPreMarginC * cb2 + (double)kPreFloor;
    float f = (float)R;
    if ((double)f < R) f = nextafterf(f, INFINITY);
    b.R = f;
    return b;
}

}  // namespace rtx
