/*
 * rtx_oracle.c — CPU oracle (TEST INFRASTRUCTURE ONLY; see rtx_oracle.h).
 *
 * Compile with -ffp-contract=off and without fast-math: every fused
 * multiply-add below is an explicit fmaf, all other float operations are
 * single IEEE-754 binary32 operations, so this file executes the same
 * operation sequence as the HIP kernel (raytrace-we-gpu_amd/csrc).
 *
 * Reference lines followed (all under /root/reference):
 *   CSVersion/ShaderCompute.hlsl  baseHash :23-28, hash1/2/3 :30-48,
 *       random_in_unit_sphere :59-66, reflect/refract/reflectance :76-97,
 *       toGamma :99-103, get_ray :118-127, set_face_normal :143-150,
 *       hit_sphere :155-186, hit_world :188-205, scatter :207-252,
 *       sample_color :255-287, CSMain :291-315
 *   Sphere.cpp:3-32, Hittable_list.cpp:3-20, Hittable.h:12-16, Ray.h:16-19,
 *   Vec3.h:83-86 (operator/ = multiply by reciprocal), Camera.h:9-26
 *   CSVersion/DxCSApp.cpp  random() :6-9, ComputeViewVals :39-61,
 *       random_world :72-134, test_world :136-157, focus_dist :488
 */
#include "rtx_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* bit casts                                                                 */
static inline uint32_t f2u(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
static inline float u2f(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* ------------------------------------------------------------------------ */
/* fp32 vector helpers (literal, uncontracted)                               */
typedef struct {
    float x, y, z;
} v3f;
static inline v3f v3(float x, float y, float z) {
    v3f r = {x, y, z};
    return r;
}
static inline v3f vadd(v3f a, v3f b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3f vsub(v3f a, v3f b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3f vneg(v3f a) { return v3(-a.x, -a.y, -a.z); }
static inline v3f vmul(v3f a, v3f b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3f vscale(float s, v3f a) { return v3(s * a.x, s * a.y, s * a.z); }
static inline float vdot(v3f a, v3f b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
/* normalize(v) = v * (1 / sqrt(dot(v, v))) */
static inline v3f vnorm(v3f v) {
    const float inv = 1.0f / sqrtf(vdot(v, v));
    return vscale(inv, v);
}
/* RTX_FRAME_LAMBERT_GUARD: Shader_RT.fx:222-225 with near_zero of
 * ShaderCompute.hlsl:70-74 (s = 1e-9). */
static inline v3f lambert_guard32(v3f v, v3f nrm, uint32_t guard) {
    const float s = 0.000000001f;
    if (guard && fabsf(v.x) < s && fabsf(v.y) < s && fabsf(v.z) < s) return nrm;
    return v;
}

/* ------------------------------------------------------------------------ */
/* RNG, ShaderCompute.hlsl:23-48                                              */
uint32_t or_base_hash(uint32_t px, uint32_t py) {
    const uint32_t qx = 1103515245u * ((px >> 1) ^ py);
    const uint32_t qy = 1103515245u * ((py >> 1) ^ px);
    const uint32_t h = 1103515245u * (qx ^ (qy >> 3));
    return h ^ (h >> 16);
}
static inline uint32_t hash_step(float *seed) {
    *seed = *seed + 0.1f;
    const float a = *seed;
    *seed = *seed + 0.1f;
    const float b = *seed;
    return or_base_hash(f2u(a), f2u(b));
}
static inline float hash1(float *seed) { return (float)hash_step(seed) / 4294967296.0f; }
static inline void hash2(float *seed, float *h0, float *h1) {
    const uint32_t n = hash_step(seed);
    *h0 = (float)(n & 0x7fffffffu) / 2147483648.0f;
    *h1 = (float)((n * 48271u) & 0x7fffffffu) / 2147483648.0f;
}
static inline v3f hash3(float *seed) {
    const uint32_t n = hash_step(seed);
    return v3((float)(n & 0x7fffffffu) / 2147483648.0f,
              (float)((n * 16807u) & 0x7fffffffu) / 2147483648.0f,
              (float)((n * 48271u) & 0x7fffffffu) / 2147483648.0f);
}

/* ------------------------------------------------------------------------ */
/* sin/cos: q = rint(x*2/pi), Cody-Waite reduction, minimax polynomials.     */
static inline void sincos_rt(float x, float *s, float *c) {
    const float q = rintf(x * 0.636619772f);
    float r = fmaf(q, -1.57079637f, x);
    r = fmaf(q, 4.37113900e-8f, r);
    const float z = r * r;
    float ps = fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f);
    ps = fmaf(z, ps, -1.6666654611e-1f);
    const float S = fmaf(r * z, ps, r);
    float pc = fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
    pc = fmaf(z, pc, 4.166664568298827e-2f);
    const float C = fmaf(z * z, pc, fmaf(-0.5f, z, 1.0f));
    const int n = ((int)q) & 3;
    *s = (n == 0) ? S : (n == 1) ? C : (n == 2) ? -S : -C;
    *c = (n == 0) ? C : (n == 1) ? -S : (n == 2) ? -C : S;
}

/* log2 for x > 0 finite: ln(m) = 2 atanh((m-1)/(m+1)), m in [sqrt(1/2), sqrt(2)] */
static inline float log2_rt(float x) {
    int e = 0;
    if (x < 1.17549435e-38f) {
        x = x * 8388608.0f;
        e = -23;
    }
    const uint32_t b = f2u(x);
    e += (int)(b >> 23) - 127;
    float m = u2f((b & 0x007fffffu) | 0x3f800000u);
    if (m > 1.41421354f) {
        m = m * 0.5f;
        e += 1;
    }
    const float f = m - 1.0f;
    const float s = f / (2.0f + f);
    const float z = s * s;
    float p = fmaf(z, 0.111111111f, 0.142857143f);
    p = fmaf(z, p, 0.2f);
    p = fmaf(z, p, 0.333333333f);
    const float s2 = s + s;
    const float ln = fmaf(s2 * z, p, s2);
    return fmaf(ln, 1.44269502f, (float)e);
}
static inline float exp2_rt(float t) {
    if (!(t == t)) return t;
    if (t >= 128.0f) return u2f(0x7f800000u);
    if (t < -150.0f) return 0.0f;
    const float nf = rintf(t);
    const float r = t - nf;
    float p = fmaf(r, 1.52527338e-5f, 1.54035304e-4f);
    p = fmaf(r, p, 1.33335581e-3f);
    p = fmaf(r, p, 9.61812911e-3f);
    p = fmaf(r, p, 5.55041087e-2f);
    p = fmaf(r, p, 2.40226507e-1f);
    p = fmaf(r, p, 6.93147181e-1f);
    p = fmaf(r, p, 1.0f);
    int n = (int)nf;
    if (n < -126) {
        p = p * 5.42101086e-20f;
        n += 64;
    }
    if (n > 127) {
        p = p * 2.0f;
        n -= 1;
    }
    return p * u2f((uint32_t)(n + 127) << 23);
}
static inline float pow_rt(float x, float y) {
    if (!(x == x)) return x;
    if (x < 0.0f) return u2f(0x7fc00000u);
    if (x == 0.0f) return 0.0f;
    if (x == u2f(0x7f800000u)) return x;
    return exp2_rt(y * log2_rt(x));
}

/* random_in_unit_sphere, ShaderCompute.hlsl:59-66 */
static inline v3f rius(float *seed) {
    const v3f h = hash3(seed);
    const float hx = h.x * 2.0f - 1.0f;
    const float phi = h.y * 6.28318530718f;
    const float r = pow_rt(h.z, 0.333333333f);
    const float sq = sqrtf(1.0f - hx * hx);
    float sn, cs;
    sincos_rt(phi, &sn, &cs);
    return v3(r * (sq * sn), r * (sq * cs), r * hx);
}
/* random_in_unit_disk, ShaderCompute.hlsl:50-57 (thin-lens extension) */
static inline v3f rind(float *seed) {
    float h0, h1;
    hash2(seed, &h0, &h1);
    const float phi = h1 * 6.28318530718f;
    const float r = sqrtf(h0 * 1.0f);
    float sn, cs;
    sincos_rt(phi, &sn, &cs);
    return v3(r * sn, r * cs, 0.0f);
}
static inline v3f reflect3(v3f v, v3f n) {
    const float k = 2.0f * vdot(v, n);
    return vsub(v, vscale(k, n));
}
static inline v3f refract3(v3f uv, v3f n, float ratio) {
    const float cos_theta = fminf(vdot(vneg(uv), n), 1.0f);
    const v3f r_perp = vscale(ratio, vadd(uv, vscale(cos_theta, n)));
    const float lp = sqrtf(vdot(r_perp, r_perp));
    const float k = -sqrtf(fabsf(1.0f - lp * lp));
    return vadd(r_perp, vscale(k, n));
}
static inline float reflectance(float cosine, float ref_idx) {
    float r0 = (1.0f - ref_idx) / (1.0f + ref_idx);
    r0 = r0 * r0;
    const float x = 1.0f - cosine;
    const float x2 = x * x;
    const float x5 = (x2 * x2) * x;
    return r0 + (1.0f - r0) * x5;
}
static inline float to_gamma(float c) { return pow_rt(c, 0.454545454545f); }

int or_math(int fn, const float *in0, const float *in1, uint32_t n, float *out) {
    if (!in0 || !out) return -1;
    if (fn == 12 || fn == 13) { /* diffuse direction, ShaderCompute.hlsl:211-212 */
        if (!in1) return -1;
        for (uint32_t i = 0; i < n; ++i) {
            const v3f p = v3(in0[3 * i], in0[3 * i + 1], in0[3 * i + 2]);
            const v3f nrm = v3(in1[6 * i], in1[6 * i + 1], in1[6 * i + 2]);
            const v3f r = v3(in1[6 * i + 3], in1[6 * i + 4], in1[6 * i + 5]);
            const v3f d = vnorm(lambert_guard32(vsub(vadd(vadd(p, nrm), r), p), nrm, fn == 13));
            out[3 * i] = d.x;
            out[3 * i + 1] = d.y;
            out[3 * i + 2] = d.z;
        }
        return 0;
    }
    for (uint32_t i = 0; i < n; ++i) {
        const float a = in0[i];
        const float b = in1 ? in1[i] : 0.0f;
        float seed = a, s, c;
        v3f h;
        switch (fn) {
            case 0: out[i] = sqrtf(a); break;
            case 1: out[i] = a / b; break;
            case 2: sincos_rt(a, &s, &c); out[i] = s; break;
            case 3: sincos_rt(a, &s, &c); out[i] = c; break;
            case 4: out[i] = log2_rt(a); break;
            case 5: out[i] = exp2_rt(a); break;
            case 6: out[i] = pow_rt(a, b); break;
            case 7: out[i] = u2f(or_base_hash(f2u(a), f2u(b))); break;
            case 8: out[3 * i] = hash1(&seed); out[3 * i + 1] = seed; out[3 * i + 2] = 0.0f; break;
            case 9: hash2(&seed, &out[3 * i], &out[3 * i + 1]); out[3 * i + 2] = seed; break;
            case 10: h = hash3(&seed); out[3 * i] = h.x; out[3 * i + 1] = h.y; out[3 * i + 2] = h.z; break;
            case 11: h = rius(&seed); out[3 * i] = h.x; out[3 * i + 1] = h.y; out[3 * i + 2] = h.z; break;
            default: return -1;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* fp32 twin: scene in the kernel's layout                                   */
typedef struct {
    uint32_t n, depth, spp;
    float *cx, *cy, *cz, *negr2, *rad, *mv; /* mv: 4 per sphere */
    int *mt;
} scene32;

static int scene32_init(scene32 *S, const or_world *w) {
    const uint32_t n = w->count;
    memset(S, 0, sizeof(*S));
    S->n = n;
    S->depth = w->depth;
    S->spp = w->spp;
    const size_t cap = n ? n : 1;
    S->cx = malloc(cap * 4);
    S->cy = malloc(cap * 4);
    S->cz = malloc(cap * 4);
    S->negr2 = malloc(cap * 4);
    S->rad = malloc(cap * 4);
    S->mv = malloc(cap * 16);
    S->mt = malloc(cap * sizeof(int));
    if (!S->cx || !S->cy || !S->cz || !S->negr2 || !S->rad || !S->mv || !S->mt) return -1;
    for (uint32_t i = 0; i < n; ++i) {
        const float r = w->spheres[4 * i + 3];
        S->cx[i] = w->spheres[4 * i + 0];
        S->cy[i] = w->spheres[4 * i + 1];
        S->cz[i] = w->spheres[4 * i + 2];
        S->negr2[i] = -(r * r);
        S->rad[i] = r;
        const float t = w->mat_types[i];
        S->mt[i] = (t == 0.0f) ? 0 : (t == 1.0f) ? 1 : (t == 2.0f) ? 2 : 3;
        for (int k = 0; k < 4; ++k) S->mv[4 * i + k] = w->mat_values[4 * i + k];
    }
    return 0;
}
static void scene32_free(scene32 *S) {
    free(S->cx);
    free(S->cy);
    free(S->cz);
    free(S->negr2);
    free(S->rad);
    free(S->mv);
    free(S->mt);
}

/* hit_world, fp32 twin (kernel spec: DESIGN.md §4 "hit_sphere"). */
static inline int hit_world32(const scene32 *S, v3f o, v3f d, float a, float inv_a, float t_min,
                              float *best_io) {
    float best = *best_io;
    int idx = -1;
    const uint32_t n = S->n;
    for (uint32_t i = 0; i < n; ++i) {
        const float ocx = o.x - S->cx[i];
        const float ocy = o.y - S->cy[i];
        const float ocz = o.z - S->cz[i];
        const float hb = fmaf(ocz, d.z, fmaf(ocy, d.y, ocx * d.x));
        const float cc = fmaf(ocz, ocz, fmaf(ocy, ocy, fmaf(ocx, ocx, S->negr2[i])));
        const float disc = fmaf(hb, hb, -(a * cc));
        if (!(disc < 0.0f)) {
            const float sq = sqrtf(disc);
            float root = (-hb - sq) * inv_a;
            int ok = !(root < t_min || best < root);
            if (!ok) {
                root = (-hb + sq) * inv_a;
                ok = !(root < t_min || best < root);
            }
            if (ok) {
                best = root;
                idx = (int)i;
            }
        }
    }
    *best_io = best;
    return idx;
}
static inline float dir_len2(v3f d) { return fmaf(d.z, d.z, fmaf(d.y, d.y, d.x * d.x)); }

/* hit record of the winner (Sphere.cpp:26-29, Hittable.h:12-16) */
static inline void hit_record32(const scene32 *S, int idx, float t, v3f o, v3f d, v3f *p, v3f *nrm,
                                int *ff) {
    *p = vadd(o, vscale(t, d));
    const float inv_r = 1.0f / S->rad[idx];
    v3f n = vscale(inv_r, vsub(*p, v3(S->cx[idx], S->cy[idx], S->cz[idx])));
    *ff = vdot(d, n) < 0.0f;
    if (!*ff) n = vneg(n);
    *nrm = n;
}

int or_hit_world_f32(const or_world *w, const float *rays, uint32_t nr, float t_min, float t_max,
                     float *out) {
    scene32 S;
    if (!w || !rays || !out) return -1;
    if (scene32_init(&S, w)) {
        scene32_free(&S);
        return -1;
    }
    for (uint32_t i = 0; i < nr; ++i) {
        const v3f o = v3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
        const v3f d = v3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        const float a = dir_len2(d);
        const float inv_a = 1.0f / a;
        float best = t_max;
        const int idx = hit_world32(&S, o, d, a, inv_a, t_min, &best);
        float *r = out + 10 * (size_t)i;
        if (idx < 0) {
            for (int k = 0; k < 10; ++k) r[k] = 0.0f;
            r[9] = -1.0f;
            continue;
        }
        v3f p, nrm;
        int ff;
        hit_record32(&S, idx, best, o, d, &p, &nrm, &ff);
        r[0] = 1.0f;
        r[1] = best;
        r[2] = p.x; r[3] = p.y; r[4] = p.z;
        r[5] = nrm.x; r[6] = nrm.y; r[7] = nrm.z;
        r[8] = ff ? 1.0f : 0.0f;
        r[9] = (float)idx;
    }
    scene32_free(&S);
    return 0;
}

typedef struct {
    v3f org, hor, ver, llc;
    float img_w, img_h;
    uint32_t width, rng_mode, frame_index, flags;
    v3f lu, lv;
    float lens_r;
    int linear; /* 1: write the linear sample sum instead of toGamma(sum/spp) */
} frame32;

static inline float pixel_seed(const frame32 *F, uint32_t spp, uint32_t x, uint32_t y, uint32_t s) {
    uint32_t h = or_base_hash(x, y);
    if (F->rng_mode == 1u)
        h = or_base_hash(h, F->frame_index * spp + s);
    else if (F->frame_index != 0u)
        h = or_base_hash(h, 0x80000000u | F->frame_index);
    return (float)h / 4294967296.0f;
}

/* CSMain for one pixel, fp32 twin (ShaderCompute.hlsl:291-315). */
static void pixel32(const scene32 *S, const frame32 *F, uint32_t x, uint32_t y, float out[4],
                    uint64_t *segs) {
    float seed = pixel_seed(F, S->spp, x, y, 0);
    v3f acc = v3(0.0f, 0.0f, 0.0f);
    uint64_t sg = 0;
    for (uint32_t s = 0; s < S->spp && S->depth > 0; ++s) {
        if (F->rng_mode == 1u) seed = pixel_seed(F, S->spp, x, y, s);
        float h0, h1, g0, g1;
        hash2(&seed, &h0, &h1);
        const float u = ((float)x + h0 * 1.1f) / (F->img_w - 1.0f);
        hash2(&seed, &g0, &g1);
        const float v = ((float)y + g1 * 1.1f) / (F->img_h - 1.0f);
        v3f o = F->org;
        v3f d = vsub(vadd(vadd(F->llc, vscale(u, F->hor)), vscale(v, F->ver)), F->org);
        if (F->lens_r > 0.0f) { /* thin lens, Shader_RT.fx:288-298 */
            const v3f rd = vscale(F->lens_r, rind(&seed));
            const v3f off = vadd(vscale(rd.x, F->lu), vscale(rd.y, F->lv));
            o = vadd(o, off);
            d = vsub(d, off);
        }
        v3f col = v3(1.0f, 1.0f, 1.0f);
        /* sample_color, :255-287 */
        for (uint32_t k = 0; k < S->depth; ++k) {
            const float a = dir_len2(d);
            const float inv_a = 1.0f / a;
            float best = u2f(0x7f800000u);
            const int idx = hit_world32(S, o, d, a, inv_a, 0.001f, &best);
            ++sg;
            if (idx >= 0) {
                v3f p, nrm, dir;
                int ff;
                hit_record32(S, idx, best, o, d, &p, &nrm, &ff);
                const int mt = S->mt[idx];
                const float *mv = S->mv + 4 * idx;
                if (mt == 0) {
                    const v3f r = rius(&seed);
                    const v3f target = vadd(vadd(p, nrm), r);
                    dir = vnorm(lambert_guard32(vsub(target, p), nrm, F->flags & 1u));
                    col = vmul(col, v3(mv[0], mv[1], mv[2]));
                } else if (mt == 1) {
                    const v3f refl = reflect3(d, nrm);
                    const v3f r = rius(&seed);
                    dir = vnorm(vadd(refl, vscale(mv[3], r)));
                    col = vmul(col, v3(mv[0], mv[1], mv[2]));
                } else if (mt == 2) {
                    const float ratio = ff ? (1.0f / mv[3]) : mv[3];
                    const v3f ud = vnorm(d);
                    const float cosine = fminf(vdot(vneg(ud), nrm), 1.0f);
                    const float sine = sqrtf(1.0f - cosine * cosine);
                    const int cant = ratio * sine > 1.0f;
                    const float refl = reflectance(cosine, ratio);
                    const float h = hash1(&seed); /* FXC: no short-circuit */
                    dir = (cant || refl > h) ? reflect3(ud, nrm) : refract3(ud, nrm, ratio);
                } else {
                    break; /* scatter false: black */
                }
                o = p;
                d = dir;
            } else {
                const v3f ud = vnorm(d);
                const float tt = 0.5f * (ud.y + 1.0f);
                const float wgt = 1.0f - tt;
                const v3f sky = v3(wgt + tt * 0.5f, wgt + tt * 0.7f, wgt + tt);
                acc = vadd(acc, vmul(col, sky));
                break;
            }
        }
    }
    const float spp = (float)S->spp;
    if (F->linear) {
        out[0] = acc.x;
        out[1] = acc.y;
        out[2] = acc.z;
    } else {
        out[0] = to_gamma(acc.x / spp);
        out[1] = to_gamma(acc.y / spp);
        out[2] = to_gamma(acc.z / spp);
    }
    out[3] = 1.0f;
    *segs += sg;
}

/* ------------------------------------------------------------------------ */
/* fp64 mode: Sphere.cpp / Hittable_list.cpp / Vec3.h algebra in double,    */
/* same fp32 RNG chain, libm transcendentals.                                */
typedef struct {
    double x, y, z;
} v3d;
static inline v3d d3(double x, double y, double z) {
    v3d r = {x, y, z};
    return r;
}
static inline v3d dadd(v3d a, v3d b) { return d3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3d dsub(v3d a, v3d b) { return d3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3d dneg(v3d a) { return d3(-a.x, -a.y, -a.z); }
static inline v3d dmul(v3d a, v3d b) { return d3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3d dscale(double t, v3d a) { return d3(t * a.x, t * a.y, t * a.z); }
static inline double ddot(v3d a, v3d b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline double dlen2(v3d a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
/* unit_vector(v) = v / v.length() = (1/len) * v   (Vec3.h:83-86, :102-105) */
static inline v3d dunit(v3d v) { return dscale(1.0 / sqrt(dlen2(v)), v); }

/* Sphere::hit (Sphere.cpp:3-32) */
static inline int sphere_hit64(const double *c4, v3d o, v3d d, double t_min, double t_max,
                               double *t_out) {
    const v3d oc = dsub(o, d3(c4[0], c4[1], c4[2]));
    const double a = dlen2(d);
    const double half_b = ddot(oc, d);
    const double c = dlen2(oc) - c4[3] * c4[3];
    const double discr = half_b * half_b - a * c;
    if (discr < 0) return 0;
    const double sqrtd = sqrt(discr);
    double root = (-half_b - sqrtd) / a;
    if (root < t_min || root > t_max) {
        root = (-half_b + sqrtd) / a;
        if (root < t_min || root > t_max) return 0;
    }
    *t_out = root;
    return 1;
}
/* Hittable_list::hit (Hittable_list.cpp:3-20) */
static inline int hit_world64(const double *sph, uint32_t n, v3d o, v3d d, double t_min,
                              double t_max, double *t_out) {
    int idx = -1;
    double closest = t_max;
    for (uint32_t i = 0; i < n; ++i) {
        double t;
        if (sphere_hit64(sph + 4 * i, o, d, t_min, closest, &t)) {
            closest = t;
            idx = (int)i;
        }
    }
    *t_out = closest;
    return idx;
}
/* rec.p = r.at(t); outward_normal = (p - center) / radius; set_face_normal */
static inline void hit_record64(const double *c4, double t, v3d o, v3d d, v3d *p, v3d *nrm, int *ff) {
    *p = dadd(o, dscale(t, d));
    v3d n = dscale(1.0 / c4[3], dsub(*p, d3(c4[0], c4[1], c4[2])));
    *ff = ddot(d, n) < 0.0;
    *nrm = *ff ? n : dneg(n);
}

int or_hit_world_f64(const double *sph, uint32_t count, const double *rays, uint32_t nr,
                     double t_min, double t_max, double *out) {
    if (!sph || !rays || !out) return -1;
    for (uint32_t i = 0; i < nr; ++i) {
        const v3d o = d3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
        const v3d d = d3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        double t;
        const int idx = hit_world64(sph, count, o, d, t_min, t_max, &t);
        double *r = out + 10 * (size_t)i;
        if (idx < 0) {
            for (int k = 0; k < 10; ++k) r[k] = 0.0;
            r[9] = -1.0;
            continue;
        }
        v3d p, nrm;
        int ff;
        hit_record64(sph + 4 * idx, t, o, d, &p, &nrm, &ff);
        r[0] = 1.0;
        r[1] = t;
        r[2] = p.x; r[3] = p.y; r[4] = p.z;
        r[5] = nrm.x; r[6] = nrm.y; r[7] = nrm.z;
        r[8] = ff ? 1.0 : 0.0;
        r[9] = (double)idx;
    }
    return 0;
}

/* Camera(width,height).get_ray(u, v) (Camera.h:9-26) */
int or_camera_simple_rays_f64(uint32_t width, uint32_t height, const double *uv, uint32_t n,
                              double *out) {
    if (!uv || !out || width == 0 || height == 0) return -1;
    const double aspect = (double)width / height;
    const double vh = 2.0, vw = aspect * vh, focal = 1.0;
    const v3d origin = d3(0, 0, 0), hor = d3(vw, 0, 0), ver = d3(0, vh, 0);
    /* origin - horizontal/2 - vertical/2 - Vec3(0,0,focal); /2 = *(1/2) */
    const v3d llc = dsub(dsub(dsub(origin, dscale(1.0 / 2, hor)), dscale(1.0 / 2, ver)), d3(0, 0, focal));
    for (uint32_t i = 0; i < n; ++i) {
        const double u = uv[2 * i], v = uv[2 * i + 1];
        const v3d dir = dsub(dadd(dadd(llc, dscale(u, hor)), dscale(v, ver)), origin);
        out[6 * i + 0] = origin.x;
        out[6 * i + 1] = origin.y;
        out[6 * i + 2] = origin.z;
        out[6 * i + 3] = dir.x;
        out[6 * i + 4] = dir.y;
        out[6 * i + 5] = dir.z;
    }
    return 0;
}

typedef struct {
    uint32_t n, depth, spp;
    double *sph; /* 4 per sphere: c.xyz, r */
    double *mv;
    int *mt;
} scene64;

static void pixel64(const scene64 *S, const frame32 *F, uint32_t x, uint32_t y, float out[4],
                    uint64_t *segs) {
    float seed = pixel_seed(F, S->spp, x, y, 0);
    v3d acc = d3(0, 0, 0);
    uint64_t sg = 0;
    const v3d org = d3(F->org.x, F->org.y, F->org.z), hor = d3(F->hor.x, F->hor.y, F->hor.z);
    const v3d ver = d3(F->ver.x, F->ver.y, F->ver.z), llc = d3(F->llc.x, F->llc.y, F->llc.z);
    for (uint32_t s = 0; s < S->spp && S->depth > 0; ++s) {
        if (F->rng_mode == 1u) seed = pixel_seed(F, S->spp, x, y, s);
        float h0, h1, g0, g1;
        hash2(&seed, &h0, &h1);
        const double u = ((double)x + h0 * 1.1) / ((double)F->img_w - 1.0);
        hash2(&seed, &g0, &g1);
        const double v = ((double)y + g1 * 1.1) / ((double)F->img_h - 1.0);
        v3d o = org;
        v3d d = dsub(dadd(dadd(llc, dscale(u, hor)), dscale(v, ver)), org);
        if (F->lens_r > 0.0f) {
            float h0d, h1d;
            hash2(&seed, &h0d, &h1d);
            const double rr = sqrt((double)h0d), ph = h1d * 6.28318530718;
            const double rx = F->lens_r * rr * sin(ph), ry = F->lens_r * rr * cos(ph);
            const v3d off = d3(rx * F->lu.x + ry * F->lv.x, rx * F->lu.y + ry * F->lv.y, rx * F->lu.z + ry * F->lv.z);
            o = dadd(o, off);
            d = dsub(d, off);
        }
        v3d col = d3(1, 1, 1);
        for (uint32_t k = 0; k < S->depth; ++k) {
            double t;
            const int idx = hit_world64(S->sph, S->n, o, d, 0.001, INFINITY, &t);
            ++sg;
            if (idx >= 0) {
                v3d p, nrm, dir;
                int ff;
                hit_record64(S->sph + 4 * idx, t, o, d, &p, &nrm, &ff);
                const int mt = S->mt[idx];
                const double *mv = S->mv + 4 * idx;
                if (mt == 0 || mt == 1) {
                    const v3f hh = hash3(&seed);
                    const double hx = hh.x * 2.0 - 1.0, phi = hh.y * 6.28318530718;
                    const double r = pow(hh.z, 1.0 / 3.0), sq = sqrt(1.0 - hx * hx);
                    const v3d rr = d3(r * sq * sin(phi), r * sq * cos(phi), r * hx);
                    if (mt == 0) {
                        v3d v = dsub(dadd(dadd(p, nrm), rr), p);
                        if ((F->flags & 1u) && fabs(v.x) < 1e-9 && fabs(v.y) < 1e-9 && fabs(v.z) < 1e-9) v = nrm;
                        dir = dunit(v);
                    } else {
                        const v3d refl = dsub(d, dscale(2.0 * ddot(d, nrm), nrm));
                        dir = dunit(dadd(refl, dscale(mv[3], rr)));
                    }
                    col = dmul(col, d3(mv[0], mv[1], mv[2]));
                } else if (mt == 2) {
                    const double ratio = ff ? (1.0 / mv[3]) : mv[3];
                    const v3d ud = dunit(d);
                    const double cosine = fmin(ddot(dneg(ud), nrm), 1.0);
                    const double sine = sqrt(1.0 - cosine * cosine);
                    const int cant = ratio * sine > 1.0;
                    double r0 = (1 - ratio) / (1 + ratio);
                    r0 = r0 * r0;
                    const double refl = r0 + (1 - r0) * pow(1 - cosine, 5);
                    const float h = hash1(&seed);
                    if (cant || refl > h) {
                        dir = dsub(ud, dscale(2.0 * ddot(ud, nrm), nrm));
                    } else {
                        const double ct = fmin(ddot(dneg(ud), nrm), 1.0);
                        const v3d rp = dscale(ratio, dadd(ud, dscale(ct, nrm)));
                        dir = dadd(rp, dscale(-sqrt(fabs(1.0 - dlen2(rp))), nrm));
                    }
                } else {
                    break;
                }
                o = p;
                d = dir;
            } else {
                const v3d ud = dunit(d);
                const double tt = 0.5 * (ud.y + 1.0);
                acc = dadd(acc, dmul(col, d3((1 - tt) + tt * 0.5, (1 - tt) + tt * 0.7, (1 - tt) + tt)));
                break;
            }
        }
    }
    out[0] = (float)pow(acc.x / S->spp, 1.0 / 2.2);
    out[1] = (float)pow(acc.y / S->spp, 1.0 / 2.2);
    out[2] = (float)pow(acc.z / S->spp, 1.0 / 2.2);
    out[3] = 1.0f;
    *segs += sg;
}

/* ------------------------------------------------------------------------ */
/* threaded row renderer                                                     */
typedef struct {
    const scene32 *s32;
    const scene64 *s64;
    const frame32 *F;
    const uint32_t *ys;
    uint32_t nys;
    float *out;
    uint32_t next; /* atomic row cursor */
    uint64_t segs; /* atomic */
} job_t;

static void *worker(void *arg) {
    job_t *J = (job_t *)arg;
    const uint32_t W = J->F->width;
    uint64_t segs = 0;
    for (;;) {
        const uint32_t r = __atomic_fetch_add(&J->next, 1u, __ATOMIC_RELAXED);
        if (r >= J->nys) break;
        const uint32_t y = J->ys[r];
        float *row = J->out + (size_t)r * W * 4;
        for (uint32_t x = 0; x < W; ++x) {
            if (J->s32)
                pixel32(J->s32, J->F, x, y, row + 4 * x, &segs);
            else
                pixel64(J->s64, J->F, x, y, row + 4 * x, &segs);
        }
    }
    __atomic_fetch_add(&J->segs, segs, __ATOMIC_RELAXED);
    return NULL;
}

static int render_rows_impl(const or_world *w, const or_frame *f, const uint32_t *ys, uint32_t nys,
                            float *out, int nthreads, int precision, uint64_t *segments, int linear);

int or_render_rows(const or_world *w, const or_frame *f, const uint32_t *ys, uint32_t nys,
                   float *out, int nthreads, int precision, uint64_t *segments) {
    return render_rows_impl(w, f, ys, nys, out, nthreads, precision, segments, 0);
}

int or_render_rows_linear(const or_world *w, const or_frame *f, const uint32_t *ys, uint32_t nys,
                          float *out, int nthreads, uint64_t *segments) {
    return render_rows_impl(w, f, ys, nys, out, nthreads, 32, segments, 1);
}

static int render_rows_impl(const or_world *w, const or_frame *f, const uint32_t *ys, uint32_t nys,
                            float *out, int nthreads, int precision, uint64_t *segments, int linear) {
    if (!w || !f || (nys && (!ys || !out)) || nthreads < 1) return -1;
    if (precision != 32 && precision != 64) return -1;
    frame32 F;
    F.org = v3(f->origin[0], f->origin[1], f->origin[2]);
    F.hor = v3(f->horizontal[0], f->horizontal[1], f->horizontal[2]);
    F.ver = v3(f->vertical[0], f->vertical[1], f->vertical[2]);
    F.llc = v3(f->lower_left[0], f->lower_left[1], f->lower_left[2]);
    F.img_w = f->img_w;
    F.img_h = f->img_h;
    F.width = f->width;
    F.rng_mode = f->rng_mode;
    F.frame_index = f->frame_index;
    F.flags = f->flags;
    F.lu = v3(f->lens_u[0], f->lens_u[1], f->lens_u[2]);
    F.lv = v3(f->lens_v[0], f->lens_v[1], f->lens_v[2]);
    F.lens_r = f->lens_u[3];
    F.linear = linear;
    scene32 S32;
    scene64 S64;
    memset(&S64, 0, sizeof(S64));
    int rc = 0;
    if (precision == 32) {
        if (scene32_init(&S32, w)) {
            scene32_free(&S32);
            return -1;
        }
    } else {
        const uint32_t n = w->count;
        S64.n = n;
        S64.depth = w->depth;
        S64.spp = w->spp;
        S64.sph = malloc((n ? n : 1) * 4 * sizeof(double));
        S64.mv = malloc((n ? n : 1) * 4 * sizeof(double));
        S64.mt = malloc((n ? n : 1) * sizeof(int));
        if (!S64.sph || !S64.mv || !S64.mt) rc = -1;
        for (uint32_t i = 0; i < n && !rc; ++i) {
            for (int k = 0; k < 4; ++k) {
                S64.sph[4 * i + k] = w->spheres[4 * i + k];
                S64.mv[4 * i + k] = w->mat_values[4 * i + k];
            }
            const float t = w->mat_types[i];
            S64.mt[i] = (t == 0.0f) ? 0 : (t == 1.0f) ? 1 : (t == 2.0f) ? 2 : 3;
        }
    }
    if (!rc) {
        job_t J;
        memset(&J, 0, sizeof(J));
        J.s32 = precision == 32 ? &S32 : NULL;
        J.s64 = precision == 64 ? &S64 : NULL;
        J.F = &F;
        J.ys = ys;
        J.nys = nys;
        J.out = out;
        if (nthreads == 1) {
            worker(&J);
        } else {
            pthread_t *th = malloc(sizeof(pthread_t) * (size_t)nthreads);
            int started = 0;
            for (int t = 0; th && t < nthreads; ++t)
                if (pthread_create(&th[t], NULL, worker, &J) == 0) ++started;
            if (!th || started == 0) worker(&J);
            for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
            free(th);
        }
        if (segments) *segments = J.segs;
    }
    if (precision == 32) scene32_free(&S32);
    free(S64.sph);
    free(S64.mv);
    free(S64.mt);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* producers                                                                 */
typedef struct {
    uint32_t state;
} msvc_rand;
static inline float msvc_random(msvc_rand *r) { /* DxCSApp.cpp:6-9 */
    r->state = r->state * 214013u + 2531011u;
    return (float)((r->state >> 16) & 0x7fffu) / 32767.0f;
}
static int put(float *sph, float *mt, float *mv, uint32_t cap, uint32_t *cnt, float cx, float cy,
               float cz, float r, float type, float a0, float a1, float a2, float a3) {
    if (*cnt >= cap) return 0;
    const uint32_t i = (*cnt)++;
    sph[4 * i] = cx; sph[4 * i + 1] = cy; sph[4 * i + 2] = cz; sph[4 * i + 3] = r;
    mt[i] = type;
    mv[4 * i] = a0; mv[4 * i + 1] = a1; mv[4 * i + 2] = a2; mv[4 * i + 3] = a3;
    return 1;
}

int or_random_world(int32_t ext, uint32_t cap, float *sph, float *mt, float *mv, uint32_t *count) {
    if (!sph || !mt || !mv || !count || ext < 0) return -1;
    msvc_rand R = {1u};
    uint32_t n = 0;
    put(sph, mt, mv, cap, &n, 0.0f, -1000.0f, 0.0f, 1000.0f, 0.0f, 0.5f, 0.5f, 0.5f, 1.0f);
    put(sph, mt, mv, cap, &n, 0.0f, 1.0f, 0.0f, 1.0f, 2.0f, 0.0f, 0.0f, 0.0f, 1.5f);
    put(sph, mt, mv, cap, &n, -4.0f, 1.0f, 0.0f, 1.0f, 0.0f, 0.4f, 0.2f, 0.1f, 1.0f);
    put(sph, mt, mv, cap, &n, 4.0f, 1.0f, 0.0f, 1.0f, 1.0f, 0.7f, 0.6f, 0.5f, 0.0f);
    for (int a = -ext; a < ext && n < cap; ++a) {
        for (int b = -ext; b < ext && n < cap; ++b) {
            const float choice = msvc_random(&R);
            const float cx = (float)((double)a + 0.9 * (double)msvc_random(&R));
            const float cz = (float)((double)b + 0.9 * (double)msvc_random(&R));
            const double dx = (double)cx - 4.0, dz = (double)cz;
            if (sqrt(dx * dx + dz * dz) > 0.9) {
                if ((double)choice < 0.8) {
                    float al[6];
                    for (int k = 0; k < 6; ++k) al[k] = msvc_random(&R);
                    put(sph, mt, mv, cap, &n, cx, 0.2f, cz, 0.2f, 0.0f, al[0] * al[1], al[2] * al[3],
                        al[4] * al[5], 0.0f);
                } else if ((double)choice < 0.95) {
                    float al[3];
                    for (int k = 0; k < 3; ++k) al[k] = msvc_random(&R) / 2.0f + 1.0f;
                    put(sph, mt, mv, cap, &n, cx, 0.2f, cz, 0.2f, 1.0f, al[0], al[1], al[2], 0.0f);
                } else {
                    put(sph, mt, mv, cap, &n, cx, 0.2f, cz, 0.2f, 2.0f, 0.0f, 0.0f, 0.0f, 1.5f);
                }
            }
        }
    }
    *count = n;
    return 0;
}

int or_test_world(float *sph, float *mt, float *mv, uint32_t *count) {
    if (!sph || !mt || !mv || !count) return -1;
    uint32_t n = 0;
    put(sph, mt, mv, 4, &n, 0.0f, -1000.5f, -1.0f, 1000.0f, 0.0f, 0.5f, 0.5f, 0.5f, 1.0f);
    put(sph, mt, mv, 4, &n, 0.0f, 0.0f, -1.0f, 0.5f, 0.0f, 0.2f, 0.4f, 0.8f, 1.0f);
    put(sph, mt, mv, 4, &n, 1.0f, 0.0f, -1.0f, 0.5f, 1.0f, 0.8f, 0.4f, 0.2f, 0.0f);
    put(sph, mt, mv, 4, &n, -1.0f, 0.0f, -1.0f, 0.5f, 2.0f, 0.5f, 0.5f, 0.5f, 1.5f);
    *count = n;
    return 0;
}

int or_camera_look_at(const float from[3], const float at[3], const float vup[3], float vfov,
                      float aspect, float focus_dist, uint32_t width, uint32_t height,
                      or_frame *out) {
    if (!from || !at || !vup || !out || !(aspect > 0.0f)) return -1;
    const v3f f = v3(from[0], from[1], from[2]), a = v3(at[0], at[1], at[2]);
    const v3f up = v3(vup[0], vup[1], vup[2]);
    const v3f fa = vsub(f, a);
    if (!(focus_dist > 0.0f)) focus_dist = sqrtf(vdot(fa, fa));
    const float theta = (float)((double)vfov * 3.1415926535897932385 / 180.0);
    const float h = tanf(theta / 2.0f);
    const float view_h = (float)(2.0 * (double)h);
    const float view_w = aspect * view_h;
    const float lw = sqrtf(vdot(fa, fa));
    const v3f w = v3(fa.x / lw, fa.y / lw, fa.z / lw);
    const v3f cu = v3(up.y * w.z - up.z * w.y, up.z * w.x - up.x * w.z, up.x * w.y - up.y * w.x);
    const float lu = sqrtf(vdot(cu, cu));
    const v3f u = v3(cu.x / lu, cu.y / lu, cu.z / lu);
    const v3f v = v3(w.y * u.z - w.z * u.y, w.z * u.x - w.x * u.z, w.x * u.y - w.y * u.x);
    const float sh = focus_dist * view_w, sv = focus_dist * view_h;
    const v3f H = v3(u.x * sh, u.y * sh, u.z * sh);
    const v3f V = v3(v.x * sv, v.y * sv, v.z * sv);
    const v3f L = vsub(vsub(vsub(f, v3(H.x * 0.5f, H.y * 0.5f, H.z * 0.5f)),
                            v3(V.x * 0.5f, V.y * 0.5f, V.z * 0.5f)),
                       v3(w.x * focus_dist, w.y * focus_dist, w.z * focus_dist));
    memset(out, 0, sizeof(*out));
    out->origin[0] = f.x; out->origin[1] = f.y; out->origin[2] = f.z; out->origin[3] = 1.0f;
    out->horizontal[0] = H.x; out->horizontal[1] = H.y; out->horizontal[2] = H.z;
    out->vertical[0] = V.x; out->vertical[1] = V.y; out->vertical[2] = V.z;
    out->lower_left[0] = L.x; out->lower_left[1] = L.y; out->lower_left[2] = L.z; out->lower_left[3] = 1.0f;
    out->lens_u[0] = u.x; out->lens_u[1] = u.y; out->lens_u[2] = u.z;
    out->lens_v[0] = v.x; out->lens_v[1] = v.y; out->lens_v[2] = v.z;
    out->img_w = (float)width;
    out->img_h = (float)width / aspect;
    out->width = width;
    out->height = height;
    return 0;
}

int or_camera_simple(uint32_t width, uint32_t height, or_frame *out) {
    if (!out || width == 0 || height == 0) return -1;
    const double aspect = (double)width / height, vh = 2.0, vw = aspect * vh;
    memset(out, 0, sizeof(*out));
    out->origin[3] = 1.0f;
    out->horizontal[0] = (float)vw;
    out->vertical[1] = (float)vh;
    out->lower_left[0] = (float)(0.0 - vw / 2);
    out->lower_left[1] = (float)(0.0 - vh / 2);
    out->lower_left[2] = -1.0f;
    out->lower_left[3] = 1.0f;
    out->lens_u[0] = 1.0f;
    out->lens_v[1] = 1.0f;
    out->img_w = (float)width;
    out->img_h = (float)height;
    out->width = width;
    out->height = height;
    return 0;
}
