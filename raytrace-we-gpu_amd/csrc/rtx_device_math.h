// rtx_device_math.h — fp32 arithmetic of the hot path, device side.
//
// Every function here is one clause of the "twin spec" in DESIGN.md §4:
// a fixed sequence of IEEE-754 binary32 operations (add/sub/mul, fmaf,
// correctly rounded div and sqrt, rint, int<->float conversions, bit
// casts). The CPU oracle (oracle/rtx_oracle.c) restates the same sequence
// in C, so GPU and CPU produce identical bits. Two compilation rules make
// that hold: -ffp-contract=off (no fma unless written as fmaf) and no
// fast-math (hipcc's default correctly rounded f32 div/sqrt stay on).
//
// Reference semantics followed (CSVersion/ShaderCompute.hlsl):
//   baseHash :23-28, hash1 :30-34, hash2 :36-41, hash3 :43-48,
//   random_in_unit_sphere :59-66, reflect :76-79, refract :81-88,
//   reflectance :90-97, toGamma :99-103.
// HLSL's sin/cos/pow are driver-defined in D3D; here they are our own
// polynomial restatements (sin/cos: Cody-Waite + minimax, pow: exp2(y*log2 x)
// — the same decomposition D3D hardware uses for pow).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtx {

struct f3 {
    float x, y, z;
};

__device__ __forceinline__ f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 operator-(f3 a) { return f3{-a.x, -a.y, -a.z}; }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ f3 operator*(float s, f3 a) { return f3{s * a.x, s * a.y, s * a.z}; }
// sqrtf, correctly rounded, with the compiler's own correction of the 1-ulp
// v_sqrt_f32 (s +- 1 ulp by the sign of the fma residuals) but without its
// rescaling and class fix-ups where they change nothing: those matter only
// for 0 < x < 2^-96 (the residuals would be denormal), which takes sqrtf.
// x = +-0, +inf, NaN and x < 0 come out of the fast sequence as sqrtf gives
// them (the residuals are NaN or -0 and select nothing).
__device__ __forceinline__ float sqrt_rn(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    float r = fmaf(-sm, s, x) <= 0.0f ? sm : s;
    r = fmaf(-sp, s, x) > 0.0f ? sp : r;
    if (__builtin_expect(x > 0.0f && x < 0x1p-96f, 0)) r = sqrtf(x);
    return r;
}

// dot = (x*x' + y*y') + z*z', three roundings of products, two of sums.
__device__ __forceinline__ float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// normalize(v) = v * (1 / sqrt(dot(v, v)))   (HLSL normalize = v * rsqrt)
__device__ __forceinline__ f3 normalize3(f3 v) {
    const float inv = 1.0f / sqrt_rn(dot3(v, v));
    return inv * v;
}

// ---- RNG (ShaderCompute.hlsl:23-48) -------------------------------------
// baseHash(uint2 p): p = 1103515245*((p>>1)^p.yx); h = 1103515245*(p.x^(p.y>>3)); h^(h>>16)
__device__ __forceinline__ uint32_t base_hash(uint32_t px, uint32_t py) {
    const uint32_t qx = 1103515245u * ((px >> 1) ^ py);
    const uint32_t qy = 1103515245u * ((py >> 1) ^ px);
    const uint32_t h = 1103515245u * (qx ^ (qy >> 3));
    return h ^ (h >> 16);
}
// float2(seed += 0.1, seed += 0.1), evaluated left to right, fp32 literal 0.1.
__device__ __forceinline__ uint32_t hash_step(float &seed) {
    seed = seed + 0.1f;
    const float a = seed;
    seed = seed + 0.1f;
    const float b = seed;
    return base_hash(__float_as_uint(a), __float_as_uint(b));
}
__device__ __forceinline__ float hash1(float &seed) {
    const uint32_t n = hash_step(seed);
    return (float)n / 4294967296.0f;  // float(0xffffffffU) == 2^32
}
__device__ __forceinline__ void hash2(float &seed, float &h0, float &h1) {
    const uint32_t n = hash_step(seed);
    h0 = (float)(n & 0x7fffffffu) / 2147483648.0f;  // float(0x7fffffff) == 2^31
    h1 = (float)((n * 48271u) & 0x7fffffffu) / 2147483648.0f;
}
__device__ __forceinline__ f3 hash3(float &seed) {
    const uint32_t n = hash_step(seed);
    return f3{(float)(n & 0x7fffffffu) / 2147483648.0f,
              (float)((n * 16807u) & 0x7fffffffu) / 2147483648.0f,
              (float)((n * 48271u) & 0x7fffffffu) / 2147483648.0f};
}

// ---- sin/cos -------------------------------------------------------------
// q = rint(x * 2/pi); r = x - q*pi/2 (two-constant Cody-Waite, fmaf);
// sin/cos of r by degree-7/8 minimax polynomials; quadrant swap.
__device__ __forceinline__ void sincos_rt(float x, float &s, float &c) {
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
    s = (n == 0) ? S : (n == 1) ? C : (n == 2) ? -S : -C;
    c = (n == 0) ? C : (n == 1) ? -S : (n == 2) ? -C : S;
}

// ---- log2 / exp2 / pow -----------------------------------------------------
// log2(x), x > 0 finite: x = m 2^e, m in [sqrt(1/2), sqrt(2)];
// ln(m) = 2 atanh(s), s = (m-1)/(m+1), odd series to s^9.
__device__ __forceinline__ float log2_rt(float x) {
    int e = 0;
    if (x < 1.17549435e-38f) {  // subnormal: scale by 2^23 (exact)
        x = x * 8388608.0f;
        e = -23;
    }
    const uint32_t b = __float_as_uint(x);
    e += (int)(b >> 23) - 127;
    float m = __uint_as_float((b & 0x007fffffu) | 0x3f800000u);
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
// exp2(t): n = rint(t), r = t - n (exact), 2^r by degree-7 Taylor, scale by 2^n.
__device__ __forceinline__ float exp2_rt(float t) {
    if (!(t == t)) return t;
    if (t >= 128.0f) return __uint_as_float(0x7f800000u);
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
        p = p * 5.42101086e-20f;  // 2^-64, exact
        n += 64;
    }
    if (n > 127) {
        p = p * 2.0f;
        n -= 1;
    }
    return p * __uint_as_float((uint32_t)(n + 127) << 23);
}
// pow(x, y) for y > 0 (the reference's exponents 1/3, 1/2.2):
// NaN -> NaN, x < 0 -> NaN, 0 -> 0, +inf -> +inf, else exp2(y * log2(x)).
__device__ __forceinline__ float pow_rt(float x, float y) {
    if (!(x == x)) return x;
    if (x < 0.0f) return __uint_as_float(0x7fc00000u);
    if (x == 0.0f) return 0.0f;
    if (x == __uint_as_float(0x7f800000u)) return x;
    return exp2_rt(y * log2_rt(x));
}

// ---- sampling / BRDF helpers ---------------------------------------------
// random_in_unit_sphere (ShaderCompute.hlsl:59-66):
//   h = hash3 * (2, 2pi, 1) - (1, 0, 0); r = pow(h.z, 1/3);
//   return r * (sqrt(1 - h.x^2) * (sin h.y, cos h.y), h.x)
__device__ __forceinline__ f3 random_in_unit_sphere(float &seed) {
    const f3 h = hash3(seed);
    const float hx = h.x * 2.0f - 1.0f;
    const float phi = h.y * 6.28318530718f;
    const float r = pow_rt(h.z, 0.333333333f);
    const float sq = sqrt_rn(1.0f - hx * hx);
    float sn, cs;
    sincos_rt(phi, sn, cs);
    return f3{r * (sq * sn), r * (sq * cs), r * hx};
}
// random_in_unit_disk (ShaderCompute.hlsl:50-57; unused by the reference,
// used by the thin-lens extension): h = hash2 * (1, 2pi); r = sqrt(h.x);
// r * (sin h.y, cos h.y). Returned as (x, y, 0).
__device__ __forceinline__ f3 random_in_unit_disk(float &seed) {
    float h0, h1;
    hash2(seed, h0, h1);
    const float phi = h1 * 6.28318530718f;
    const float r = sqrt_rn(h0 * 1.0f);
    float sn, cs;
    sincos_rt(phi, sn, cs);
    return f3{r * sn, r * cs, 0.0f};
}
// reflect(v, n) = v - 2*dot(v,n)*n   (:76-79)
__device__ __forceinline__ f3 reflect3(f3 v, f3 n) {
    const float k = 2.0f * dot3(v, n);
    return v - k * n;
}
// refract (:81-88); length(x)*length(x) kept literally.
__device__ __forceinline__ f3 refract3(f3 uv, f3 n, float ratio) {
    const float cos_theta = fminf(dot3(-uv, n), 1.0f);
    const f3 r_perp = ratio * (uv + cos_theta * n);
    const float lp = sqrt_rn(dot3(r_perp, r_perp));
    const float k = -sqrt_rn(fabsf(1.0f - lp * lp));
    return r_perp + k * n;
}
// reflectance (:90-97); pow(1-cos, 5) as x^2 * x^2 * x.
__device__ __forceinline__ float reflectance(float cosine, float ref_idx) {
    float r0 = (1.0f - ref_idx) / (1.0f + ref_idx);
    r0 = r0 * r0;
    const float x = 1.0f - cosine;
    const float x2 = x * x;
    const float x5 = (x2 * x2) * x;
    return r0 + (1.0f - r0) * x5;
}
// toGamma (:99-103): pow(c, 1/2.2); 1/2.2 folded in double then rounded.
__device__ __forceinline__ float to_gamma(float c) { return pow_rt(c, 0.454545454545f); }

}  // namespace rtx
