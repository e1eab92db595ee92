// rtx_seed.h — the chain RNG's seed after n hash steps, without taking them.
//
// The reference's RNG state is one float (ShaderCompute.hlsl:295) and every
// hash call advances it by two fp32 additions of the literal 0.1
// (`float2(seed += 0.1, seed += 0.1)`, :30-48). A pixel's samples share that
// chain: sample k+1 starts where sample k's hash calls left the seed, so the
// samples of one pixel cannot run in parallel. The speculative chain
//  traces the sample that STARTS at every possible position of
// a heavy pixel's seed sequence in parallel and then follows the chain by
// lookups; a lane tracing position k needs s_k = the seed after 2k additions,
// which seed_advance computes in O(binades) instead of O(k) steps.
//
// Exactness. For s >= 0.25 in the binade [2^E, 2^(E+1)) with ulp u, and a
// step that stays below 2^(E+1) (s + 0.1 < 2^(E+1)), fl(s + 0.1f) = s + r_E
// with r_E = 0.1f rounded to a multiple of u: round-to-nearest of t + A for a
// multiple t of u only depends on A mod u, and A = 0.1f = 13421773 * 2^-27
// (odd mantissa) is a tie (A mod u = u/2) only for u = 2^-26, the binade
// [1/8, 1/4) — below 0.25 the function takes literal steps. So within a binade
// the sequence is s + j * r_E, exactly, until the step that crosses the binade
// top, which is taken literally. All arithmetic is exact in double (values
// are multiples of u <= 2^(E+1): 24 significant bits; j < 2^25).
// tests/seed_check.cpp compares it with the literal additions on the CPU and
// test_gpu_parity.py::test_seed_advance_matches_literal_steps on the GPU.
// Inputs below 0 take literal steps (the product's seeds are h / 2^32 >= 0
// and only grow); NaN and +inf are fixed points of the addition.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define RTX_SEED_HD __host__ __device__ __forceinline__
#else
#define RTX_SEED_HD static inline
#endif

namespace rtx {

RTX_SEED_HD float seed_advance(float s, uint32_t n) {
    const float A = 0.1f;
    if (!(s == s) || s == __builtin_inff()) return s;  // NaN, +inf: s + 0.1 == s
    while (n != 0u && !(s >= 0.25f)) {  // ties below 0.25; negative seeds (not produced) step literally
        s = s + A;
        --n;
    }
    while (n != 0u) {
        uint32_t bits;
        __builtin_memcpy(&bits, &s, 4);
        const int E = (int)((bits >> 23) & 255u) - 127;  // s >= 0.25: normal
        const double top = __builtin_ldexp(1.0, E + 1);
        const double D = top - (double)s - (double)A;  // exact: the room before a step would cross `top`
        const float s1 = s + A;
        if (D <= 0.0) {  // this step leaves the binade: take it literally
            s = s1;
            --n;
            continue;
        }
        const double r = (double)s1 - (double)s;  // the binade's step (exact)
        if (r == 0.0) return s;                    // u > 0.2: the seed no longer moves
        // j steps of r are exact while each step starts below top - A:
        // (j - 1) * r < D; the largest such j
        uint64_t j = (uint64_t)__builtin_ceil(D / r);
        while (j > 1u && (double)(j - 1u) * r >= D) --j;
        while ((double)j * r < D) ++j;
        if (j > n) j = n;
        s = (float)((double)s + (double)j * r);
        n -= (uint32_t)j;
    }
    return s;
}

}  // namespace rtx
