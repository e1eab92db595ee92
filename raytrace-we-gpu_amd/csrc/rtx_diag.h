// rtx_diag.h — diagnostic hooks of the render kernels. They are compiled in
// only by the Makefile's variant builds (prof: per-section clock sums and
// scan/resolve event counts, tools/section_prof.py; ptime: per-pixel start /
// end times, tools/pixel_timeline.py; cprof: per-section clocks of tier-1
// coop segments, tools/coop_prof.py; rays: a sample of lane-mode wave
// iterations' rays, tools/ray_sample.py). In the product build every hook below
// is empty and the per-wave Diag state has no members, so the hot loops'
// text carries one call per hook and no diagnostic code.
#pragma once

#include "rtx_internal.h"

#ifndef RTX_DIAG_PROF  // per-section clock sums into the wave_times buffer
#define RTX_DIAG_PROF 0
#endif
#ifndef RTX_DIAG_PIXEL  // per-pixel (start | mode, end) s_memrealtime into wave_times[2*gid..]
#define RTX_DIAG_PIXEL 0
#endif
#ifndef RTX_DIAG_COOP  // per-section clocks of tier-N (N = its value) coop segments into wave_times[0..7]
#define RTX_DIAG_COOP 0
#endif
#ifndef RTX_DIAG_RAYS  // every RTX_DIAG_RAYS-th lane-mode wave iteration's rays into wave_times
#define RTX_DIAG_RAYS 0
#endif

namespace rtx {
namespace {

#if RTX_DIAG_PROF
// Event counters, one set per wave in LDS: [0] blocks scanned [1] blocks
// recorded (some lane had a candidate) [2] resolve iterations [3] lanes
// falling back to the in-order scan [4] candidate entries (lanes) [5] candidate
// spheres (the resolve's work, summed over the wave's lanes) [6] blocks of the
// culled scan whose bound some lane passed
__device__ __forceinline__ uint32_t *diag_slots() {
    __shared__ uint32_t s[4][8];
    return s[(threadIdx.x / 64) & 3u];
}
__device__ __forceinline__ void diag_add(int k, uint32_t v) {
    const uint64_t m = __ballot(1);
    if ((int)(threadIdx.x & 63u) == __ffsll((long long)m) - 1) diag_slots()[k] += v;
}
#define RTX_DIAG_ADD(k, v) diag_add(k, v)
#else
#define RTX_DIAG_ADD(k, v)
#endif

// Coop section clocks (groups_impl / groups_sm): cp = the wave's tier-N
// counters or null, tq = the running timestamp.
#define RTX_CP(k)                                                   \
    if (RTX_DIAG_COOP && cp) {                                      \
        const unsigned long long tn = __builtin_readcyclecounter(); \
        cp[k] += tn - *tq;                                          \
        *tq = tn;                                                   \
    }

// Per-wave state of the section profile (prof: [0] refill [1] hit_world
// [2] shade [3] tail mode clocks [4] iterations [5] tail iterations [6]
// active lanes summed over iterations) and of the coop profile (cprof:
// [0] ray exchange + line setup [1] scan + resolve [2] reduction [3] shade
// [4] loop between segments [5] segments).
struct Diag {
#if RTX_DIAG_RAYS
    uint32_t rit = 0;
#endif
#if RTX_DIAG_PROF
    unsigned long long pr[7] = {0, 0, 0, 0, 0, 0, 0};
    unsigned long long tq = 0;
#endif
#if RTX_DIAG_COOP
    unsigned long long cpa[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long ctq = 0;
    bool was_coop = false;
#endif
    __device__ __forceinline__ void begin() {
#if RTX_DIAG_PROF
        if ((threadIdx.x & 63u) == 0u)
            for (int k = 0; k < 8; ++k) diag_slots()[k] = 0u;
        tq = __builtin_readcyclecounter();
#endif
#if RTX_DIAG_COOP
        ctq = __builtin_readcyclecounter();
#endif
    }
    // close section k (prof)
    __device__ __forceinline__ void section(int k) {
#if RTX_DIAG_PROF
        const unsigned long long tn = __builtin_readcyclecounter();
        pr[k] += tn - tq;
        tq = tn;
#else
        (void)k;
#endif
    }
    __device__ __forceinline__ void iteration(uint64_t act) {
#if RTX_DIAG_PROF
        pr[4]++;
        pr[6] += __popcll(act);
#else
        (void)act;
#endif
    }
    __device__ __forceinline__ void tail_iteration() {
#if RTX_DIAG_PROF
        pr[5]++;
#endif
    }
    // a coop segment of a wave of `tier` starts: the counters to pass to
    // hit_world_groups (null unless cprof profiles this tier)
    __device__ __forceinline__ unsigned long long *coop_begin(uint32_t tier, unsigned long long *&tqp) {
#if RTX_DIAG_COOP
        tqp = &ctq;
        if (tier != (uint32_t)RTX_DIAG_COOP) return nullptr;
        const unsigned long long tn = __builtin_readcyclecounter();
        if (was_coop) cpa[4] += tn - ctq;
        ctq = tn;
        return cpa;  // the coop code counts its segments in cpa[5]
#else
        (void)tier;
        tqp = nullptr;
        return nullptr;
#endif
    }
    __device__ __forceinline__ void coop_end(unsigned long long *cp, uint32_t tier) {
#if RTX_DIAG_COOP
        if (cp) {
            const unsigned long long tn = __builtin_readcyclecounter();
            cpa[3] += tn - ctq;
            ctq = tn;
        }
        was_coop = tier == (uint32_t)RTX_DIAG_COOP;
#else
        (void)cp;
        (void)tier;
#endif
    }
    // rays (RTX_DIAG_RAYS): a sampled lane-mode iteration appends one record
    // of 64 lanes x 4 words (o.x o.y | o.z d.x | d.y d.z | live, slot) at
    // wave_times[64 + 256 * r], r = wave_times[0]++ (records past the buffer
    // are dropped). Called wave-uniformly.
    __device__ __forceinline__ void rays(const KParams &P, f3 o, f3 d, bool live, uint32_t slot) {
#if RTX_DIAG_RAYS
        if (!P.wave_times) return;
        const uint32_t w = blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u;
        if ((++rit + w * 13u) % (uint32_t)RTX_DIAG_RAYS != 0u) return;
        unsigned long long r = 0;
        if ((threadIdx.x & 63u) == 0u) r = atomicAdd(&P.wave_times[0], 1ull);
        r = __shfl(r, 0, 64);
        const unsigned long long base = 64ull + 256ull * r;
        if (base + 256ull > 2ull * P.wave_cap) return;
        auto pk = [](float a, float b) {
            return ((unsigned long long)__float_as_uint(b) << 32) | __float_as_uint(a);
        };
        unsigned long long *q = P.wave_times + base + 4u * (threadIdx.x & 63u);
        q[0] = pk(o.x, o.y);
        q[1] = pk(o.z, d.x);
        q[2] = pk(d.y, d.z);
        q[3] = ((unsigned long long)slot << 32) | (live ? 1u : 0u);
#else
        (void)P, (void)o, (void)d, (void)live, (void)slot;
#endif
    }
    // the wave's sums into P.wave_times
    __device__ __forceinline__ void finish(const KParams &P) {
#if RTX_DIAG_PROF
        if (P.wave_times && (threadIdx.x & 63u) == 0u) {
            for (int k = 0; k < 7; ++k) atomicAdd(&P.wave_times[k], pr[k]);
            for (int k = 0; k < 7; ++k) atomicAdd(&P.wave_times[8 + k], (unsigned long long)diag_slots()[k]);
        }
#endif
#if RTX_DIAG_COOP
        if (P.wave_times && (threadIdx.x & 63u) == 0u)
            for (int k = 0; k < 6; ++k) atomicAdd(&P.wave_times[k], cpa[k]);
#endif
        (void)P;
    }
};

// ptime: a pixel starts (mode 0 lane queue, 1 tier 1, 2 tier 2) / ends
__device__ __forceinline__ void diag_pixel_start(const KParams &P, uint32_t gid, unsigned long long mode) {
#if RTX_DIAG_PIXEL
    if (P.wave_times && gid < P.wave_cap) P.wave_times[2 * gid] = (__builtin_amdgcn_s_memrealtime() << 2) | mode;
#else
    (void)P;
    (void)gid;
    (void)mode;
#endif
}
__device__ __forceinline__ void diag_pixel_end(const KParams &P, uint32_t gid) {
#if RTX_DIAG_PIXEL
    if (P.wave_times && gid < P.wave_cap) P.wave_times[2 * gid + 1] = __builtin_amdgcn_s_memrealtime();
#else
    (void)P;
    (void)gid;
#endif
}
constexpr bool kDiagAny = RTX_DIAG_PROF || RTX_DIAG_PIXEL || RTX_DIAG_COOP || RTX_DIAG_RAYS;

}  // namespace
}  // namespace rtx
