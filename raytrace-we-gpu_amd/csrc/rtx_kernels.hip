// rtx_kernels.hip — the hot path: CSMain / sample_color / hit_world /
// hit_sphere / scatter of CSVersion/ShaderCompute.hlsl:155-315 as a CDNA4
// (gfx950, wave64) HIP kernel.
//
// Design:
//  * chain RNG (the reference, ShaderCompute.hlsl:295,304-309): one lane per
//    pixel; the spp x depth double loop is flattened into a per-lane state
//    machine (a lane whose path ends starts its pixel's next sample in the
//    same iteration), persistent lanes pull pixels from a cost-ordered queue,
//    and the heaviest pixels are traced by groups of lanes (k_render);
//  * per-sample RNG (rtx_frame.rng_mode 1): one lane per (pixel, sample)
//    (k_render_ps): samples are independent, so a wave's lanes trace
//    consecutive samples of a batch of pixels and fold each pixel's sample
//    colours in sample order afterwards;
//  * hit_world is a line-distance prefiltered scan over the sphere array
//    (scalar loads of AoSoA-8 blocks, packed-fp32 pairs, one max + ballot
//    per 8 spheres = the wave-level early-out on all-miss), then the
//    flagged spheres are resolved with the reference's own ops
//    (Hittable_list.cpp:3-20 / ShaderCompute.hlsl:188-205);
//  * the hit record (p, normal, front_face, material) is built once per
//    segment for the winning sphere, not for every accepted candidate —
//    identical values, because the reference's final record is the last
//    accepted one.
// Measured-and-rejected variants (LDS-resident spheres, pre-prefilter scans,
// ...) are in git history and DESIGN.md §7.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>

#include "rtx_device_math.h"
#include "rtx_diag.h"
#include "rtx_internal.h"
#include "rtx_prefilter.h"

// The device code is written for gfx950 only: its wave64 DPP/permlane
// exchanges, the s_waitcnt encoding of agent_store_order and the cross-XCD
// promotion hand-off rely on that target's behaviour.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "rtx_kernels.hip targets gfx950 (MI355X) only"
#endif

namespace rtx {

namespace {

constexpr float kTMin = 0.001f;  // hit_world(cur_ray, 0.001, 1.#INF, h), :262

struct FrameVals {
    f3 org, hor, ver, llc;
    float img_w, img_h;
    f3 lu, lv;
    float lens_r;
};
// The frame constants (camera, image size, lens: the PerFrame cbuffer's
// values) are read where a sample starts, straight from the launch's kernel
// arguments (scalar loads through an opaque kernarg pointer), not held for
// the whole kernel: held, their 21 SGPRs were spilled to VGPR lanes and
// every sample start paid ~18 v_readlane restores in VALU issue slots.
// Every kernel that starts samples takes `const KParams` as its only
// argument, so the kernarg segment begins with it.
struct Frame {};
typedef const __attribute__((address_space(4))) KParams *kparams_cp;
__device__ __forceinline__ FrameVals frame_vals() {
    // opaque (reloaded at each use, never hoisted into live SGPRs): passed
    // through a VGPR by an empty asm (an SGPR-constrained asm in divergent
    // code does not compile), then made uniform again by readfirstlane
    const uint64_t a = (uint64_t)(uintptr_t)__builtin_amdgcn_kernarg_segment_ptr();
    uint32_t lo = (uint32_t)a, hi = (uint32_t)(a >> 32);
    asm volatile("" : "+v"(lo), "+v"(hi));
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
    kparams_cp kp = (kparams_cp)(uintptr_t)(((uint64_t)hi << 32) | lo);
    FrameVals F;
    F.org = mk3(kp->org[0], kp->org[1], kp->org[2]);
    F.hor = mk3(kp->hor[0], kp->hor[1], kp->hor[2]);
    F.ver = mk3(kp->ver[0], kp->ver[1], kp->ver[2]);
    F.llc = mk3(kp->llc[0], kp->llc[1], kp->llc[2]);
    F.img_w = kp->img_w;
    F.img_h = kp->img_h;
    F.lu = mk3(kp->lens_u[0], kp->lens_u[1], kp->lens_u[2]);
    F.lv = mk3(kp->lens_v[0], kp->lens_v[1], kp->lens_v[2]);
    F.lens_r = kp->lens_r;
    return F;
}

// get_ray (ShaderCompute.hlsl:118-127): dir = llc + s*H + t*V - origin.
__device__ __forceinline__ void get_ray(const FrameVals &F, float s, float t, f3 &o, f3 &d) {
    o = F.org;
    d = ((F.llc + s * F.hor) + t * F.ver) - F.org;
}

// CSMain's per-sample jitter (ShaderCompute.hlsl:306-307): two hash2 calls,
// u takes .x of the first, v takes .y of the second.
__device__ __forceinline__ void start_sample(const Frame &, uint32_t x, uint32_t y, float &seed,
                                             f3 &o, f3 &d) {
    const FrameVals F = frame_vals();
    float h0, h1, g0, g1;
    hash2(seed, h0, h1);
    const float u = ((float)x + h0 * 1.1f) / (F.img_w - 1.0f);
    hash2(seed, g0, g1);
    const float v = ((float)y + g1 * 1.1f) / (F.img_h - 1.0f);
    get_ray(F, u, v, o, d);
    if (F.lens_r > 0.0f) {  // thin lens (extension; pinhole ops above unchanged)
        const f3 rd = F.lens_r * random_in_unit_disk(seed);
        const f3 off = rd.x * F.lu + rd.y * F.lv;
        o = o + off;
        d = d - off;
    }
}

// a = |d|^2 (Sphere.cpp:8; HLSL length(d)*length(d), :160), fma form.
__device__ __forceinline__ float dir_len2(f3 d) { return fmaf(d.z, d.z, fmaf(d.y, d.y, d.x * d.x)); }

// Compile-time knobs. The diagnostics are separate builds (rtx_diag.h;
// Makefile variants prof/ptime/cprof); the candidate-list capacities below
// are also set by the stress build. Everything else is a fixed product
// constant.
constexpr int kCoopMax = 32;            // tail mode: a wave with <= this many active lanes traces their rays together
constexpr int kCoopMaxLarge = 8;       // the same above kCoopLds spheres: 32 made C5 1.86 -> 2.40 s (group reads from L2/HBM)
                                        // (8 -> 32 with the sphere-pair coop: parts 1/4/8 -0.8..1.5 ms, R3e)
constexpr uint32_t kHeavy2 = 8;         // tier-2 heavy pixels per group-coop wave
constexpr uint32_t kHeavy1 = 1;         // tier-1 heavy pixels per wave
constexpr double kHeavyAlpha = 2.0;     // tier 2 (small share) iff key > alpha * a lane's share of the summed keys
constexpr double kHeavy1Alpha = 1.7;    // tier 1 iff key > alpha1 * share
constexpr double kHeavy1AlphaSmall = 1.6;   // the same for a small frame share (2.5 until round 4, 4.0 until R4b)
constexpr double kHeavyRhoLow = 2.5;        // "low" share: fewer pixels than this * resident lanes
constexpr double kHeavy1AlphaLow = 1.8;     // tier-1 bar for a low share (2.0 until S6l, 3.0 until round 4, 3.5 until R4b)
constexpr double kHeavyRho = 1.2;       // "small" frame share: fewer pixels than rho * resident lanes
constexpr double kHeavyRho2 = 3.5;      // "medium" frame share: fewer pixels than rho2 * resident lanes
// tier 2 for a medium share: key > this * share (default: none). 1.2 until round 4 (2-way split 37 -> 34 ms
// in r5a-b, before k_trace); with tier 1 in k_trace's pixel groups, tier-2 waves (8 rays, 8 lanes each: ~6x the
// lane time per segment of lane mode) cost more throughput than they save: parts 4 20.4 -> 18.1 ms, parts 2
// 28.4 -> 26.4 without them (profiles/R6p_tier2_sweep_r4_r2.jsonl)
constexpr double kHeavy2AlphaMedium = 1e30;
constexpr double kHeavy2AlphaLarge = 1e30;  // tier 2 for a larger share (default: none)
// k_trace waves (tier 1 outside k_render) as a fraction of the resident waves, by share class.
// Round 4 (k_trace traces 4 tier-1 pixels per wave, the heaviest alone; profiles/R6i_*, R6j_*): with
// the tier-1 bars above and promotion for small / low / medium shares, parts 8 15.0 -> 13.2-13.8 ms,
// parts 4 20.3 -> 19.6-20.0, parts 2 29.6 -> 28.5. The whole frame is no faster with it.
constexpr double kTraceSmall = 0.35, kTraceLow = 0.3, kTraceMedium = 0.15, kTraceLarge = 0.0;
// promotion thresholds (projected further segments; 0: off): a whole frame
// 50.0 -> 46.5 ms at 300-500 (700: 48.5, 1000: 49-51); a 2-way split
// 30.6-31.1 -> 29.6-30.0 ms at 250-500; 4- and 8-way splits: with k_trace's
// pixel groups serving the queue, 300-400 (150: 40 ms at R = 8, the queue
// floods; profiles/R6j_*)
constexpr double kPromSmall = 400.0, kPromLow = 500.0, kPromMedium = 400.0, kPromLarge = 400.0;  // low: 300 until S6l
// scenes without the coop's LDS copy (C5: 100k spheres, a lane-mode segment ~2 ms for the heaviest
// pixels): any part, C5 1,827 -> 1,638 ms at 60 (150: 1,734, 25: 1,657; profiles/R4b_c5_promL.jsonl)
constexpr double kPromBig = 60.0;
// k_trace: tier-1 pixels per wave (1, 2, 4 or 8: rtx_set_schedule), and the key bar (x share)
// above which a pixel is traced alone in its wave nonetheless
constexpr uint32_t kTraceGroup = 4;
constexpr double kTraceSolo = 6.0;
// pre-pass segment cap for row-split parts (0: none; see launch_render)
constexpr uint32_t kCapSplit = 0;
// Lane-mode wave priority from the lanes' projected remaining chains (k_render,
// rtx_schedule.prio_bar*): levels 1/2/3 above these x the mean pixel's
// segments. Against the static hot slots (the queue's first 20 % of the
// resident lanes at priority 3): parts 2 26.4-27.0 -> 25.9-26.0 ms, parts 4
// 18.4-18.9 -> 17.6-17.7, parts 8 13.6 -> 13.2, the whole frame flat (0.75/1.25/2:
// parts 8 slower; 0.25/0.5/1 and 0.35/0.7/1.1: parts 4 slower; profiles/R6t_*, R6u_*)
constexpr double kDynPrio1 = 0.5, kDynPrio2 = 1.0, kDynPrio3 = 1.5;
// Cost pre-pass cap (whole-frame parts only: in a row-split share a capped,
// under-rated key keeps heavy pixels out of the tiers — parts 2/4/8 30/21/15
// -> 34/26/26 ms, profiles/R4h_parts.jsonl): a pixel still tracing after
// this many segments stops, the render traces it from sample 0.
#ifndef RTX_COST_CAP  // small scenes: the stopped pixel's cost is the cap
#define RTX_COST_CAP 16  // C2 44.48 -> 43.72 ms (8: 48.05, 32: 43.99; profiles/R4g_ab_c2_prepass_cap.jsonl)
#endif
#ifndef RTX_COST_CAP_LARGE  // above kScanPfMin spheres (1-spp pre-pass): its cost saturates the key (top bucket)
#define RTX_COST_CAP_LARGE 24  // C5 1,672 -> 1,623 ms (12: 1,659; the cap as the cost: 12 1,666, 6 1,952; R4g, R4h)
#endif
constexpr uint32_t kCostCap = RTX_COST_CAP, kCostCapLarge = RTX_COST_CAP_LARGE;
// The persistent (large-scene) pre-pass stops once at most this fraction of
// its lanes still hold a pixel (pre_stop; 0: runs to the end)
#ifndef RTX_PRE_STOP
#define RTX_PRE_STOP 0.25
#endif
constexpr double kPreStopFrac = RTX_PRE_STOP;
constexpr uint32_t kPrioFracX100 = 20;  // hot-wave priority: prio_slots = this % of the resident lanes
constexpr int kTailPrio = 1;            // wave priority of a normal wave in its coop tail
constexpr uint32_t kRB = 256;           // threads per render workgroup
#ifndef RTX_WAVES_PER_SIMD
#define RTX_WAVES_PER_SIMD 5  // occupancy request for the render kernels: 96 VGPRs (the compiler's own
                              // choice is 100: 4 waves); the few spills (SGPRs to VGPR lanes, ~7 VGPR
                              // dwords to scratch) sit in per-segment and coop code, none in the scan loop
#endif
#define RTX_RENDER_BOUNDS __launch_bounds__(kRB, RTX_WAVES_PER_SIMD)
// The large-scene chain kernels (kPF). With the full scan (RTX_CULL=0: lists
// of RTX_CAND_PF entries and a 1-KiB scan tile per wave, ~34 KB of LDS per
// workgroup) 4 workgroups fit a CU's 160 KB of LDS, i.e. 4 waves per SIMD:
// compiled for 5 they spilled 134 VGPRs for occupancy they never got, for 4
// they had 128. The culled scan (no tile) is latency-bound and its two line
// bases (the stretched one for flat bounds) spill 63 VGPRs at 128: compiled
// for 3 waves (166 VGPRs, no spills) the C5 frame is 2.5 % faster than at 4
// and writes no spill lines (R8u).
#ifndef RTX_WAVES_PER_SIMD_PF
#define RTX_WAVES_PER_SIMD_PF (RTX_CULL ? 3 : 4)
#endif
#define RTX_RENDER_BOUNDS_T(kPF) __launch_bounds__(kRB, (kPF) ? RTX_WAVES_PER_SIMD_PF : RTX_WAVES_PER_SIMD)
// kLin (the linear-scan mode, rtx_set_scan_mode: a large scene without the
// culled layout scans every block through the per-wave LDS tile): 4 waves per
// SIMD, what its LDS allows
#define RTX_RENDER_BOUNDS_T2(kPF, kLin) \
    __launch_bounds__(kRB, (kPF) ? ((kLin) ? 4 : RTX_WAVES_PER_SIMD_PF) : RTX_WAVES_PER_SIMD)
#ifndef RTX_PS_WAVES_PF  // the per-sample kernel's large-scene instance (A/B: 4 = 128 VGPRs)
#define RTX_PS_WAVES_PF RTX_WAVES_PER_SIMD
#endif
#define RTX_PS_BOUNDS_T(kPF) __launch_bounds__(kRB, (kPF) ? RTX_PS_WAVES_PF : RTX_WAVES_PER_SIMD)

// Candidate list: per lane kCand slots in LDS, slot-major
// (slot j of lane t at [j * kRB + t]: conflict-free), plus one dump slot
// that absorbs writes past the end (the lane then falls back, see below).
#ifndef RTX_CAND  // candidate-list capacity per lane (entries; a full list is resolved in rounds)
#define RTX_CAND 12
#endif
constexpr int kCand = RTX_CAND;
constexpr uint32_t kListBytes = (kCand + 1) * kRB * sizeof(uint32_t);  // 13,312 B at 256
static_assert(kListBytes % 16 == 0, "LDS carve must stay 16-byte aligned");
// The kPF kernels (scenes > kScanPfMin, no LDS sphere copy) have the LDS to
// spare for longer lists: fewer scan pauses on large scenes (C5).
#ifndef RTX_CAND_PF
#define RTX_CAND_PF 24
#endif
template <bool kPF>
constexpr uint32_t cand_of() { return kPF ? (uint32_t)RTX_CAND_PF : (uint32_t)kCand; }
template <bool kPF>
constexpr uint32_t list_bytes() { return (cand_of<kPF>() + 1) * kRB * sizeof(uint32_t); }
static_assert(list_bytes<true>() % 16 == 0 && RTX_CAND_PF >= 1, "LDS carve must stay 16-byte aligned");

static_assert(kRB / 64 == 4, "rtx_diag.h keeps 4 waves per workgroup");

// Roots of a sphere whose disc >= 0 (or NaN): near root first, far root if
// the near one is outside [t_min, best] (Sphere.cpp:15-24); strict
// rejection `root < t_min || t_max < root` (ShaderCompute.hlsl:171,174)
// lets a later sphere win an exact tie.
__device__ __forceinline__ void sphere_roots(float hb, float disc, float inv_a, float t_min,
                                             float &best, int &idx, int i) {
    const float sq = sqrt_rn(disc);
    float root = (-hb - sq) * inv_a;
    bool ok = !(root < t_min || best < root);
    if (!ok) {
        root = (-hb + sq) * inv_a;
        ok = !(root < t_min || best < root);
    }
    if (ok) {
        best = root;
        idx = i;
    }
}

// One ray against `nblk` AoSoA-8 blocks (global sphere index of block b's
// first sphere: 8 * (blk0 + b)), in index order; `best` is closest_so_far
// (t_max shrinks on every accepted hit, :196-200). Returns the winning
// index or `idx`. This is the exact fallback of the prefiltered hit_world
// (a lane with a non-finite root redoes the range with it).
//
// Per sphere ("hit_sphere"): oc = o - c; hb = oc.d;
// cc = |oc|^2 - r^2; disc = hb^2 - a*cc. NaN disc falls through like the
// reference's `if (d < 0) return false`. 8 spheres per step: their reads
// issue together and one wave-uniform branch skips the root work when no
// lane's ray line meets any of them (all-miss early out).
template <typename Ptr>
__device__ __forceinline__ int hit_blocks_seq(Ptr soa, uint32_t nblk, uint32_t blk0, f3 o, f3 d,
                                              float a, float inv_a, float t_min, float &best,
                                              int idx) {
    for (uint32_t b = 0; b < nblk; ++b) {
        const Ptr blk = soa + 32 * b;
        float hb[8], disc[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float ocx = o.x - blk[k];
            const float ocy = o.y - blk[8 + k];
            const float ocz = o.z - blk[16 + k];
            hb[k] = fmaf(ocz, d.z, fmaf(ocy, d.y, ocx * d.x));
            const float cc = fmaf(ocz, ocz, fmaf(ocy, ocy, fmaf(ocx, ocx, blk[24 + k])));
            disc[k] = fmaf(hb[k], hb[k], -(a * cc));
        }
        // max() drops a NaN operand: a batch mixing NaN and negative discs
        // needs an fp32 overflow in hb^2 or a*cc, which rtx_upload_world's
        // bound (|scene values| <= 1e15) rules out; an all-NaN batch (NaN
        // ray) yields NaN and is taken, like the reference.
        float m = disc[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) m = fmaxf(m, disc[k]);
        if (__ballot(!(m < 0.0f)) != 0ull) {
            const int g = (int)(8 * (blk0 + b));
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (!(disc[k] < 0.0f)) sphere_roots(hb[k], disc[k], inv_a, t_min, best, idx, g + k);
        }
    }
    return idx;
}

typedef const __attribute__((address_space(4))) float *cfloat_p;  // constant AS: scalar loads

// ---- prefiltered scan (rtx_prefilter.h) -----------------------------------
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v fma2(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }

// Q = R - pu^2 - pv^2 for sphere pairs (v_pk_fma_f32), 8 spheres per step
// from the `pre` blocks, starting at block b; one max + ballot skips a step
// in which no lane's line comes near any of the 8. A lane with flagged
// spheres appends ONE entry per 8-sphere block: local index of the block's
// first sphere | 8-bit mask << 24 (so n_pad <= 2^24, checked at upload).
// Returns the block to resume at: nblk, or earlier once some lane's list is
// full (kCand entries) and must be resolved first (wave-uniform).
//
// kPF (scenes above kScanPfMin): the block's 32 floats are double-buffered in SGPRs. The
// next block's two s_load_dwordx16 are issued (inline asm: the compiler
// otherwise sinks them to the end of the iteration and waits at once) before
// this block's ~25 VALU instructions and waited for after them, so a scalar
// cache miss (every block of a large scene) runs under the block's compute.
// Scalar loads return out of order, so the wait is lgkmcnt(0); it names the
// loaded registers ("+s") so that nothing reads them before it. Every path
// out of the loop body passes a wait, so no load is in flight at exit.
#ifndef RTX_PACK  // kPF scans start where the workgroup's other waves are (hit_world_pre_ld)
#define RTX_PACK 1
#endif
#ifndef RTX_PACK_EVERY
#define RTX_PACK_EVERY 16
#endif
#ifndef RTX_PACK_LAG
#define RTX_PACK_LAG 8
#endif
constexpr uint32_t kPackEvery = RTX_PACK_EVERY;  // blocks between position updates (a power of two)
constexpr uint32_t kPackLag = RTX_PACK_LAG;      // a new scan starts this many blocks behind the last update
typedef float f16v __attribute__((ext_vector_type(16)));
// Issue block p's loads; the "+v" operands (the line's basis, which every
// VALU instruction of the scan reads) keep the compiler from scheduling the
// previous block's compute above the issue.
__device__ __forceinline__ void sload_blk(cfloat_p p, f16v &lo, f16v &hi, f2v &d0, f2v &d1, f2v &d2, f2v &d3,
                                          f2v &d4, f2v &d5, f2v &d6) {
    asm volatile("s_load_dwordx16 %0, %9, 0x0\n\ts_load_dwordx16 %1, %9, 0x40"
                 : "=&s"(lo), "=&s"(hi), "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6)
                 : "s"(p));
}
__device__ __forceinline__ void sload_wait(f16v &lo, f16v &hi) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(lo), "+s"(hi));
}
// One run of blocks [b, end), all flat (kFlat: the 5-op test, k0/k1 = the
// per-ray ku/kv of rtx_prefilter.h line_test_flat) or not (the 7-op test,
// k0/k1 = nou/nov). Returns the block to resume at; `full` when it stopped
// because some lane's list is full.
#ifndef RTX_PF_LDS  // large scenes stream through a per-wave LDS tile of RTX_PF_LDS KiB (below; 0: SGPR double buffer)
#define RTX_PF_LDS 1  // C5 1,880-1,907 -> 1,811-1,847 ms (profiles/R3w_*, R3x_*)
#endif
#ifndef RTX_PF_RING  // A/B: the tile stream as a ring of RTX_PF_RING 1-KiB slots filled by LDS-DMA (0: VGPR staging)
#define RTX_PF_RING 0
#endif
constexpr uint32_t kPfSlots = RTX_PF_RING > RTX_PF_LDS ? RTX_PF_RING : RTX_PF_LDS;
constexpr uint32_t kPfLdsBytes = (kRB / 64) * 64 * 16 * kPfSlots;  // kPfSlots KiB per wave
// LDS-DMA (global_load_lds_dwordx4): lane l's 16 bytes at gsrc land at LDS byte
// address lds_base + 16 l (wave-uniform base, in M0). An asm load is outside
// the compiler's s_waitcnt bookkeeping: the caller counts it with vmcnt. The
// lgkmcnt(0) first: the slot's earlier ds_reads have returned before it is
// overwritten.
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
__device__ __forceinline__ void glds16(const void *gsrc, uint32_t lds_base) {
    unsigned keep;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_base)
                 : "memory");
}
#ifndef RTX_SCAN_LDS  // A/B build: the small-scene scan reads its blocks from the block's LDS copy
#define RTX_SCAN_LDS 0  // (broadcast ds_read_b128, 8 per block) instead of scalar loads
#endif
template <bool kPF, bool kFlat, bool kTile = false>
__device__ __forceinline__ uint32_t scan_range(cfloat_p pre, uint32_t b, uint32_t end, const LineTest &T,
                                               float k0, float k1, uint32_t *my, uint32_t &cnt, bool &full,
                                               uint32_t *pack, const float *lds_pr, uint64_t bmask = ~0ull,
                                               uint32_t bm_lo = 0u) {
    f2v ux = {T.ux, T.ux}, uy = {T.uy, T.uy}, uz = {T.uz, T.uz}, vy = {T.vy, T.vy};
    f2v vz = {T.vz, T.vz}, ku = {k0, k0}, kv = {k1, k1};
    const f2v th = {T.thr, T.thr};
    // Q of one sphere pair (cy unused on a flat run)
    auto qpair = [&](f2v cx, f2v cy, f2v cz, f2v R) -> f2v {
        f2v pu, pv;
        if constexpr (kFlat) {  // line_test_q_flat: c.v - o.v is one fma
            pu = fma2(cx, ux, fma2(cz, uz, ku));
            pv = fma2(cz, vz, kv);
        } else {                // line_test_q
            pu = fma2(cx, ux, fma2(cy, uy, fma2(cz, uz, ku)));
            pv = fma2(cy, vy, fma2(cz, vz, kv));
        }
        return fma2(-pv, pv, fma2(-pu, pu, R));
    };
    // A block's four pair results q: the ballot, and each flagging lane's
    // list entry; true when some lane's list is full and the scan must stop
    // after this block.
    auto finish = [&](const f2v *q, uint32_t bb) -> bool {
        // a chain, so that it folds into v_max3_f32
        const float mx = fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(q[0].x, q[0].y), q[1].x), q[1].y), q[2].x),
                                                 q[2].y), q[3].x), q[3].y);
        RTX_DIAG_ADD(0, 1u);
        if (__ballot(!(mx < T.thr)) != 0ull) {
            RTX_DIAG_ADD(1, 1u);
            // q - thr >= +0 exactly when q >= thr (q is finite; thr = -inf
            // gives +inf): the sign bits, shifted in from sphere 7 down to
            // sphere 0, are the NOT-flagged mask.
            uint32_t inv = 0;
#pragma unroll
            for (int p = 3; p >= 0; --p) {
                const f2v s = q[p] - th;
                inv = (inv << 1) | (__float_as_uint(s.y) >> 31);
                inv = (inv << 1) | (__float_as_uint(s.x) >> 31);
            }
            const uint32_t mask = ~inv & 0xffu;
            my[cnt * kRB] = (8u * bb) | (mask << 24);  // cnt < kCand here
            cnt += mask != 0u ? 1u : 0u;
            return __ballot(cnt == cand_of<kPF>()) != 0ull;
        }
        return false;
    };
    // One 8-sphere block (blk(i) = its i-th float)
    auto step = [&](auto blk, uint32_t bb) -> bool {
        f2v q[4];
#pragma unroll
        for (int p = 0; p < 4; ++p)
            q[p] = qpair(f2v{blk(2 * p), blk(2 * p + 1)}, kFlat ? f2v{0.0f, 0.0f} : f2v{blk(8 + 2 * p), blk(9 + 2 * p)},
                         f2v{blk(16 + 2 * p), blk(17 + 2 * p)}, f2v{blk(24 + 2 * p), blk(25 + 2 * p)});
        return finish(q, bb);
    };
    full = true;
    // kTile (k_render's large-scene lane mode, which passes its tile): the
    // tile stream is the only scan instantiated there, so the SGPR ping-pong
    // below (64 SGPRs) does not crowd that kernel's registers
    if (kTile && kPF && RTX_PF_RING && lds_pr != nullptr) {
        // A/B build: the scene streams through a ring of
        // kNR 1-KiB slots (8 blocks each) per wave, filled by LDS-DMA with no
        // VGPR staging: kNR - 1 tiles in flight while one is scanned. Before
        // tile j is scanned, tile j + kNR - 1 is issued into the slot tile
        // j - 1 used, and vmcnt(kNR - 1) retires tile j (vector-memory
        // operations complete in issue order). Tiles past `end` re-read the
        // last block (a constant count of loads in flight); a scan that stops
        // for a full list leaves its loads in flight (the next scan's counted
        // waits cover them: they are older), one that reaches `end` drains.
        // Every lane of the wave runs this (the DMA writes one 16-byte piece
        // per lane).
        constexpr uint32_t kNR = RTX_PF_RING ? RTX_PF_RING : 2u;  // (the branch is dead when 0)
        static_assert(kNR >= 2 && kNR <= 8, "ring of 2..8 slots");
        float4 *ring = const_cast<float4 *>(reinterpret_cast<const float4 *>(lds_pr)) +
                       64u * kNR * ((threadIdx.x & 255u) >> 6);
        const uint32_t rbase = (uint32_t)__builtin_amdgcn_readfirstlane(lds_addr(ring));
        const float4 *gp = (const float4 *)(const float *)pre;
        const uint32_t lane = threadIdx.x & 63u;
        auto issue = [&](uint32_t tb, uint32_t slot) {
            glds16(gp + 8u * min(tb + (lane >> 3), end - 1u) + (lane & 7u), rbase + 1024u * slot);
        };
        uint32_t tb = b - b % 8u;
#pragma unroll
        for (uint32_t k = 0; k + 1 < kNR; ++k) issue(tb + 8u * k, k);
        for (uint32_t j = 0;; ++j) {
            issue(tb + 8u * (kNR - 1u), (j + kNR - 1u) % kNR);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kNR - 1u) : "memory");
            const float4 *q0 = ring + 64u * (j % kNR);
            const uint32_t e = min(tb + 8u, end);
            for (; b < e; ++b) {
                const float4 *q = q0 + 8u * (b - tb);
                float4 v[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) v[t] = q[t];
                auto blk = [&](int i) {
                    const float4 w = v[i >> 2];
                    const int c = i & 3;
                    return c == 0 ? w.x : c == 1 ? w.y : c == 2 ? w.z : w.w;
                };
                if (step(blk, b)) return b + 1;
            }
            if (tb + 8u >= end) break;
            tb += 8u;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (kTile && kPF && RTX_PF_LDS && lds_pr != nullptr) {
        // A/B build: the scene streams through a per-wave
        // LDS tile of 8 * RTX_PF_LDS blocks (RTX_PF_LDS KiB: coalesced 16-byte
        // loads, one per lane per KiB, the next tile's loads in flight while
        // this one is scanned), and each block is read from it with 8
        // broadcast ds_read_b128 into VGPRs. Every lane of the wave runs this
        // (hit_world_pre_ld's `live`).
        constexpr uint32_t kT = 8u * RTX_PF_LDS;  // blocks per tile
        float4 *tl = const_cast<float4 *>(reinterpret_cast<const float4 *>(lds_pr)) +
                     64u * RTX_PF_LDS * ((threadIdx.x & 255u) >> 6);
        const float4 *gp = (const float4 *)(const float *)pre;
        const uint32_t lane = threadIdx.x & 63u;
        auto fetch = [&](uint32_t tb, uint32_t k) {
            return gp[8u * min(tb + 8u * k + (lane >> 3), end - 1u) + (lane & 7u)];
        };
        uint32_t tb = b - b % kT;
        float4 cur[RTX_PF_LDS ? RTX_PF_LDS : 1];
#pragma unroll
        for (uint32_t k = 0; k < RTX_PF_LDS; ++k) cur[k] = fetch(tb, k);
        for (;;) {
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (uint32_t k = 0; k < RTX_PF_LDS; ++k) tl[64u * k + lane] = cur[k];
            __builtin_amdgcn_wave_barrier();
            const bool more = tb + kT < end;
            if (more) {
#pragma unroll
                for (uint32_t k = 0; k < RTX_PF_LDS; ++k) cur[k] = fetch(tb + kT, k);
            }
            const uint32_t e = min(tb + kT, end);
            for (; b < e; ++b) {
                // (reading the floats at their use, or staging the block in
                // two halves, measured 7 % slower at C5: R7b, R7d)
                const float4 *q = tl + 8u * (b - tb);
                float4 v[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) v[t] = q[t];
                auto blk = [&](int i) {
                    const float4 w = v[i >> 2];
                    const int c = i & 3;
                    return c == 0 ? w.x : c == 1 ? w.y : c == 2 ? w.z : w.w;
                };
                if (step(blk, b)) return b + 1;
            }
            if (!more) break;
            tb += kT;
        }
    } else if (!kTile && kPF) {  // (the same for small scenes measured 6 % slower: R7c)
        // ping-pong between two SGPR buffers (no copies): A holds block b
        f16v a_lo, a_hi, b_lo, b_hi;
        sload_blk(pre + 32 * b, a_lo, a_hi, ux, uy, uz, vy, vz, ku, kv);
        sload_wait(a_lo, a_hi);
        for (;;) {
            sload_blk(pre + 32 * min(b + 1, end - 1), b_lo, b_hi, ux, uy, uz, vy, vz, ku, kv);
            bool f = step([&](int i) { return i < 16 ? a_lo[i] : a_hi[i - 16]; }, b);
            sload_wait(b_lo, b_hi);
            if (f) return b + 1;
            if (++b >= end) break;
            // publish the position at b = 0 mod kPackEvery, from this half of
            // the ping-pong only: it sees blocks of one parity, so only scans
            // that started at an odd block publish — in practice the flat run
            // that resumes at block 1 after the ground sphere's block 0, i.e.
            // the wrapped leg of a segment. Publishing from both halves (every
            // scan) measured no faster than no pack at all, this 4-7 % faster
            // (DESIGN.md §7 R4k-q).
            if (kPF && RTX_PACK && pack && (b & (kPackEvery - 1u)) == 0u && (threadIdx.x & 63u) == 0u) *pack = b;
            sload_blk(pre + 32 * min(b + 1, end - 1), a_lo, a_hi, ux, uy, uz, vy, vz, ku, kv);
            f = step([&](int i) { return i < 16 ? b_lo[i] : b_hi[i - 16]; }, b);
            sload_wait(a_lo, a_hi);
            if (f) return b + 1;
            if (++b >= end) break;
        }
    } else {
        if (RTX_SCAN_LDS && lds_pr) {
            for (; b < end; ++b) {  // pair p of block b: [cx0 cx1 cy0 cy1 cz0 cz1 R0 R1] (SphLds)
                const float4 *q = reinterpret_cast<const float4 *>(lds_pr + 32u * b);
                float4 v[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) v[t] = q[t];
                auto blk = [&](int i) {  // AoSoA-8 float i of the block
                    const int c = i >> 3, sp = i & 7, pp = sp >> 1, w = sp & 1;
                    const float4 A = v[2 * pp], B = v[2 * pp + 1];
                    const float a = w ? A.y : A.x, bb = w ? A.w : A.z, cc = w ? B.y : B.x, dd = w ? B.w : B.z;
                    return c == 0 ? a : c == 1 ? bb : c == 2 ? cc : dd;
                };
                if (step(blk, b)) return b + 1;
            }
        } else if (bmask != ~0ull) {
            // the layer grid's blocks (hit_world_pre_ld: bit j = block bm_lo + j,
            // wave-uniform; end <= bm_lo + 64): the set ones, in order
            while (b < end) {
                const uint64_t r = bmask & (~0ull << (b - bm_lo));
                if (r == 0ull) break;
                b = bm_lo + (uint32_t)__builtin_ctzll(r);
                if (b >= end) break;
                const cfloat_p blk = pre + 32 * b;
                if (step([&](int i) { return blk[i]; }, b)) return b + 1;
                ++b;
            }
        } else {
            for (; b < end; ++b) {
                const cfloat_p blk = pre + 32 * b;
                if (step([&](int i) { return blk[i]; }, b)) return b + 1;
            }
        }
    }
    full = false;
    return end;
}

// The scan over blocks [b, nblk): the scene's flat run [flat_lo, flat_hi)
// (rtx_internal.h KScene) with the 5-op test, the rest with the 7-op one.
// Returns the block to resume at: nblk, or earlier once some lane's list is
// full (wave-uniform). kPF scans publish their position to `pack` (below).
template <bool kPF, bool kTile = false>
__device__ __forceinline__ uint32_t scan_prefilter(cfloat_p pre, uint32_t b, uint32_t nblk, const LineTest &T,
                                                   const KScene &S, uint32_t *list, uint32_t &cnt,
                                                   uint32_t *pack = nullptr, const float *lds_pr = nullptr,
                                                   uint64_t gm = ~0ull) {
    cnt = 0;
    uint32_t *my = list + threadIdx.x;
    const LineFlat K = line_test_flat(T, S.flat_cy);
    while (b < nblk) {
        bool full;
        if (b < S.flat_lo) {
            b = scan_range<kPF, false, kTile>(pre, b, min(S.flat_lo, nblk), T, T.nou, T.nov, my, cnt, full, pack, lds_pr);
        } else if (b < S.flat_hi) {
            b = scan_range<kPF, true, kTile>(pre, b, min(S.flat_hi, nblk), T, K.ku, K.kv, my, cnt, full, pack, lds_pr,
                                             gm, S.flat_lo);
        } else {
            b = scan_range<kPF, false, kTile>(pre, b, nblk, T, T.nou, T.nov, my, cnt, full, pack, lds_pr);
        }
        if (full) break;
    }
    return b;
}

// Resolve the lane's list (m entries: first sphere index | mask << 24)
// with the reference's own ops (Sphere.cpp:6-24 / ShaderCompute.hlsl:
// 155-186), one candidate per lane per iteration, no branch inside an
// iteration. Sphere data: cen[i] = (center, radius) in one load; -(r*r) is
// the same fp32 product the upload negates into soa; a padded index (>= n)
// reads sphere n-1, whose copy it is. A prefilter false positive (exact
// disc < 0) is skipped, like the reference's `if (d < 0) return false`.
// Returns false if a candidate has a non-finite root (the lane then takes
// hit_blocks_seq).
// The running closest hit of a resolve as one 64-bit key: the root's bits
// (c >= t_min > 0, or t_max = +inf: bits order like values) above
// ~(index + 1), so the smaller key is the smaller root, then the larger
// index among equal roots — the in-order scan's rule (`t_max < root`
// rejects, :171) as a single unsigned compare. No hit: index -1 (low word ~0).
__device__ __forceinline__ uint64_t hit_key(float best, int idx) {
    return ((uint64_t)__float_as_uint(best) << 32) | (uint32_t) ~(uint32_t)(idx + 1);
}
__device__ __forceinline__ void key_hit(uint64_t k, float &best, int &idx) {
    best = __uint_as_float((uint32_t)(k >> 32));
    idx = (int)~(uint32_t)k - 1;
}

// One candidate: sc = (center, radius) of sphere g; live = it is one.
// key: the running closest hit (hit_key).
__device__ __forceinline__ void resolve_one(float4 sc, int g, bool live, f3 o, f3 d, float a, float inv_a,
                                            float t_min, uint64_t &key, bool &ok) {
    const float inf = __uint_as_float(0x7f800000u);
    const float ocx = o.x - sc.x;
    const float ocy = o.y - sc.y;
    const float ocz = o.z - sc.z;
    const float hb = fmaf(ocz, d.z, fmaf(ocy, d.y, ocx * d.x));
    const float cc = fmaf(ocz, ocz, fmaf(ocy, ocy, fmaf(ocx, ocx, -(sc.w * sc.w))));
    const float disc = fmaf(hb, hb, -(a * cc));
    const bool cand = live & !(disc < 0.0f);
    const float sq = sqrt_rn(disc);
    const float rn = (-hb - sq) * inv_a;
    const float rf = (-hb + sq) * inv_a;
    const bool fin = fabsf(rn) < inf && fabsf(rf) < inf;
    ok = ok & (!cand | fin);
    // near root if it is >= t_min, else the far one; accepted if >= t_min
    // and its key beats the running one (roots finite here: a lane with a
    // non-finite one is redone by hit_blocks_seq)
    const float c = !(rn < t_min) ? rn : rf;
    const uint64_t k = ((uint64_t)__float_as_uint(c) << 32) | (uint32_t) ~(uint32_t)(g + 1);
    const bool acc = cand & !(c < t_min) & (k < key);
    key = acc ? k : key;
}

// `ld(i)` returns (center, radius) of sphere i < n.
// The candidate stream is software-pipelined: the next candidate's sphere
// is loaded before the current one is tested, so a load from L2/HBM (cen,
// large scenes) runs under the previous test (the order of tests is
// unchanged; C5 -1.5 %, C2 neutral: DESIGN.md §7 R2z).
// `gi(p)` maps a list position to the scene index (the culled layout's
// position map; identity for `pre`).
struct GiIdentity {
    __device__ __forceinline__ uint32_t operator()(uint32_t p) const { return p; }
};
// kPos: ld takes the list position (clamped to n - 1) instead of the scene
// index (the culled layout keeps a copy of the spheres in position order, so
// the data load and the index load are independent).
template <typename Ld, typename Gi = GiIdentity, bool kPos = false>
__device__ __forceinline__ bool resolve_pre_t(Ld ld, uint32_t n, const uint32_t *list, uint32_t m, f3 o, f3 d,
                                              float a, float inv_a, float t_min, float &best, int &idx,
                                              uint32_t cap = (uint32_t)kCand, Gi gi = Gi()) {
    bool ok = true;
    uint32_t j = 0;
    uint32_t e = list[threadIdx.x];  // entry 0 (unused when m == 0)
    RTX_DIAG_ADD(4, (uint32_t)__popcll(__ballot(m != 0u)));
#if RTX_DIAG_PROF
    {  // candidates of the wave (the resolve's rounds are their max over lanes)
        uint32_t c = 0;
        for (uint32_t q = 0; q < m; ++q) c += (uint32_t)__popc(list[min(q, cap) * kRB + threadIdx.x] >> 24);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) c += (uint32_t)__shfl_xor((int)c, off, 64);
        RTX_DIAG_ADD(5, c);
    }
#endif
    // next candidate: sphere index i (live = the lane has one), then advance
    uint32_t pos = 0;  // (kPos) the position of the candidate next() returns
    auto next = [&](uint32_t &i, bool &live) {
        live = j < m;
        pos = (e & 0xffffffu) + (uint32_t)__builtin_ctz(live ? (e >> 24) : 1u);
        if constexpr (kPos) pos = min(pos, n - 1u);
        i = gi(pos);
        e &= e - (1u << 24);  // drop that candidate from the mask
        const bool adv = live && (e >> 24) == 0u;
        j += adv ? 1u : 0u;
        const uint32_t nx = list[min(j, cap) * kRB + threadIdx.x];
        e = adv ? nx : e;
    };
    uint32_t i0;
    bool l0;
    next(i0, l0);
    float4 v0 = kPos ? ld(pos) : ld(min(i0, n - 1u));
    uint64_t key = hit_key(best, idx);
    while (__ballot(l0) != 0ull) {
        RTX_DIAG_ADD(2, 1u);
        uint32_t i1;
        bool l1;
        next(i1, l1);
        const float4 v1 = kPos ? ld(pos) : ld(min(i1, n - 1u));
        resolve_one(v0, (int)i0, l0, o, d, a, inv_a, t_min, key, ok);
        i0 = i1;
        l0 = l1;
        v0 = v1;
    }
    key_hit(key, best, idx);
    return ok;
}
__device__ __forceinline__ bool resolve_pre(const float4 *__restrict__ cen, uint32_t n, const uint32_t *list,
                                            uint32_t m, f3 o, f3 d, float a, float inv_a, float t_min,
                                            float &best, int &idx) {
    return resolve_pre_t([cen](uint32_t i) { return cen[i]; }, n, list, m, o, d, a, inv_a, t_min, best, idx);
}

// The culled scan (KScene::cpre / cbnd, small scenes; DESIGN.md §3 "culled
// scan"): blocks [b, n_cpad / 8) of the spatially ordered layout, in groups
// of 8. A group's 8 block bounds are tested like 8 spheres (the same 7/5-op
// test, against thr_b = thr * kCullThrScale: rtx_prefilter.h cull_bound), one
// ballot per bound; only the blocks some lane's line passes are scanned, with
// scan_range's per-block test and list entries (positions of the layout:
// the resolve maps them through cperm). Returns the block to resume at: the
// end, or the block after the one at which some lane's list filled (a resumed
// group is tested again, its earlier blocks masked off). Wave-uniform.
// A bound also fails when it is wholly behind the lane's origin (the half
// test H, Hs: rtx_prefilter.h HalfTest; 5 more fp32 ops per bound, 4 flat).
__device__ __forceinline__ uint32_t scan_culled(const KScene &S, uint32_t b, const LineTest &T, const LineTest &Ts,
                                                const HalfTest &H, const HalfTest &Hs, uint32_t *list,
                                                uint32_t &cnt) {
    cnt = 0;
    uint32_t *my = list + threadIdx.x;
    const uint32_t nblk = S.n_cpad / 8u;
    const LineFlat K = line_test_flat(T, S.flat_cy);
    // flat bounds: the ray stretched along y (rtx_prefilter.h kCullSy), the 5-op test
    const LineFlat Ks = line_test_flat(Ts, kCullSy * S.flat_cy);
    const f2v uxs = {Ts.ux, Ts.ux}, uzs = {Ts.uz, Ts.uz}, vzs = {Ts.vz, Ts.vz}, kus = {Ks.ku, Ks.ku},
              kvs = {Ks.kv, Ks.kv};
    const float thr_bs = Ts.thr * kCullThrScaleSy;
    f2v ux = {T.ux, T.ux}, uy = {T.uy, T.uy}, uz = {T.uz, T.uz}, vy = {T.vy, T.vy}, vz = {T.vz, T.vz};
    f2v ku = {K.ku, K.ku}, kv = {K.kv, K.kv};
    const f2v nou = {T.nou, T.nou}, nov = {T.nov, T.nov};
    const f2v th = {T.thr, T.thr};
    const float thr_b = T.thr * kCullThrScale;
    const f2v hdx = {H.dx, H.dx}, hdy = {H.dy, H.dy}, hdz = {H.dz, H.dz}, hnod = {H.nod, H.nod};
    const f2v ha = {H.a, H.a}, htha = {H.tha, H.tha};
    const float kws1 = half_test_kw(Hs, kCullSy * S.flat_cy), kwf1 = half_test_kw(H, S.flat_cy);
    const f2v kwf = {kwf1, kwf1};
    const f2v kws = {kws1, kws1}, has = {Hs.a, Hs.a}, hthas = {Hs.tha, Hs.tha};
    // Q of the 4 pairs of an AoSoA-8 block of spheres or bounds (blk(i): its i-th float)
    auto quad = [&](auto flat, auto blk, f2v *q) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const f2v cx = {blk(2 * p), blk(2 * p + 1)};
            const f2v cz = {blk(16 + 2 * p), blk(17 + 2 * p)};
            const f2v R = {blk(24 + 2 * p), blk(25 + 2 * p)};
            f2v pu, pv;
            if constexpr (decltype(flat)::value) {
                pu = fma2(cx, ux, fma2(cz, uz, ku));
                pv = fma2(cz, vz, kv);
            } else {
                const f2v cy = {blk(8 + 2 * p), blk(9 + 2 * p)};
                pu = fma2(cx, ux, fma2(cy, uy, fma2(cz, uz, nou)));
                pv = fma2(cy, vy, fma2(cz, vz, nov));
            }
            q[p] = fma2(-pv, pv, fma2(-pu, pu, R));
        }
    };
    // one block of spheres: scan_range's finish (ballot, list entry). Its
    // floats are read first, all of them, so that they arrive by a few wide
    // scalar loads and one wait.
    auto step = [&](auto flat, uint32_t bb) -> bool {
        const cfloat_p blk = (cfloat_p)S.cpre + 32u * bb;
        float v[32];
#pragma unroll
        for (int i = 0; i < 32; ++i)
            if (!decltype(flat)::value || i < 8 || i >= 16) v[i] = blk[i];
        f2v q[4];
        quad(flat, [&](int i) { return v[i]; }, q);
        const float mx = fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(q[0].x, q[0].y), q[1].x), q[1].y), q[2].x),
                                             q[2].y), q[3].x), q[3].y);
        RTX_DIAG_ADD(0, 1u);
        if (__ballot(!(mx < T.thr)) != 0ull) {
            RTX_DIAG_ADD(1, 1u);
            uint32_t inv = 0;
#pragma unroll
            for (int p = 3; p >= 0; --p) {
                const f2v sq = q[p] - th;
                inv = (inv << 1) | (__float_as_uint(sq.y) >> 31);
                inv = (inv << 1) | (__float_as_uint(sq.x) >> 31);
            }
            // the flagged spheres wholly behind the lane's origin drop out
            // (the half test per sphere; only for blocks some lane flags)
            uint32_t hm = 0xffu;
            if (RTX_CULL_HALF_SPHERES) {
                hm = 0u;
#pragma unroll
                for (int p = 3; p >= 0; --p) {
                    const f2v cx = {v[2 * p], v[2 * p + 1]}, cz = {v[16 + 2 * p], v[17 + 2 * p]};
                    const f2v R = {v[24 + 2 * p], v[25 + 2 * p]};
                    f2v pw;
                    if constexpr (decltype(flat)::value) {
                        pw = fma2(cx, hdx, fma2(cz, hdz, kwf));
                    } else {
                        const f2v cy = {v[8 + 2 * p], v[9 + 2 * p]};
                        pw = fma2(cx, hdx, fma2(cy, hdy, fma2(cz, hdz, hnod)));
                    }
                    const f2v q2 = fma2(-pw, pw, fma2(R, ha, htha));
                    hm = (hm << 1) | (half_test_pass(pw.y, q2.y) ? 1u : 0u);
                    hm = (hm << 1) | (half_test_pass(pw.x, q2.x) ? 1u : 0u);
                }
            }
            const uint32_t mask = ~inv & hm & 0xffu;
            my[cnt * kRB] = (8u * bb) | (mask << 24);
            cnt += mask != 0u ? 1u : 0u;
            return __ballot(cnt == cand_of<true>()) != 0ull;
        }
        return false;
    };
    using Flat = std::integral_constant<bool, true>;
    using Full = std::integral_constant<bool, false>;
    // the wave-OR of the 8 bound tests of an AoSoA-8 group of bounds: bit j
    // when some lane's line passes bound j (8 ballots). Flat bounds are in
    // the stretched space: the stretched ray's 5-op test against thr_bs.
    // A lane passes a bound when its line passes it and the bound is not
    // wholly behind its origin (the half test; stretched for flat bounds).
    auto bound_mask1 = [&](cfloat_p grp, bool flat) -> uint32_t {
        float v[32];
        f2v q[4], pw[4], q2[4];
        float thr = thr_b;
        if (flat) {
#pragma unroll
            for (int i = 0; i < 32; ++i)
                if (i < 8 || i >= 16) v[i] = grp[i];
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const f2v cx = {v[2 * p], v[2 * p + 1]}, cz = {v[16 + 2 * p], v[17 + 2 * p]};
                const f2v R = {v[24 + 2 * p], v[25 + 2 * p]};
                const f2v pu = fma2(cx, uxs, fma2(cz, uzs, kus));
                const f2v pv = fma2(cz, vzs, kvs);
                q[p] = fma2(-pv, pv, fma2(-pu, pu, R));
                pw[p] = fma2(cx, hdx, fma2(cz, hdz, kws));
                q2[p] = fma2(-pw[p], pw[p], fma2(R, has, hthas));
            }
            thr = thr_bs;
        } else {
#pragma unroll
            for (int i = 0; i < 32; ++i) v[i] = grp[i];
            quad(Full(), [&](int i) { return v[i]; }, q);
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const f2v cx = {v[2 * p], v[2 * p + 1]}, cy = {v[8 + 2 * p], v[9 + 2 * p]};
                const f2v cz = {v[16 + 2 * p], v[17 + 2 * p]}, R = {v[24 + 2 * p], v[25 + 2 * p]};
                pw[p] = fma2(cx, hdx, fma2(cy, hdy, fma2(cz, hdz, hnod)));
                q2[p] = fma2(-pw[p], pw[p], fma2(R, ha, htha));
            }
        }
        uint32_t m = 0;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const bool px = !(q[p].x < thr) && (!RTX_CULL_HALF || half_test_pass(pw[p].x, q2[p].x));
            const bool py = !(q[p].y < thr) && (!RTX_CULL_HALF || half_test_pass(pw[p].y, q2[p].y));
            m |= (__ballot(px) != 0ull ? 1u : 0u) << (2 * p);
            m |= (__ballot(py) != 0ull ? 1u : 0u) << (2 * p + 1);
        }
        return m;
    };
    auto first_bits = [](uint32_t n) { return n >= 8u ? 0xffu : (1u << n) - 1u; };
    // 8 bounds whose entries cover blocks from b0 on: flat (stored and tested
    // stretched) iff b0 >= cflat_lo (cflat_lo is a multiple of 512 blocks, so
    // no test straddles it: rtx_api.hip build_cull)
    auto bound_mask = [&](cfloat_p grp, uint32_t b0) -> uint32_t { return bound_mask1(grp, b0 >= S.cflat_lo); };
    // Three levels above the blocks: a group bound covers the 64 spheres of 8
    // blocks, a super bound the 512 of 8 groups; the super bounds are tested 8
    // at a time (4,096 spheres), then, for each passing super-group, its 8
    // group bounds, for each passing group its 8 block bounds, then the
    // passing blocks' spheres. A resumed scan (b inside a range) masks off
    // the super-groups, groups and blocks before b.
    const uint32_t ng = (nblk + 7u) / 8u, nsg = (ng + 7u) / 8u, nhg = (nsg + 7u) / 8u;
    for (uint32_t hg = b >> 9; hg < nhg; ++hg) {
        uint32_t m3 = first_bits(nsg - 8u * hg);
        if (RTX_CULL_LEVELS >= 3) m3 &= bound_mask((cfloat_p)S.cbnd3 + 32u * hg, 512u * hg);
        if (hg == (b >> 9)) m3 &= 0xffu << ((b >> 6) & 7u);
        while (m3 != 0u) {
            const uint32_t sg = 8u * hg + (uint32_t)__builtin_ctz(m3);
            m3 &= m3 - 1u;
            uint32_t m2 = bound_mask((cfloat_p)S.cbnd2 + 32u * sg, 64u * sg) & first_bits(ng - 8u * sg);
            if (sg == (b >> 6)) m2 &= 0xffu << ((b >> 3) & 7u);
            RTX_DIAG_ADD(6, (uint32_t)__popc(m2));
            while (m2 != 0u) {
                const uint32_t g = 8u * sg + (uint32_t)__builtin_ctz(m2);
                m2 &= m2 - 1u;
                uint32_t m = bound_mask((cfloat_p)S.cbnd + 32u * g, 8u * g) & first_bits(nblk - 8u * g);
                if (g == (b >> 3)) m &= 0xffu << (b & 7u);
                while (m != 0u) {
                    const uint32_t bb = 8u * g + (uint32_t)__builtin_ctz(m);
                    m &= m - 1u;
                    if (bb >= S.cflat_lo ? step(Flat(), bb) : step(Full(), bb)) return bb + 1u;
                }
            }
        }
    }
    return nblk;
}

// hit_world over the culled layout: same (best, idx) as hit_world_pre (the
// resolution rule is order-independent; the bounds never drop a reference
// candidate). The resolve reads a candidate's (centre, radius) from ccen and
// its scene index (the key's tie-break) from cperm, both by layout position.
// The ray stretched along y for the flat bounds (rtx_prefilter.h kCullSy;
// tests/prefilter_check.cpp runs the same ops).
__device__ __forceinline__ LineTest line_test_stretched(const KScene &S, f3 o, f3 d) {
    const float dys = kCullSy * d.y;
    const float as = fmaf(d.z, d.z, fmaf(dys, dys, d.x * d.x));
    return line_test_setup(o.x, kCullSy * o.y, o.z, d.x, dys, d.z, as, S.smag * kCullSy);
}
// The half test of the stretched ray (the same as, a, as line_test_stretched).
__device__ __forceinline__ HalfTest half_test_stretched(f3 o, f3 d, float thr_bs, float t_min) {
    const float dys = kCullSy * d.y;
    const float as = fmaf(d.z, d.z, fmaf(dys, dys, d.x * d.x));
    return half_test_setup(o.x, kCullSy * o.y, o.z, d.x, dys, d.z, as, thr_bs, t_min);
}
__device__ __forceinline__ int hit_world_culled(const KScene &S, f3 o, f3 d, float a, float inv_a, float t_min,
                                                float &best, uint32_t *list) {
    const LineTest T = line_test_setup(o.x, o.y, o.z, d.x, d.y, d.z, a, S.smag);
    const LineTest Ts = line_test_stretched(S, o, d);
    const HalfTest H = half_test_setup(o.x, o.y, o.z, d.x, d.y, d.z, a, T.thr * kCullThrScale, t_min);
    const HalfTest Hs = half_test_stretched(o, d, Ts.thr * kCullThrScaleSy, t_min);
    const float best0 = best;
    int idx = -1;
    bool ok = true;
    const uint32_t nblk = S.n_cpad / 8u;
    auto ld = [&S](uint32_t p) { return S.ccen[p]; };
    auto gi = [&S](uint32_t p) { return S.cperm[p]; };
    uint32_t b = 0;
    do {
        uint32_t cnt;
        b = scan_culled(S, b, T, Ts, H, Hs, list, cnt);
        ok = resolve_pre_t<decltype(ld), decltype(gi), true>(ld, S.n_cpad, list, cnt, o, d, a, inv_a, t_min, best,
                                                              idx, cand_of<true>(), gi) &&
             ok;
    } while (b < nblk);
    if (!ok) {
        RTX_DIAG_ADD(3, (uint32_t)__popcll(__ballot(1)));
        best = best0;
        idx = hit_blocks_seq((cfloat_p)S.soa, S.n_pad / 8, 0, o, d, a, inv_a, t_min, best, -1);
    }
    return idx;
}

// The layer grid (rtx_grid.h): the blocks of the flat run some
// lane of the wave may need — the OR of the lanes' walks. Only the lanes that
// reach hit_world take part (an inactive lane needs nothing); the OR goes
// through one LDS word per wave, the list's spare row at the wave's first two
// lanes (`spare`: the list's row `cap`, never a list entry). A lane outside
// the prefilter's safe range marks every block.
__device__ __forceinline__ uint64_t grid_wave_mask(const KScene &S, f3 o, f3 d, const LineTest &T, uint32_t *spare) {
    const LayerGrid G = *S.grid;  // wave-uniform: scalar loads
    const uint64_t *gc = reinterpret_cast<const uint64_t *>(S.grid + 1);
    const uint64_t mine = T.thr == -__uint_as_float(0x7f800000u)
                              ? ~0ull
                              : grid_mask(G, [gc](uint32_t k) { return gc[k]; }, o.x, o.y, o.z, d.x, d.y, d.z);
    unsigned long long *w = reinterpret_cast<unsigned long long *>(spare + (threadIdx.x & ~63u));
    const uint32_t lead = (uint32_t)__builtin_amdgcn_readfirstlane((int)threadIdx.x);
    if (threadIdx.x == lead) __hip_atomic_store(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __hip_atomic_fetch_or(w, (unsigned long long)mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const unsigned long long v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// hit_world with the prefiltered scan: same (best, idx) as the in-order
// reference scan. Candidates are resolved in rounds (a round ends when some
// lane's list is full); the (min c, largest index) rule is
// order-independent, so rounds compose. A non-finite root takes
// hit_blocks_seq.
// `ld(i)` returns (center, radius) of sphere i for the resolve (cen in HBM,
// or, for scenes up to kCoopLds spheres, the block's LDS copy of them).
// pack (kPF kernels, RTX_PACK): the workgroup's LDS word holding the block a
// wave of it scanned last (published every kPackEvery blocks). A segment's
// scan starts kPackLag blocks behind it and wraps round — [b0, nblk) then
// [0, b0): the resolution rule is order-independent, so any start gives the
// in-order answer — so the workgroup's waves stream the 100k-sphere array
// together and a block one wave brought into the scalar cache serves the
// waves that trail it, instead of every wave missing on every block.
// start (no pack word): the block to start at (rtx_debug_hit_world_from),
// wave-uniform.
template <bool kPF, typename Ld, bool kTile = false, bool kGridOk = true>
__device__ __forceinline__ int hit_world_pre_ld(const KScene &S, Ld ld, f3 o, f3 d, float a, float inv_a,
                                                float t_min, float &best, uint32_t *list, uint32_t *pack = nullptr,
                                                uint32_t start = 0, const float *lds_pr = nullptr,
                                                bool live = true) {
    const cfloat_p pre = (cfloat_p)S.pre;
    const uint32_t nblk = S.n_pad / 8;
    LineTest T = line_test_setup(o.x, o.y, o.z, d.x, d.y, d.z, a, S.smag);
    if (!live) {  // a lane without a ray (RTX_PF_LDS: every lane fills the tile): nothing is flagged
        T.ux = T.uy = T.uz = T.vy = T.vz = T.nou = T.nov = 0.0f;
        T.thr = __uint_as_float(0x7f800000u);
    }
    // the layer grid (small scenes, rtx_grid.h): the flat run's blocks some lane of the wave needs
    uint64_t gm = ~0ull;
    if constexpr (!kPF && kGridOk) {
        if (RTX_GRID && S.grid != nullptr) gm = grid_wave_mask(S, o, d, T, list + cand_of<kPF>() * kRB);
    }
    const float best0 = best;
    int idx = -1;
    bool ok = true;
    uint32_t b0 = nblk ? start % nblk : 0u;
    if (RTX_PACK && kPF && pack) {
        const uint32_t at = __builtin_amdgcn_readfirstlane(*pack);  // wave-uniform (SGPR)
        b0 = at < nblk ? (at + nblk - kPackLag) % nblk : 0u;  // nblk > 128 > kPackLag
    }
    uint32_t b = b0, end = nblk;
    for (;;) {
        uint32_t cnt;
        b = scan_prefilter<kPF, kTile>(pre, b, end, T, S, list, cnt, pack, lds_pr, gm);
        ok = resolve_pre_t(ld, S.n, list, cnt, o, d, a, inv_a, t_min, best, idx, cand_of<kPF>()) && ok;
        if (b < end) continue;
        if (end == nblk && b0 != 0u) {  // wrap round to the start
            b = 0;
            end = b0;
            continue;
        }
        break;
    }
    if (!ok) {
        RTX_DIAG_ADD(3, (uint32_t)__popcll(__ballot(1)));
        best = best0;
        idx = hit_blocks_seq((cfloat_p)S.soa, nblk, 0, o, d, a, inv_a, t_min, best, -1);
    }
    return idx;
}
// kGridOk false: no layer grid (a kernel that has no other use for its code:
// the large-scene kernels' rare exact fallback)
template <bool kPF, bool kGridOk = true>
__device__ __forceinline__ int hit_world_pre(const KScene &S, f3 o, f3 d, float a, float inv_a,
                                             float t_min, float &best, uint32_t *list, uint32_t *pack = nullptr,
                                             uint32_t start = 0) {
    const float4 *__restrict__ cen = S.cen;
    auto ld = [cen](uint32_t i) { return cen[i]; };
    return hit_world_pre_ld<kPF, decltype(ld), false, kGridOk>(S, ld, o, d, a, inv_a, t_min, best, list, pack, start);
}

// ---- group-cooperative hit_world (frame tail, heavy tiers) -----------------
// Once the pixel queue is empty a wave runs on until its last pixel ends,
// and the frame ends on the most expensive pixels; the heaviest pixels of a
// frame share (k_heavy_split) are its critical path from the start. Such
// rays are traced together, several lanes per ray (hit_world_groups).
//
// Sphere sources. Scenes up to kCoopLds spheres keep a block-wide LDS copy
// (SphLds): AoSoA-2, pair p = spheres 2p and 2p + 1 as [cx0 cx1 cy0 cy1 cz0
// cz1 R0 R1] (R: the prefilter's inflated r^2, rtx_prefilter.h), padded to a
// multiple of kCoopPad spheres with copies of sphere n - 1, then the radii.
// A pair is two 16-byte LDS reads that land in the register pairs
// v_pk_fma_f32 takes; consecutive lanes read consecutive pairs (no bank
// conflicts). Larger scenes read the same pairs from `pre` (AoSoA-8) and the
// resolve's (centre, radius) from `cen` (SphGlobal). A padded copy computes
// the same roots as sphere n - 1 and can only win where it would (later
// index wins ties): callers clamp the winner to n - 1 (rtx_internal.h).
constexpr uint32_t kCoopSlots = 32;                                   // rays per wave in coop mode (LDS slots)
constexpr uint32_t kCoopWaveBytes = kCoopSlots * 10 * sizeof(float);  // per-wave coop scratch (1280 B)
constexpr uint32_t kCoopBytes = (kRB / 64) * kCoopWaveBytes;
constexpr uint32_t kCoopLds = 640;  // scenes up to this many spheres keep the coop's LDS copy (<= 12.5 KiB: 5 blocks/CU)
constexpr uint32_t kCoopPad = 128;  // the LDS copy's sphere count is padded to a multiple of this
static_assert(kCoopMax <= (int)kCoopSlots, "kCoopMax must be <= 32");
__host__ __device__ constexpr uint32_t coop_npad(uint32_t n) { return (n + kCoopPad - 1u) / kCoopPad * kCoopPad; }
__host__ __device__ constexpr uint32_t coop_lds_bytes(uint32_t n) {
    return coop_npad(n) * 4u * (uint32_t)sizeof(float) + n * (uint32_t)sizeof(float);
}
static_assert(coop_lds_bytes(kCoopLds) <= 12800, "LDS copy of the scene: 5 render blocks per CU");

struct SphLds {
    static constexpr bool kPadded = true;  // npairs is a multiple of 64: every group's steps stay inside
    const float *pr;   // [npairs][8]
    const float *rad;  // [n]
    uint32_t n, npairs;
    __device__ __forceinline__ void pair(uint32_t p, f2v &cx, f2v &cy, f2v &cz, f2v &R) const {
        const float4 *q = reinterpret_cast<const float4 *>(pr + 8u * p);
        const float4 a = q[0], b = q[1];
        cx = f2v{a.x, a.y};
        cy = f2v{a.z, a.w};
        cz = f2v{b.x, b.y};
        R = f2v{b.z, b.w};
    }
    // (centre, radius) of sphere j for the resolve: the same floats as cen[j]
    __device__ __forceinline__ float4 sphere(uint32_t j) const {
        const float *q = pr + 8u * (j >> 1) + (j & 1u);
        return make_float4(q[0], q[2], q[4], rad[min(j, n - 1u)]);
    }
};
struct SphGlobal {
    static constexpr bool kPadded = false;  // pair indices are clamped to npairs - 1
    const float *pre;   // AoSoA-8, n_pad spheres
    const float4 *cen;  // [n]
    uint32_t n, npairs; // npairs = n_pad / 2
    __device__ __forceinline__ void pair(uint32_t p, f2v &cx, f2v &cy, f2v &cz, f2v &R) const {
        const float *b = pre + 32u * (p >> 2) + 2u * (p & 3u);
        cx = *reinterpret_cast<const f2v *>(b);
        cy = *reinterpret_cast<const f2v *>(b + 8);
        cz = *reinterpret_cast<const f2v *>(b + 16);
        R = *reinterpret_cast<const f2v *>(b + 24);
    }
    __device__ __forceinline__ float4 sphere(uint32_t j) const { return cen[min(j, n - 1u)]; }
};

// Build the block's LDS copy (all threads of the block; the caller
// synchronises): sphere i < npad at pair i/2, slot i%2 (copies of n - 1
// beyond n), radii after the pairs.
__device__ __forceinline__ SphLds lds_copy(const KScene &S, float *base, bool on, uint32_t nthreads = kRB) {
    SphLds l;
    l.n = S.n;
    l.npairs = coop_npad(S.n) / 2u;
    l.pr = base;
    l.rad = base + 8u * l.npairs;
    if (on) {
        float *pr = base, *rad = base + 8u * l.npairs;
        for (uint32_t i = threadIdx.x; i < 2u * l.npairs; i += nthreads) {
            const float4 c = S.pre4[min(i, S.n - 1u)];
            float *q = pr + 8u * (i >> 1) + (i & 1u);
            q[0] = c.x;
            q[2] = c.y;
            q[4] = c.z;
            q[6] = c.w;
            if (i < S.n) rad[i] = S.cen[i].w;
        }
    }
    return l;
}
__device__ __forceinline__ SphGlobal sph_global(const KScene &S) {
    SphGlobal g;
    g.pre = S.pre;
    g.cen = S.cen;
    g.n = S.n;
    g.npairs = S.n_pad / 2u;
    return g;
}

// Reduction over aligned groups of 2^lg lanes (lg wave-uniform, whole wave
// active): DPP inside a row of 16 (quad_perm xor 1 and xor 2, then the
// half-row and row mirrors, which pair each lane with one in the other half),
// then gfx950's v_permlane16_swap (rows 2i <-> 2i + 1: xor 16) and
// v_permlane32_swap (halves: xor 32) — VALU exchanges, no LDS round trip.
// With both operands the same register, a swap leaves each lane with its
// own value in one result and its partner's in the other, so op(r0, r1) is
// the xor-16 / xor-32 step. Every lane of a group ends with the group's min
// (or max).
template <bool kMax>
__device__ __forceinline__ uint32_t group_reduce_u32(uint32_t v, uint32_t lg) {
    auto op = [](uint32_t x, uint32_t y) { return kMax ? max(x, y) : min(x, y); };
    if (lg >= 1u) v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));
    if (lg >= 2u) v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));
    if (lg >= 3u) v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false));
    if (lg >= 4u) v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false));
    if (lg >= 5u) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        v = op((uint32_t)r[0], (uint32_t)r[1]);
    }
    if (lg >= 6u) {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        v = op((uint32_t)r[0], (uint32_t)r[1]);
    }
    return v;
}

// Group coop (the frame tail, tier 1 and tier 2; any ray count). The rays
// go in chunks of at most kGfRays; a chunk of m rays gives ray r the
// g = 64 / 2^ceil(log2 m) lanes [r*g, r*g + g), and lane k of a group tests
// sphere pairs k, k + g, k + 2g, ... (src.pair) as v_pk_fma_f32 pairs
// (line_test_q's ops per element; the 7-op test). The pairs a wave reads
// at one step are g consecutive ones, the same g for every group: a
// broadcast, conflict-free LDS read, or coalesced lines. A step's flags
// go into a per-lane 32-bit mask (16 steps per round); each round's flagged
// spheres are resolved with the reference's ops (resolve_one), one per lane
// per iteration, and the group reduces (min c, then the largest index among
// equal c) with DPP: the in-order scan's answer (deferral).
// A non-finite root in a group sends its ray to the exact sequential path
// (`seq`). Per ray-segment this issues about as many instructions as a
// lane-mode segment (the scan's lane-ops are split, not repeated), at a
// fraction of its latency.
constexpr uint32_t kGfRays = 32;    // rays per chunk (g >= 2 lanes per ray; ws holds 32 rays + their results)
static_assert(kGfRays * 10 * sizeof(float) <= kCoopWaveBytes, "coop scratch: 8 floats per ray + 2 result words");
#ifndef RTX_GF_STEPS  // scan steps (2 spheres each) per resolve round: a 32-bit flag mask (stress build: 1)
#define RTX_GF_STEPS 16
#endif
constexpr uint32_t kGfSteps = RTX_GF_STEPS;
static_assert(kGfSteps >= 1 && kGfSteps <= 16, "flag mask: 2 bits per step in 32");
template <typename Src>
__device__ __forceinline__ int hit_world_groups(const KScene &S, const Src &src, uint64_t act, bool active, f3 o, f3 d,
                                                float a, float inv_a, float t_min, float *ws, float &best, bool &seq,
                                                unsigned long long *cp = nullptr, unsigned long long *tq = nullptr) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t m_all = (uint32_t)__popcll(act);
    const uint32_t rank_all =
        __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
    uint32_t *keys = reinterpret_cast<uint32_t *>(ws + 8 * kGfRays);  // [kGfRays][2]: the group results
    const float inf = __uint_as_float(0x7f800000u);
    int result = -1;
    seq = false;
#pragma unroll 1
    for (uint32_t c0 = 0; c0 < m_all; c0 += kGfRays) {
        const uint32_t m = min(m_all - c0, kGfRays);
        const bool mine = active && rank_all >= c0 && rank_all < c0 + m;
        const uint32_t rank = rank_all - c0;
        if (mine) {
            float *w = ws + 8 * rank;
            w[0] = o.x;
            w[1] = o.y;
            w[2] = o.z;
            w[3] = d.x;
            w[4] = d.y;
            w[5] = d.z;
            w[6] = a;
            w[7] = inv_a;
        }
        __builtin_amdgcn_wave_barrier();
        if (RTX_DIAG_COOP && cp && c0 == 0u) cp[5]++;
        RTX_CP(0)
        const uint32_t lg = m <= 1u ? 6u : 6u - (32u - (uint32_t)__builtin_clz(m - 1u));  // log2(g)
        const uint32_t g = 1u << lg;
        const uint32_t r = lane >> lg, k = lane & (g - 1u);
        const bool valid = r < m;
        const float *w = ws + 8 * (valid ? r : 0u);
        const f3 ro = mk3(w[0], w[1], w[2]), rd = mk3(w[3], w[4], w[5]);
        const float ra = w[6], ria = w[7];
        const LineTest T = line_test_setup(ro.x, ro.y, ro.z, rd.x, rd.y, rd.z, ra, S.smag);
        const f2v ux = {T.ux, T.ux}, uy = {T.uy, T.uy}, uz = {T.uz, T.uz}, vy = {T.vy, T.vy}, vz = {T.vz, T.vz};
        const f2v nou = {T.nou, T.nou}, nov = {T.nov, T.nov}, th = {T.thr, T.thr};
        uint64_t key = hit_key(inf, -1);
        bool ok = true;
        const uint32_t nsteps = valid ? (src.npairs + g - 1u) >> lg : 0u;
        const uint32_t plast = src.npairs - 1u;
#pragma unroll 1
        for (uint32_t s0 = 0; __ballot(s0 < nsteps) != 0ull; s0 += kGfSteps) {
            // scan: steps [s0, s1), pair p = st * g + k (spheres 2p, 2p + 1).
            // The NOT-flagged bits are shifted in (q - thr >= +0 exactly when
            // flagged, q finite): after the round, bit 2i + w of ~im is
            // sphere 2p + w of step s1 - 1 - i.
            uint32_t im = 0;
            const uint32_t s1 = min(s0 + kGfSteps, nsteps);
            auto step = [&](uint32_t st) {
                f2v cx, cy, cz, R;
                src.pair(Src::kPadded ? (st << lg) + k : min((st << lg) + k, plast), cx, cy, cz, R);
                const f2v pu = fma2(cx, ux, fma2(cy, uy, fma2(cz, uz, nou)));
                const f2v pv = fma2(cy, vy, fma2(cz, vz, nov));
                const f2v q = fma2(-pv, pv, fma2(-pu, pu, R)) - th;
                im = (im << 1) | (__float_as_uint(q.y) >> 31);
                im = (im << 1) | (__float_as_uint(q.x) >> 31);
            };
            uint32_t st = s0;
            for (; st + 2u <= s1; st += 2u) {
                step(st);
                step(st + 1u);
            }
            if (st < s1) step(st);
            const uint32_t nb = 2u * (s1 > s0 ? s1 - s0 : 0u);
            uint32_t fm = ~im & (nb >= 32u ? ~0u : ((1u << nb) - 1u));
            // resolve this round's flags, one sphere per lane per iteration
#pragma unroll 1
            while (__ballot(fm != 0u) != 0ull) {
                const bool live = fm != 0u;
                const uint32_t bit = live ? (uint32_t)__builtin_ctz(fm) : 0u;
                fm &= fm - 1u;
                const uint32_t p = ((s1 - 1u - (bit >> 1)) << lg) + k;
                const uint32_t j = 2u * (Src::kPadded ? p : min(p, plast)) + (bit & 1u);
                resolve_one(src.sphere(j), (int)j, live, ro, rd, ra, ria, t_min, key, ok);
            }
        }
        RTX_CP(1)
        // the group's (min c, then the largest index among equal c)
        const uint32_t cb0 = (uint32_t)(key >> 32);
        const uint32_t cb = group_reduce_u32<false>(cb0, lg);
        const uint32_t ib = group_reduce_u32<true>(cb0 == cb ? ~(uint32_t)key : 0u, lg);  // index + 1, 0: none
        const uint64_t badm = __ballot(!ok);
        if (valid && k == 0u) {
            const uint64_t gm = (g == 64u ? ~0ull : ((1ull << g) - 1ull)) << (r * g);
            keys[2 * r] = (badm & gm) != 0ull ? 0xffffffffu : ib;  // ~0: a non-finite root in the group
            keys[2 * r + 1] = cb;
        }
        __builtin_amdgcn_wave_barrier();
        RTX_CP(2)
        if (mine) {
            const uint32_t kb = keys[2 * rank], kc = keys[2 * rank + 1];
            if (kb == 0xffffffffu) {
                seq = true;
            } else if (kb != 0u) {
                const float c = __uint_as_float(kc);
                if (c <= best) {  // accepted iff c <= t_max
                    best = c;
                    result = (int)(kb - 1u);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();  // the next chunk reuses the LDS
    }
    return active ? result : -1;
}

// Group coop over the culled layout (large scenes: the frame tail, the
// heavy tiers, promoted pixels). Same chunks, ray exchange, reduction and
// `seq` rule as hit_world_groups; the scan is the culled one's hierarchy,
// split over the group's g lanes: lane k tests the group bounds (the top
// level, each over 64 spheres) k, k + g, ...; for a group its line passes,
// the lane tests the group's 8 block bounds, then the spheres of the blocks
// that pass, and resolves each flagged sphere on the spot (resolve_one:
// ccen and cperm by layout position). Lanes diverge inside a passing group;
// a ray's line passes ~2 % of the C5 scene's groups, so a 64-lane ray
// visits about one group per lane instead of scanning 1,563 spheres per
// lane. Bounds and spheres use the 7-op test (the margins cover it on
// flat blocks too, rtx_prefilter.h).
template <bool kBfs = true>
__device__ __forceinline__ int hit_world_groups_culled(const KScene &S, uint64_t act, bool active, f3 o, f3 d,
                                                       float a, float inv_a, float t_min, float *ws, float &best,
                                                       bool &seq) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t m_all = (uint32_t)__popcll(act);
    const uint32_t rank_all =
        __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
    uint32_t *keys = reinterpret_cast<uint32_t *>(ws + 8 * kGfRays);
    const float inf = __uint_as_float(0x7f800000u);
    const uint32_t nblk = S.n_cpad / 8u, ngrp = (nblk + 7u) / 8u;
    int result = -1;
    seq = false;
#pragma unroll 1
    for (uint32_t c0 = 0; c0 < m_all; c0 += kGfRays) {
        const uint32_t m = min(m_all - c0, kGfRays);
        const bool mine = active && rank_all >= c0 && rank_all < c0 + m;
        const uint32_t rank = rank_all - c0;
        if (mine) {
            float *w = ws + 8 * rank;
            w[0] = o.x;
            w[1] = o.y;
            w[2] = o.z;
            w[3] = d.x;
            w[4] = d.y;
            w[5] = d.z;
            w[6] = a;
            w[7] = inv_a;
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t lg = m <= 1u ? 6u : 6u - (32u - (uint32_t)__builtin_clz(m - 1u));  // log2(g)
        const uint32_t g = 1u << lg;
        const uint32_t r = lane >> lg, k = lane & (g - 1u);
        const bool valid = r < m;
        const float *w = ws + 8 * (valid ? r : 0u);
        const f3 ro = mk3(w[0], w[1], w[2]), rd = mk3(w[3], w[4], w[5]);
        const float ra = w[6], ria = w[7];
        const LineTest T = line_test_setup(ro.x, ro.y, ro.z, rd.x, rd.y, rd.z, ra, S.smag);
        const LineTest Ts = line_test_stretched(S, ro, rd);  // the flat bounds' space (kCullSy)
        const float thr_b = T.thr * kCullThrScale, thr_bs = Ts.thr * kCullThrScaleSy;
        const HalfTest H = half_test_setup(ro.x, ro.y, ro.z, rd.x, rd.y, rd.z, ra, thr_b, t_min);
        const HalfTest Hs = half_test_stretched(ro, rd, thr_bs, t_min);
        // bit j: entry j of an AoSoA-8 block (bounds or spheres) passes Q >= thr, the 7-op test of line L;
        // for bounds (Hh) also the half test
        auto block_mask = [&](const float *blk, const LineTest &L, float thr,
                              const HalfTest *Hh = nullptr) -> uint32_t {
            const f2v ux = {L.ux, L.ux}, uy = {L.uy, L.uy}, uz = {L.uz, L.uz}, vy = {L.vy, L.vy}, vz = {L.vz, L.vz};
            const f2v nou = {L.nou, L.nou}, nov = {L.nov, L.nov};
            const float4 *b4 = reinterpret_cast<const float4 *>(blk);
            float4 v[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) v[t] = b4[t];
            uint32_t msk = 0;
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const float4 X = v[p >> 1], Y = v[2 + (p >> 1)], Z = v[4 + (p >> 1)], Rr = v[6 + (p >> 1)];
                const bool hi = p & 1;
                const f2v cx = {hi ? X.z : X.x, hi ? X.w : X.y}, cy = {hi ? Y.z : Y.x, hi ? Y.w : Y.y};
                const f2v cz = {hi ? Z.z : Z.x, hi ? Z.w : Z.y}, R = {hi ? Rr.z : Rr.x, hi ? Rr.w : Rr.y};
                const f2v pu = fma2(cx, ux, fma2(cy, uy, fma2(cz, uz, nou)));
                const f2v pv = fma2(cy, vy, fma2(cz, vz, nov));
                const f2v q = fma2(-pv, pv, fma2(-pu, pu, R));
                bool px = !(q.x < thr), py = !(q.y < thr);
                if (RTX_CULL_HALF && Hh) {
                    const f2v hdx = {Hh->dx, Hh->dx}, hdy = {Hh->dy, Hh->dy}, hdz = {Hh->dz, Hh->dz};
                    const f2v hnod = {Hh->nod, Hh->nod}, ha = {Hh->a, Hh->a}, htha = {Hh->tha, Hh->tha};
                    const f2v pw = fma2(cx, hdx, fma2(cy, hdy, fma2(cz, hdz, hnod)));
                    const f2v q2 = fma2(-pw, pw, fma2(R, ha, htha));
                    px = px && half_test_pass(pw.x, q2.x);
                    py = py && half_test_pass(pw.y, q2.y);
                }
                msk |= (px ? 1u : 0u) << (2 * p);
                msk |= (py ? 1u : 0u) << (2 * p + 1);
            }
            return msk;
        };
        // one bound (7-op order), line and half test
        auto bound_pass = [&](const float *q, bool flat) -> bool {
            const LineTest &L = flat ? Ts : T;
            const HalfTest &Hh = flat ? Hs : H;
            if (line_test_q(L, q[0], q[8], q[16], q[24]) < (flat ? thr_bs : thr_b)) return false;
            if (!RTX_CULL_HALF) return true;
            const float pw = half_test_pw(Hh, q[0], q[8], q[16]);
            return half_test_pass(pw, half_test_q2(Hh, pw, q[24]));
        };
        uint64_t key = hit_key(inf, -1);
        bool ok = true;
        // 8 bounds whose entries cover blocks from b0 on (flat, i.e. stretched,
        // iff b0 >= cflat_lo: no test straddles it)
        auto bounds_mask = [&](const float *blk, uint32_t b0) -> uint32_t {
            return b0 >= S.cflat_lo ? block_mask(blk, Ts, thr_bs, &Hs) : block_mask(blk, T, thr_b, &H);
        };
        auto first_bits = [](uint32_t n) { return n >= 8u ? 0xffu : (1u << n) - 1u; };
        const uint32_t nsg = (ngrp + 7u) / 8u;
        if (kBfs && m == 1u && RTX_CULL_BFS) {
            // One ray, the whole wave: breadth first. Each level's passing
            // entries are expanded 8 at a time, one child per lane (entry e's
            // bound at (AoSoA-8) floats 32 (e >> 3) + (e & 7) + {0, 8, 16, 24}),
            // so a level costs one round of loads for the wave instead of a
            // lane walking its subtree load after dependent load.
            auto test_entry = [&](const float *arr, uint32_t e, bool flat) {
                return bound_pass(arr + 32u * (e >> 3) + (e & 7u), flat);
            };
            auto test_sphere = [&](uint32_t pos) {
                const float *q = S.cpre + 32u * (pos >> 3) + (pos & 7u);
                if (line_test_q(T, q[0], q[8], q[16], q[24]) < T.thr) return false;
                if (!RTX_CULL_HALF_SPHERES) return true;
                const float pw = half_test_pw(H, q[0], q[8], q[16]);
                return half_test_pass(pw, half_test_q2(H, pw, q[24]));
            };
            // the child this lane takes: of the (lane >> 3)-th set bit of the
            // uniform mask m (the next 8 set bits are consumed)
            auto take8 = [&](uint64_t &mm, uint32_t &parent) -> bool {
                uint32_t sel = ~0u;
#pragma unroll
                for (uint32_t j = 0; j < 8u; ++j) {
                    const uint32_t bit = mm != 0ull ? (uint32_t)__builtin_ctzll(mm) : ~0u;
                    if (mm != 0ull) mm &= mm - 1ull;
                    if ((lane >> 3) == j) sel = bit;
                }
                parent = sel;
                return sel != ~0u;
            };
#pragma unroll 1
            for (uint32_t base = 0; base < nsg; base += 64u) {
                const uint32_t si = base + lane;
                uint64_t m3 = __ballot(si < nsg && (RTX_CULL_LEVELS < 3 ||
                                                    test_entry(S.cbnd3, si, 64u * si >= S.cflat_lo)));
#pragma unroll 1
                while (m3 != 0ull) {
                    uint32_t ps;
                    const bool h3 = take8(m3, ps);
                    const uint32_t gi = h3 ? 8u * (base + ps) + (lane & 7u) : 0u;
                    uint64_t m2 = __ballot(h3 && gi < ngrp &&
                                           test_entry(S.cbnd2, gi, 8u * gi >= S.cflat_lo));
#pragma unroll 1
                    while (m2 != 0ull) {
                        uint32_t pg;
                        const bool h2 = take8(m2, pg);
                        // pg: a lane index of the level above, i.e. group 8 (base + ps') + (pg & 7) of that lane's
                        // super-group: recover the group from the lane that tested it
                        const uint32_t gsel = (uint32_t)__shfl((int)gi, (int)(h2 ? pg : 0u), 64);
                        const uint32_t bb = h2 ? 8u * gsel + (lane & 7u) : 0u;
                        uint64_t m1 = __ballot(h2 && bb < nblk && test_entry(S.cbnd, bb, bb >= S.cflat_lo));
#pragma unroll 1
                        while (m1 != 0ull) {
                            uint32_t pb;
                            const bool h1 = take8(m1, pb);
                            const uint32_t bsel = (uint32_t)__shfl((int)bb, (int)(h1 ? pb : 0u), 64);
                            const uint32_t pos = h1 ? 8u * bsel + (lane & 7u) : 0u;
                            const bool fl = h1 && test_sphere(pos);
                            if (fl) resolve_one(S.ccen[pos], (int)S.cperm[pos], true, ro, rd, ra, ria, t_min, key, ok);
                        }
                    }
                }
            }
        } else {
        const uint32_t nsteps = valid ? (nsg + g - 1u) >> lg : 0u;
#pragma unroll 1
        for (uint32_t st = 0; st < nsteps; ++st) {
            const uint32_t si = (st << lg) + k;  // super-group si: its bound (512 spheres) in cbnd3
            if (si >= nsg) break;
            const float *sb = S.cbnd3 + 32u * (si >> 3) + (si & 7u);
            if (RTX_CULL_LEVELS >= 3 && !bound_pass(sb, 64u * si >= S.cflat_lo)) continue;
            uint32_t mg = bounds_mask(S.cbnd2 + 32u * si, 64u * si) & first_bits(ngrp - 8u * si);
#pragma unroll 1
            while (mg != 0u) {
                const uint32_t gi = 8u * si + (uint32_t)__builtin_ctz(mg);
                mg &= mg - 1u;
                uint32_t mb = bounds_mask(S.cbnd + 32u * gi, 8u * gi) & first_bits(nblk - 8u * gi);
#pragma unroll 1
                while (mb != 0u) {
                    const uint32_t bb = 8u * gi + (uint32_t)__builtin_ctz(mb);
                    mb &= mb - 1u;
                    uint32_t ms = block_mask(S.cpre + 32u * bb, T, T.thr, RTX_CULL_HALF_SPHERES ? &H : nullptr);
#pragma unroll 1
                    while (ms != 0u) {
                        const uint32_t pos = 8u * bb + (uint32_t)__builtin_ctz(ms);
                        ms &= ms - 1u;
                        resolve_one(S.ccen[pos], (int)S.cperm[pos], true, ro, rd, ra, ria, t_min, key, ok);
                    }
                }
            }
        }
        }
        // the group's (min c, then the largest index among equal c)
        const uint32_t cb0 = (uint32_t)(key >> 32);
        const uint32_t cb = group_reduce_u32<false>(cb0, lg);
        const uint32_t ib = group_reduce_u32<true>(cb0 == cb ? ~(uint32_t)key : 0u, lg);  // index + 1, 0: none
        const uint64_t badm = __ballot(!ok);
        if (valid && k == 0u) {
            const uint64_t gm = (g == 64u ? ~0ull : ((1ull << g) - 1ull)) << (r * g);
            keys[2 * r] = (badm & gm) != 0ull ? 0xffffffffu : ib;  // ~0: a non-finite root in the group
            keys[2 * r + 1] = cb;
        }
        __builtin_amdgcn_wave_barrier();
        if (mine) {
            const uint32_t kb = keys[2 * rank], kc = keys[2 * rank + 1];
            if (kb == 0xffffffffu) {
                seq = true;
            } else if (kb != 0u) {
                const float c = __uint_as_float(kc);
                if (c <= best) {  // accepted iff c <= t_max
                    best = c;
                    result = (int)(kb - 1u);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();  // the next chunk reuses the LDS
    }
    return active ? result : -1;
}

#ifndef RTX_PROM_EXACT_RATE  // A/B: a restarted pixel's promotion rate over its samples from 0 (1) or from cost_spp (0)
#define RTX_PROM_EXACT_RATE 1
#endif
// Lane state: the pixel it is tracing and that pixel's current path.
constexpr uint32_t kSeg0Restart = 0x80000000u;  // Lane::seg0 flag (a lane's segs stay far below 2^31)
struct Lane {
    f3 o, d, col, acc;
    float a, inv_a, seed;
    uint32_t sample, bounce, segs;
    uint32_t x, y, gid;  // pixel (global image coords) and its output slot
    uint32_t slot;       // its pixel-queue slot (priority of the heaviest pixels' waves)
    uint32_t seg0;       // segs when the pixel started (cost pre-pass: per-pixel segments);
                         // kSeg0Restart: the render restarted it from sample 0 (cost_cap)
    uint32_t c0;         // the pre-pass's segments of a resumed pixel (dynamic priority; else 0)
    bool active;         // tracing a pixel
    uint32_t cb, ce;     // the wave's private run of queue slots (refill; wave-uniform)
};

__device__ __forceinline__ void set_dir(Lane &L, f3 d) {
    L.d = d;
    L.a = dir_len2(d);
    L.inv_a = 1.0f / L.a;
}

__device__ __forceinline__ float pixel_seed(const KParams &P, uint32_t x, uint32_t y, uint32_t s) {
    // Reference: p = float(baseHash(DTid.xy)) / float(0xffffffffU)  (:295)
    uint32_t h = base_hash(x, y);
    if (P.rng_mode == 1u)  // per-sample re-seed (extension)
        h = base_hash(h, P.frame_index * P.spp + s);
    else if (P.frame_index != 0u)  // progressive frames (extension)
        h = base_hash(h, 0x80000000u | P.frame_index);
    return (float)h / 4294967296.0f;
}

__device__ __forceinline__ void begin_sample(const KParams &P, const Frame &F, uint32_t x, uint32_t y,
                                             Lane &L) {
    if (P.rng_mode == 1u) L.seed = pixel_seed(P, x, y, L.sample);
    f3 o, d;
    start_sample(F, x, y, L.seed, o, d);
    L.o = o;
    set_dir(L, d);
    L.col = mk3(1.0f, 1.0f, 1.0f);
    L.bounce = 0;
}

// accColor /= spp; toGamma; float4(c, 1) (:312-314) for local pixel gid,
// whose linear sample sum is `sum`. `slot`: the pixel's queue slot in a
// cost-ordered render with a slot-ordered staging image (KParams::out_slot):
// the pixel goes to out_slot[slot] and k_unpermute moves it to out[gid] with
// coalesced stores; ~0u (or no staging): straight to out[gid].
__device__ __forceinline__ void output_pixel(const KParams &P, uint32_t gid, f3 sum, uint32_t slot = ~0u) {
    float n = (float)P.spp;
    if (P.accum) {  // progressive: running linear sum over frames
        float4 a = P.accum[gid];
        a.x = a.x + sum.x;
        a.y = a.y + sum.y;
        a.z = a.z + sum.z;
        P.accum[gid] = a;
        sum = mk3(a.x, a.y, a.z);
        n = (float)(P.accum_frames * P.spp);
    }
    float4 o;
    o.x = to_gamma(sum.x / n);
    o.y = to_gamma(sum.y / n);
    o.z = to_gamma(sum.z / n);
    o.w = 1.0f;
    if (P.out_slot && slot != ~0u) {
        o.w = __uint_as_float(P.stage_tag);  // this launch's staged pixel (k_unpermute writes w = 1)
        P.out_slot[slot] = o;
    } else {
        P.out[gid] = o;
    }
}

#ifndef RTX_EXTRA_BYTES
#define RTX_EXTRA_BYTES 0
#endif
// A pixel's output (output_pixel), or the scheduling pre-pass's record of it.
template <bool kCost = false>
__device__ __forceinline__ void write_pixel(const KParams &P, const Lane &L) {
    if constexpr (kCost) {  // scheduling pre-pass: record the pixel's segments
        P.cost_out[L.gid] = L.segs - L.seg0;
        // and its state after these samples: the render resumes from it
        if (P.state) P.state[L.gid] = make_float4(L.acc.x, L.acc.y, L.acc.z, L.seed);
        return;
    }
    output_pixel(P, L.gid, L.acc, L.slot);
    // A/B build (HBM traffic): the pixel's final state also
    // goes back to its (dead) resume slot: +16 B per pixel of the same
    // scattered cost-order stores as the image
    if (RTX_EXTRA_BYTES && P.state) P.state[L.gid] = make_float4(L.acc.x, L.acc.y, L.acc.z, L.seed);
}

// Diffuse direction before normalisation, target - p (ShaderCompute.hlsl:
// 211-212), with the optional near-zero guard (RTX_FRAME_LAMBERT_GUARD,
// §8f-4): the prototype's lambert (Shader_RT.fx:222-225) with the compute
// shader's unused near_zero (ShaderCompute.hlsl:70-74, s = 1e-9).
__device__ __forceinline__ f3 lambert_guard(f3 v, f3 nrm, bool guard) {
    const float s = 0.000000001f;
    const bool nz = fabsf(v.x) < s && fabsf(v.y) < s && fabsf(v.z) < s;
    return guard && nz ? nrm : v;
}

// One finished hit_world call of sample_color (:262-284). On a hit, scatter
// (:207-252) moves the lane's ray (o, d, a, inv_a) and multiplies col by the
// attenuation; the path goes on unless the material does not scatter or the
// depth is exhausted (black, :286). On a miss, `sky_col` = col * the sky
// gradient (:279-283), the sample's colour. LaneT: any lane state with o, d,
// a, inv_a, col, seed, bounce (Lane, PsLane).
enum { kSegContinue = 0, kSegSky = 1, kSegBlack = 2 };
// A wave's lanes take different branches here (sky, Lambert/metal,
// dielectric) and every branch with a live lane costs the whole wave, so the
// operations the branches have in common run once, for all the lanes that
// need them, each lane still executing exactly the HLSL's op sequence:
//  * normalize(d): the sky (:281) and the dielectric (:231);
//  * one hash step: random_in_unit_sphere's hash3 (:60) and the dielectric's
//    hash1 (:241) each consume exactly one `float2(seed += .1, seed += .1)`
//    and baseHash of it; the lane then converts the hash as its call would;
//  * sqrt(1 - x*x): random_in_unit_sphere's sqrt(1 - h.x^2) (:63) and the
//    dielectric's sin_theta = sqrt(1 - cos_theta^2) (:234).
// The seed-determined part of a Lambert/metal scatter (random_in_unit_sphere,
// :59-66): the hash step and everything computed from it before the hit is
// known — the wave-wide pixel trace (trace_pixel_wave) evaluates it before
// the scan, off the segment's critical path. The same ops as path_segment's
// own evaluation, so the same bits; discarded when the segment does not
// scatter (the seed then does not advance).
struct ScatterSpec {
    float seed;   // after the hash step
    uint32_t hn;  // the step's baseHash
    float hx, sq, r, sn, cs;
};
__device__ __forceinline__ ScatterSpec scatter_spec(float seed) {
    ScatterSpec s;
    s.seed = seed;
    s.hn = hash_step(s.seed);
    s.hx = ((float)(s.hn & 0x7fffffffu) / 2147483648.0f) * 2.0f - 1.0f;
    const float phi = ((float)((s.hn * 16807u) & 0x7fffffffu) / 2147483648.0f) * 6.28318530718f;
    const float hz = (float)((s.hn * 48271u) & 0x7fffffffu) / 2147483648.0f;
    s.sq = sqrt_rn(1.0f - s.hx * s.hx);
    s.r = pow_rt(hz, 0.333333333f);
    sincos_rt(phi, s.sn, s.cs);
    return s;
}

// The hit sphere's record inputs: (centre, radius), material code, values.
struct HitMat {
    float4 sc;
    int mt;
    float4 mv;
};
__device__ __forceinline__ HitMat hit_mat(const KScene &S, int hit) {
    HitMat m;
    m.sc = S.cen[hit];
    m.mt = S.mtype[hit];
    m.mv = S.mval[hit];
    return m;
}

// path_segment with the hit's record inputs given (hit >= 0; M unused on a
// miss) and, with kSpec, the scatter's seed-determined part precomputed.
template <bool kSpec, typename LaneT>
__device__ __forceinline__ int path_segment_m(const KParams &P, LaneT &L, int hit, float t, const HitMat &M,
                                              const ScatterSpec &sp, f3 &sky_col) {
    int mt = 3;
    f3 p = L.o, nrm = L.d;
    bool ff = false;
    float4 mv = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (hit >= 0) {
        const float4 sc = M.sc;
        p = L.o + t * L.d;                             // Ray::at, Ray.h:16-19
        const float inv_r = 1.0f / sc.w;               // Vec3 operator/, Vec3.h:83-86
        nrm = inv_r * (p - mk3(sc.x, sc.y, sc.z));     // Sphere.cpp:28
        ff = dot3(L.d, nrm) < 0.0f;                    // set_face_normal, :143-150
        if (!ff) nrm = -nrm;
        mt = M.mt;
        mv = M.mv;
    }
    const bool sky = hit < 0;
    const bool diel = !sky && mt == 2;
    f3 ud = L.d;
    if (sky || diel) ud = normalize3(L.d);
    if (sky) {
        const float tt = 0.5f * (ud.y + 1.0f);
        const float w = 1.0f - tt;
        const f3 sk = mk3(w + tt * 0.5f, w + tt * 0.7f, w + tt);
        sky_col = L.col * sk;
        return kSegSky;
    }
    if (mt != 0 && mt != 1 && !diel) return kSegBlack;  // unknown material: sample is black (:251, :274)
    uint32_t hn;
    if constexpr (kSpec) {
        hn = sp.hn;
        L.seed = sp.seed;
    } else {
        hn = hash_step(L.seed);
    }
    float x, cosine = 0.0f, ratio = 0.0f, hx = 0.0f, phi = 0.0f, hz = 0.0f;
    if (diel) {  // DIELECTRIC (:229-249), atten = 1
        ratio = ff ? (1.0f / mv.w) : mv.w;
        cosine = fminf(dot3(-ud, nrm), 1.0f);
        x = cosine;
    } else if constexpr (!kSpec) {  // random_in_unit_sphere's hash3 (:43-48, :59-66)
        hx = ((float)(hn & 0x7fffffffu) / 2147483648.0f) * 2.0f - 1.0f;
        phi = ((float)((hn * 16807u) & 0x7fffffffu) / 2147483648.0f) * 6.28318530718f;
        hz = (float)((hn * 48271u) & 0x7fffffffu) / 2147483648.0f;
        x = hx;
    } else {
        x = sp.hx;
    }
    const float sq = (kSpec && !diel) ? sp.sq : sqrt_rn(1.0f - x * x);
    f3 dir;
    if (diel) {
        const bool cant = ratio * sq > 1.0f;
        // FXC's `||` does not short-circuit: hash1 always advances the seed.
        const float refl = reflectance(cosine, ratio);
        const float h = (float)hn / 4294967296.0f;  // hash1 (:30-34)
        dir = (cant || refl > h) ? reflect3(ud, nrm) : refract3(ud, nrm, ratio);
    } else {
        // Lambert and metal share random_in_unit_sphere and normalize: run
        // them once for both kinds of lane (each lane's ops are the HLSL's).
        float r, sn, cs;
        if constexpr (kSpec) {
            r = sp.r;
            sn = sp.sn;
            cs = sp.cs;
            hx = sp.hx;
        } else {
            r = pow_rt(hz, 0.333333333f);
            sincos_rt(phi, sn, cs);
        }
        const f3 rius = f3{r * (sq * sn), r * (sq * cs), r * hx};
        const f3 v = mt == 0 ? ((p + nrm) + rius) - p                // DIFFUSE (:209-217)
                             : reflect3(L.d, nrm) + mv.w * rius;     // METAL (:219-227)
        dir = normalize3(lambert_guard(v, nrm, mt == 0 && (P.flags & kFrameLambertGuard) != 0u));
        L.col = L.col * mk3(mv.x, mv.y, mv.z);
    }
    L.o = p;
    L.d = dir;
    L.a = dir_len2(dir);
    L.inv_a = 1.0f / L.a;
    L.bounce++;
    return L.bounce >= P.depth ? kSegBlack : kSegContinue;  // depth exhausted -> black (:286)
}
template <typename LaneT>
__device__ __forceinline__ int path_segment(const KParams &P, LaneT &L, int hit, float t, f3 &sky_col) {
    HitMat M;
    if (hit >= 0) M = hit_mat(P.scene, hit);
    return path_segment_m<false>(P, L, hit, t, M, ScatterSpec{}, sky_col);
}

// Cross-XCD hand-off without cache maintenance. On gfx950 an agent-scope
// release writes back the issuing XCD's L2 (buffer_wbl2) and an acquire
// invalidates it (buffer_inv): issued per iteration they evict the scene and
// queue lines of every k_render wave on that XCD (parts 8 with promotion on:
// 15 -> 38 ms). Relaxed agent-scope loads and stores are already
// coherent across XCDs (sc1: they bypass the non-coherent L2 state), so the
// hand-off only needs the stores to complete in order: wait for every
// outstanding vector-memory operation (vmcnt 0) before the flag store, and
// keep the compiler from moving atomics across the wait.
__device__ __forceinline__ void agent_store_order() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt/lgkmcnt unconstrained (gfx9 encoding)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// Promotion (KParams::prom): once the queue is exhausted, a lane whose pixel
// is projected, at a sample boundary, to need more than prom_min further
// segments (its own rate so far in this launch times the samples left) hands
// the pixel's state (gid, sample, seed, acc) to the promotion queue and goes
// idle; a wave with nothing else to do (an idle k_render wave, or k_trace
// after tier 1) traces the rest of the pixel with all its lanes. Entries are
// published with agent-scope atomics (the consumer may sit on another XCD,
// whose L2 does not see these stores otherwise): the fields, a wait for their
// completion, then the epoch word (agent_store_order).
__device__ __forceinline__ bool promote(const KParams &P, const Lane &L, uint32_t min_segs) {
    // samples traced in this launch (>= 1 here): after the pre-pass's
    // cost_spp, or from sample 0 for a pixel the pre-pass stopped (cost_cap;
    // kSeg0Restart in seg0)
    const bool restarted = RTX_PROM_EXACT_RATE && (L.seg0 & kSeg0Restart) != 0u;
    const uint32_t done = max(restarted ? L.sample : L.sample - min(L.sample, P.cost_spp), 1u);
    const uint32_t segs = L.segs - (L.seg0 & ~kSeg0Restart);
    if ((uint64_t)segs * (P.spp - L.sample) <= (uint64_t)min_segs * done) return false;
    const uint32_t slot = atomicAdd(&P.prom[0], 1u);
    if (slot >= P.prom_cap) return false;  // queue full: the lane keeps its pixel
    // whoever finishes a promoted pixel writes it to out[gid] directly: its
    // staging slot says so (w = 0; an output pixel's w is 1), k_unpermute skips it
    if (P.out_slot && L.slot != ~0u) P.out_slot[L.slot] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    uint32_t *e = P.prom_q + 8u * slot;
    __hip_atomic_store(e + 0, L.gid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(e + 1, L.sample, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(e + 2, __float_as_uint(L.seed), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(e + 3, __float_as_uint(L.acc.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(e + 4, __float_as_uint(L.acc.y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(e + 5, __float_as_uint(L.acc.z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    agent_store_order();
    __hip_atomic_store(e + 7, P.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// Chain-RNG lane: one segment, then the pixel's next sample when the path
// ends (acc += colour in sample order, :269-284), or the pixel's output
// after its last sample (clears `active`). prom_thr (0: none): promote the
// pixel at a sample boundary if it is projected to need more segments than
// this (KParams::prom_min once the wave's queue is exhausted). Returns true
// when the pixel was promoted.
template <bool kCost = false>
__device__ __forceinline__ bool shade(const KParams &P, const Frame &F, Lane &L, int hit, float t,
                                      uint32_t prom_thr = 0u) {
    L.segs++;
    f3 c;
    const int r = path_segment(P, L, hit, t, c);
    if (r == kSegSky) L.acc = L.acc + c;
    const bool ended = r != kSegContinue;
    if (ended) {
        L.sample++;
        if (L.sample >= P.spp) {
            write_pixel<kCost>(P, L);
            L.active = false;
            diag_pixel_end(P, L.gid);
        } else if (!kCost && prom_thr != 0u && promote(P, L, prom_thr)) {
            L.active = false;  // the promotion queue owns the pixel now
            return true;
        } else {
            begin_sample(P, F, L.x, L.y, L);
        }
    } else if (kCost && P.cost_cap != 0u && L.segs - L.seg0 >= P.cost_cap) {
        // pre-pass: a pixel this long is heavy whatever its remaining
        // samples cost; it stops here (its key: the cap) and the render
        // traces it from sample 0 (state seed NaN). Its segments so far are
        // not counted: the render redoes them with the same operations.
        P.cost_out[L.gid] = P.cost_capped;
        P.state[L.gid] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(0x7fc00000u));
        L.segs = L.seg0;
        L.active = false;
        diag_pixel_end(P, L.gid);
    }
    return false;
}

__device__ __forceinline__ void lane_pixel(const KParams &P, uint32_t gid, uint32_t &x, uint32_t &y) {
    const uint32_t lr = gid / P.width;  // local row
    x = gid - lr * P.width;
    const uint32_t j = lr / P.tile_rows;
    const uint32_t w = lr - j * P.tile_rows;
    y = (j * P.nparts + P.part) * P.tile_rows + w;
}

// Segment counter: wave sum, one 64-bit atomic per wave.
__device__ __forceinline__ void count_segments(const KParams &P, uint32_t segs) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) segs += __shfl_xor(segs, off, 64);
    if ((threadIdx.x & 63u) == 0u && segs != 0u) atomicAdd(P.counters, (unsigned long long)segs);
}

// The kernel's frame token (start_sample reads the constants through
// frame_vals). frame_vals assumes the kernarg segment begins with the
// kernel's KParams; the check build (RTX_CHECK_KERNARG, on in the stress
// build the GPU tests run) compares what it reads there with `P` — the
// kernel's own argument at every call site — and flags the launch
// (kErrKernarg: rtx_sync / rtx_get_stats report it) if a kernel ever breaks
// that layout.
#ifndef RTX_CHECK_KERNARG
#define RTX_CHECK_KERNARG 0
#endif
__device__ __forceinline__ Frame load_frame(const KParams &P) {
    if constexpr (RTX_CHECK_KERNARG != 0) {
        const FrameVals v = frame_vals();
        const bool same = __float_as_uint(v.img_w) == __float_as_uint(P.img_w) &&
                          __float_as_uint(v.img_h) == __float_as_uint(P.img_h) &&
                          __float_as_uint(v.org.x) == __float_as_uint(P.org[0]) &&
                          __float_as_uint(v.llc.z) == __float_as_uint(P.llc[2]) &&
                          __float_as_uint(v.lens_r) == __float_as_uint(P.lens_r);
        if (!same && P.errors && (threadIdx.x & 63u) == 0u) atomicOr(P.errors, kErrKernarg);
    }
    return Frame{};
}

// Start pixel `gid` (local index of this launch's rows) on this lane.
// Launches with spp == 0 or depth == 0 never get here (k_render_trivial).
__device__ __forceinline__ void start_pixel(const KParams &P, const Frame &F, uint32_t gid, Lane &L) {
    L.gid = gid;
    lane_pixel(P, gid, L.x, L.y);
    L.seg0 = L.segs;
    const float4 st = P.state && !P.cost_out ? P.state[gid] : make_float4(0.f, 0.f, 0.f, 0.f);
    L.c0 = 0u;
    if (P.state && !P.cost_out && !__builtin_isnan(st.w)) {  // after the pre-pass's cost_spp samples (identical state)
        L.acc = mk3(st.x, st.y, st.z);
        L.sample = P.cost_spp;
        L.seed = st.w;
        if (P.cost_in) L.c0 = P.cost_in[gid];
    } else {  // a fresh pixel, or one the pre-pass stopped (cost_cap)
        L.acc = mk3(0.0f, 0.0f, 0.0f);
        L.sample = 0;
        L.seed = pixel_seed(P, L.x, L.y, 0);
        if (P.state && !P.cost_out) L.seg0 |= kSeg0Restart;  // promote() counts its samples from 0
    }
    L.active = true;
    begin_sample(P, F, L.x, L.y, L);
}

// s_setprio takes an immediate: a wave-uniform priority 0..3 by branch.
__device__ __forceinline__ void set_prio(uint32_t p) {
    switch (__builtin_amdgcn_readfirstlane(p)) {
        case 0: __builtin_amdgcn_s_setprio(0); break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        default: __builtin_amdgcn_s_setprio(3); break;
    }
}

// Dynamic lane-mode wave priority (KParams::cost_in, rtx_schedule.prio_bar*):
// the wave's longest projected remaining chain (segments per sample so far,
// the pre-pass's included, times the samples left) against the bars x the
// mean pixel's segments m; a pixel the pre-pass stopped counts as long until
// its first sample ends.
__device__ __forceinline__ uint32_t dyn_level(const KParams &P, const Lane &L, float m) {
    float rem = 0.0f;
    if (L.active) {
        const bool rs = (L.seg0 & kSeg0Restart) != 0u;
        const float segs = (float)(L.segs - (L.seg0 & ~kSeg0Restart) + L.c0);
        rem = rs && L.sample == 0u ? 3.0e38f : segs * (float)(P.spp - L.sample) / (float)max(L.sample, 1u);
    }
    return __ballot(rem > P.dyn_bar[2] * m) != 0ull   ? 3u
           : __ballot(rem > P.dyn_bar[1] * m) != 0ull ? 2u
           : __ballot(rem > P.dyn_bar[0] * m) != 0ull ? 1u
                                                      : 0u;
}

// Persistent-lane pixel queue: every idle lane of the wave takes the next
// slot of [lo, hi) (the queue counter counts from lo); ONE atomic per wave
// per refill (ballot + lane rank). Returns true once the queue is
// exhausted (wave-uniform).
__device__ __forceinline__ bool refill(const KParams &P, const Frame &F, uint32_t lo, uint32_t hi, Lane &L) {
    const uint64_t idle = __ballot(!L.active);
    if (idle == 0ull) return false;
    const uint32_t cnt = (uint32_t)__popcll(idle);
    if (P.chunk > 1u) {
        // The wave's idle lanes take consecutive slots of a private run
        // [cb, ce) of the queue, re-stocked P.chunk slots at a time, so that
        // its lanes hold pixels from few runs of the cost order (coherent
        // rays) instead of one slot per refill from wherever the queue head
        // is. Slot by slot for the last eighth of the queue (no pixel waits
        // in a busy wave's run while other waves are idle).
        const uint32_t lane = threadIdx.x & 63u;
        const uint32_t rank = (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
        const uint32_t avail = L.ce - L.cb;
        uint32_t nb = 0, n = 0;
        if (cnt > avail) {
            n = cnt - avail;
            if (L.cb < hi - (hi - lo) / 8u) n = max(n, P.chunk);
            if (lane == 0u) nb = atomicAdd(P.queue, n);
            nb = lo + (uint32_t)__shfl((int)nb, 0, 64);
        }
        if (!L.active) {
            const uint32_t g = rank < avail ? L.cb + rank : nb + (rank - avail);
            if (g < hi) {
                start_pixel(P, F, P.perm ? P.perm[g] : g, L);
                L.slot = g;
                diag_pixel_start(P, L.gid, 0);
            }
        }
        if (cnt > avail) {
            L.cb = nb + (cnt - avail);
            L.ce = min(nb + n, hi);
            return L.cb >= hi;
        }
        L.cb += cnt;
        return false;
    }
    const int leader = __ffsll((long long)idle) - 1;
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t base = 0;
    if ((int)lane == leader) base = atomicAdd(P.queue, cnt);
    base = lo + __shfl(base, leader, 64);
    if (!L.active) {
        const uint32_t g = base + (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
        if (g < hi) {
            start_pixel(P, F, P.perm ? P.perm[g] : g, L);
            L.slot = g;
            diag_pixel_start(P, L.gid, 0);
        }
    }
    return base + cnt >= hi;
}

// Heavy pixels (the front of the cost-ordered queue, k_heavy_split) are
// the frame's critical path: a pixel's samples are sequential (the
// reference's RNG chain), so a pixel that costs more segments than a lane's
// share of the frame cannot finish in lane mode however early it starts.
// They are traced in group-coop mode (hit_world_groups), at a raised wave
// priority, in two tiers: tier 1 = slots [0, k1), the very heaviest, up to
// kHeavy1 per wave (64 / kHeavy1 lanes per ray: the shortest time per
// segment); tier 2 = slots [k1, kh), up to kHeavy2 per wave. An idle wave
// tries tier 1 first; a tier-2 wave tops itself up from tier 2. Returns the
// wave's tier (0: not heavy any more).
struct HeavyState {
    uint32_t k1, kh;     // tier ends
    bool t1_done, t2_done;
    uint32_t tier;       // 1, 2, or 0 (normal wave)
};
__device__ __forceinline__ bool take_from(const KParams &P, const Frame &F, uint32_t *ctr, uint32_t lo, uint32_t hi,
                                          uint32_t room, uint64_t act, Lane &L, bool &done) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t h = 0;
    if (lane == 0u) h = atomicAdd(ctr, room);
    h = lo + __shfl(h, 0, 64);
    if (h >= hi) {
        done = true;
        return false;
    }
    const uint32_t take = min(room, hi - h);
    const uint32_t rk = (uint32_t)__popcll(~act & ((1ull << lane) - 1ull));
    if (!L.active && rk < take) {
        start_pixel(P, F, P.perm[h + rk], L);
        L.slot = h + rk;
        diag_pixel_start(P, L.gid, ctr == P.heavy ? 1ull : 2ull);
    }
    if (h + room >= hi) done = true;
    return true;
}
__device__ __forceinline__ void take_heavy(const KParams &P, const Frame &F, HeavyState &H, Lane &L) {
    const uint64_t act = __ballot(L.active);
    const uint32_t have = (uint32_t)__popcll(act);
    if (have == 0u) H.tier = 0;
    if (have == 0u && !H.t1_done && take_from(P, F, P.heavy, 0, H.k1, kHeavy1, act, L, H.t1_done)) {
        H.tier = 1;
        return;
    }
    if (H.tier == 1u) return;  // tier-1 waves keep to their few rays
    if (!H.t2_done && have < kHeavy2 && take_from(P, F, P.heavy + 2, H.k1, H.kh, kHeavy2 - have, act, L, H.t2_done))
        H.tier = 2;
}

// ---- tier 1 traced by groups of lanes (k_trace) ----------------------------
// A pixel whose chain is the critical path of the frame (or of a rank's
// share) is traced to its end by a group of g = 2^lg lanes of a wave (lg 6:
// the whole wave), every lane of the group holding the same Lane state: lane
// k of the group scans sphere pairs k, k + g, ... (the group coop's scan,
// from the LDS copy), the group reduces (min c, then the largest index among
// equal c: the in-order scan's answer) and shades uniformly with the
// lane-mode functions. Taken off each segment's critical path: the scatter's
// seed-determined part (scatter_spec) is evaluated before the scan, and each
// lane loads the material of its own best candidate while the group reduces;
// the winner's is then read from its lane. A non-finite root takes the exact
// in-order scan (the group's lanes, the same ray). Several groups per wave
// trace several chains for little more issue than one: the scan's pairs are
// split over fewer lanes, everything else is issued once for all groups.
// One segment of every active group (the group's lanes hold its pixel's
// state W; lanes of groups without a pixel flag nothing); `ended`: the
// group's pixel finished its last sample (W.acc, W.seed final).
// kLg: the group size is a compile-time constant (k_trace dispatches on the
// wave's lg): the shifts, the reduction's DPP steps and the winner's
// material fetch are then as cheap as in a whole-wave-only kernel (a
// runtime lg cost the one-pixel-per-wave case 2.0 -> 2.5 us per segment,
// profiles/R6f_pixel_timeline_r8.jsonl).
template <uint32_t kLg, typename Src>
__device__ __forceinline__ void trace_group_segment(const KParams &P, const Frame &F, const Src &src, Lane &W,
                                                    bool &ended) {
    constexpr uint32_t lg = kLg;
    const KScene &S = P.scene;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t g = 1u << lg, k = lane & (g - 1u);
    const uint64_t gm = lg >= 6u ? ~0ull : ((1ull << g) - 1ull) << (lane & ~(g - 1u));  // my group's lanes
    const float inf = __uint_as_float(0x7f800000u);
    const int last = (int)S.n - 1;
    const ScatterSpec sp = scatter_spec(W.seed);
    LineTest T = line_test_setup(W.o.x, W.o.y, W.o.z, W.d.x, W.d.y, W.d.z, W.a, S.smag);
    if (lg < 6u && !W.active) {  // a group without a pixel: nothing is flagged (a whole wave is always active)
        T.ux = T.uy = T.uz = T.vy = T.vz = T.nou = T.nov = 0.0f;
        T.thr = inf;
    }
    const f2v ux = {T.ux, T.ux}, uy = {T.uy, T.uy}, uz = {T.uz, T.uz}, vy = {T.vy, T.vy}, vz = {T.vz, T.vz};
    const f2v nou = {T.nou, T.nou}, nov = {T.nov, T.nov}, th = {T.thr, T.thr};
    uint64_t key = hit_key(inf, -1);
    bool ok = true;
    const uint32_t nsteps = src.npairs >> lg;  // SphLds: npairs is a multiple of 64
#pragma unroll 1
    for (uint32_t s0 = 0; s0 < nsteps; s0 += kGfSteps) {
        // the group coop's scan and resolve (hit_world_groups)
        uint32_t im = 0;
        const uint32_t s1 = min(s0 + kGfSteps, nsteps);
        auto step = [&](uint32_t st) {
            f2v cx, cy, cz, R;
            src.pair((st << lg) + k, cx, cy, cz, R);
            const f2v pu = fma2(cx, ux, fma2(cy, uy, fma2(cz, uz, nou)));
            const f2v pv = fma2(cy, vy, fma2(cz, vz, nov));
            const f2v q = fma2(-pv, pv, fma2(-pu, pu, R)) - th;
            im = (im << 1) | (__float_as_uint(q.y) >> 31);
            im = (im << 1) | (__float_as_uint(q.x) >> 31);
        };
        uint32_t st = s0;
        for (; st + 2u <= s1; st += 2u) {
            step(st);
            step(st + 1u);
        }
        if (st < s1) step(st);
        const uint32_t nb = 2u * (s1 - s0);
        uint32_t fm = ~im & (nb >= 32u ? ~0u : ((1u << nb) - 1u));
#pragma unroll 1
        while (__ballot(fm != 0u) != 0ull) {
            const bool live = fm != 0u;
            const uint32_t bit = live ? (uint32_t)__builtin_ctz(fm) : 0u;
            fm &= fm - 1u;
            const uint32_t p = ((s1 - 1u - (bit >> 1)) << lg) + k;
            const uint32_t j = 2u * p + (bit & 1u);
            resolve_one(src.sphere(j), (int)j, live, W.o, W.d, W.a, W.inv_a, kTMin, key, ok);
        }
    }
    // each lane's best candidate: its material is loaded during the reduction
    const uint32_t lo = ~(uint32_t)key;  // index + 1, 0: none
    const uint32_t jl = lo != 0u ? min(lo - 1u, (uint32_t)last) : 0u;
    const int mt_l = S.mtype[jl];
    const float4 mv_l = S.mval[jl];
    const uint32_t cb0 = (uint32_t)(key >> 32);
    const uint32_t cb = group_reduce_u32<false>(cb0, lg);
    const uint32_t ib = group_reduce_u32<true>(cb0 == cb ? lo : 0u, lg);
    const uint64_t win = __ballot(ib != 0u && lo == ib && cb0 == cb) & gm;  // lanes holding the group's winner
    const uint64_t bad = __ballot(!ok) & gm;                               // a non-finite root in the group
    // the winner's material from its lane: v_readlane when the group is the
    // whole wave (lg 6: uniform), else a permute (every lane takes part)
    HitMat M;
    if constexpr (lg >= 6u) {
        const int wl = win != 0ull ? (int)__builtin_ctzll(win) : 0;
        M.mt = __builtin_amdgcn_readlane(mt_l, wl);
        M.mv = make_float4(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(mv_l.x), wl)),
                           __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mv_l.y), wl)),
                           __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mv_l.z), wl)),
                           __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mv_l.w), wl)));
    } else {
        const int wl = win != 0ull ? (int)__builtin_ctzll(win) : (int)lane;
        M.mt = __shfl(mt_l, wl, 64);
        M.mv = make_float4(__shfl(mv_l.x, wl, 64), __shfl(mv_l.y, wl, 64), __shfl(mv_l.z, wl, 64),
                           __shfl(mv_l.w, wl, 64));
    }
    ended = false;
    if (lg < 6u && !W.active) return;
    int hit = -1;
    float t = inf;
    if (bad != 0ull) {  // the exact in-order scan, the group's ray in every lane of it
        hit = hit_blocks_seq((cfloat_p)S.soa, S.n_pad / 8u, 0, W.o, W.d, W.a, W.inv_a, kTMin, t, -1);
        if (hit >= 0) {
            hit = min(hit, last);
            M = hit_mat(S, hit);
        }
    } else if (ib != 0u) {
        hit = min((int)(ib - 1u), last);
        t = __uint_as_float(cb);
        M.sc = src.sphere((uint32_t)hit);  // the same floats as cen[hit]
    }
    W.segs++;
    f3 c;
    const int r = path_segment_m<true>(P, W, hit, t, M, sp, c);
    if (r == kSegSky) W.acc = W.acc + c;
    if (r != kSegContinue) {
        W.sample++;
        if (W.sample >= P.spp) {
            ended = true;
            return;
        }
        begin_sample(P, F, W.x, W.y, W);
    }
}

// Move the wave's pixels into fewer, larger groups: the n-th active group of
// lg (n < m active groups) becomes group n of nlg — every lane of the new
// group copies the Lane state of a lane of the old one (all lanes of a group
// hold the same state); new groups past m are idle.
__device__ __forceinline__ void regroup(Lane &W, uint32_t lg, uint32_t nlg, uint64_t act) {
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t lead = 0;  // the first lane of every active group
    for (uint32_t r = 0; r < (64u >> lg); ++r)
        if ((act >> (r << lg)) & 1ull) lead |= 1ull << (r << lg);
    const uint32_t m = (uint32_t)__popcll(lead);
    const uint32_t rn = lane >> nlg;
    uint64_t mm = lead;
    for (uint32_t i = 0; i < rn && mm != 0ull; ++i) mm &= mm - 1ull;
    const bool has = rn < m;
    const int src = has ? (int)__builtin_ctzll(mm) : (int)lane;
    auto mvf = [src](float &v) { v = __shfl(v, src, 64); };
    auto mvu = [src](uint32_t &v) { v = (uint32_t)__shfl((int)v, src, 64); };
    mvf(W.o.x); mvf(W.o.y); mvf(W.o.z);
    mvf(W.d.x); mvf(W.d.y); mvf(W.d.z);
    mvf(W.col.x); mvf(W.col.y); mvf(W.col.z);
    mvf(W.acc.x); mvf(W.acc.y); mvf(W.acc.z);
    mvf(W.a); mvf(W.inv_a); mvf(W.seed);
    mvu(W.sample); mvu(W.bounce); mvu(W.segs);
    mvu(W.x); mvu(W.y); mvu(W.gid); mvu(W.slot); mvu(W.seg0); mvu(W.c0);
    W.active = has;
}

// Promotion queue service: wait for an entry and load it into W (every lane
// the same state, at the entry's sample boundary), or return false once every
// pixel k_render owns is written. prom[2] counts them (k_render waves when
// they go idle; whoever finishes a promoted pixel), `target` is their number
// (npix, less tier 1 when k_trace runs it): k_trace's own pixels are not in
// it, so k_render's exit never waits for k_trace, which HIP does not promise
// to run at the same time. Promoted pixels are counted by whoever finishes
// them, so the count reaches `target` only when the queue holds nothing
// more. The tail is read after the count: a pixel is promoted (slot claimed,
// entry stored) before its old wave can go idle and flush. `helper` (k_trace):
// serve only while k_render runs — prom[3] is set by its first workgroup; a
// k_trace that sees it unset leaves (k_render then serves its own
// promotions), one that sees it set waits on a kernel that is already
// running. All relaxed
// (agent_store_order). Polls sleep ~8k clocks at priority 0. Safety valve: a
// server that sees no pixel written for kPromValveTicks leaves and flags the
// launch (KParams::errors: rtx_sync / rtx_get_stats report it), so a bug shows
// as an error, never as a hung GPU or a silently unwritten pixel.
// Progress is a pixel written (prom[2]) or a heartbeat: every wave still
// tracing once its queue is exhausted (k_render) and every k_trace wave
// stores the time into prom[4] at most every kBeatTicks (beat), so a long
// but live chain — a big scene, a high spp — never trips the valve however
// long it runs without another pixel finishing; only a launch in
// which nothing traces any more does. The stress build (make all) runs with
// a 20 ms valve (a beat every 1.25 ms), so its GPU tests exercise exactly
// that.
// The valve's clock runs only while the server itself runs (Valve): a poll
// that comes more than a beat period after the server's previous one means
// the server was not running either (its wave descheduled, the queue
// preempted), which is no evidence that nothing else ran, so the clock
// restarts there. A server that keeps polling on time with nothing written
// and no heartbeat still leaves after kPromValveTicks. The wait for a claimed
// entry's epoch has its own clock from the claim and its own bit
// (kErrPromEntryWait). The first firing leaves its record in KParams::err_diag.
// (kPromValveTicks: rtx_internal.h)
constexpr unsigned long long kBeatTicks = kPromValveTicks / 16u;
constexpr uint32_t kBeatShift = 10;  // prom[4] holds s_memrealtime >> 10 (10.24 us units, wraps every ~12 h)
__device__ __forceinline__ void flag_error(const KParams &P, uint32_t bit) {
    if (P.errors && (threadIdx.x & 63u) == 0u) atomicOr(P.errors, bit);
}
struct Valve {  // 32-bit s_memrealtime ticks (wrap after 42 s; the valve is shorter): few SGPRs in k_render
    uint32_t t0, last, stalls;
    __device__ __forceinline__ void start() {
        t0 = last = (uint32_t)__builtin_amdgcn_s_memrealtime();
        stalls = 0u;
    }
    __device__ __forceinline__ void progress() { t0 = last; }  // a pixel written or a heartbeat seen
    // one poll; true once the server has polled on time for kPromValveTicks
    // since it last saw progress
    __device__ __forceinline__ bool expired() {
        const uint32_t now = (uint32_t)__builtin_amdgcn_s_memrealtime();
        if (now - last > (uint32_t)kBeatTicks) {  // the server itself did not run: restart the clock
            t0 = now;
            ++stalls;
        }
        last = now;
        return now - t0 > (uint32_t)kPromValveTicks;
    }
};
static_assert(kPromValveTicks < (1ull << 31), "the valve's 32-bit clock");
// The valve fired: flag the launch and, if no server has yet, record what
// this one saw in one 64-bit word (rtx_internal.h KParams::err_diag; the host
// adds the launch's queue counters, which stay in memory after it). Kept to
// one atomic: the record's code sits in k_render, whose registers are tight
// (a larger record moved the C2 render's spill code).
#ifndef RTX_VALVE_RECORD  // A/B build: 0 = the error bit alone
#define RTX_VALVE_RECORD 1
#endif
__device__ __forceinline__ void valve_fire(const KParams &P, uint32_t bit, uint32_t who, const Valve &V) {
    flag_error(P, bit);
    if (!RTX_VALVE_RECORD || P.err_diag == nullptr || (threadIdx.x & 63u) != 0u) return;
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    const uint32_t bt = __hip_atomic_load(&P.prom[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t since = min(((uint32_t)now - V.t0) >> kBeatShift, 0xffffu);  // 10.24 us units
    const uint32_t age = (uint32_t)(now >> kBeatShift) - bt;                    // the same units
    const unsigned long long rec = (unsigned long long)(bit | who << 4 | min(V.stalls, 0xffu) << 8 | since << 16) |
                                   (unsigned long long)age << 32;
    atomicCAS(P.err_diag, 0ull, rec);
}
// The heartbeat (wave-uniform; `last` is the wave's previous beat).
__device__ __forceinline__ void beat(const KParams &P, unsigned long long &last) {
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    if (now - last > kBeatTicks) {
        last = now;
        if ((threadIdx.x & 63u) == 0u)
            __hip_atomic_store(&P.prom[4], (uint32_t)(now >> kBeatShift), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
__device__ __forceinline__ bool take_promoted(const KParams &P, const Frame &F, uint32_t npix, uint32_t target,
                                              bool helper, Lane &W) {
    Valve V;
    V.start();
    uint32_t seen = ~0u;
    __builtin_amdgcn_s_setprio(0);
    auto ld = [](const uint32_t *p) {
        return (uint32_t)__builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    };
    uint32_t seen_beat = 0;
    for (;;) {
        const uint32_t done = ld(&P.prom[2]);
        if (done >= target) return false;
        if (helper && ld(&P.prom[3]) == 0u) return false;  // k_render has not started: it serves itself
        const uint32_t bt = ld(&P.prom[4]);
        if (done != seen || bt != seen_beat) {  // progress (a pixel written, or a heartbeat): the valve restarts
            seen = done;
            seen_beat = bt;
            V.progress();
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        const uint32_t t = min(ld(&P.prom[0]), P.prom_cap);
        const uint32_t h = ld(&P.prom[1]);
        uint32_t got = ~0u;
        if (h < t && (threadIdx.x & 63u) == 0u) got = atomicCAS(&P.prom[1], h, h + 1u) == h ? h : ~0u;
        got = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)got, 0, 64));
        if (got != ~0u) {
            const uint32_t *e = P.prom_q + 8u * got;
            V.start();  // the entry's producer publishes it right after claiming the slot: a clock of its own
            bool late = false;
            while (__hip_atomic_load(e + 7, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != P.epoch) {
                __builtin_amdgcn_s_sleep(1);
                if (V.expired()) {
                    late = true;
                    break;
                }
            }
            if (late) {
                valve_fire(P, kErrPromEntryWait, 1u, V);
                return false;
            }
            __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the fields are read after the epoch matched
            W.gid = __hip_atomic_load(e + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            W.sample = __hip_atomic_load(e + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            W.seed = __uint_as_float(__hip_atomic_load(e + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            W.acc = mk3(__uint_as_float(__hip_atomic_load(e + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
                        __uint_as_float(__hip_atomic_load(e + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
                        __uint_as_float(__hip_atomic_load(e + 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
            if (W.gid >= npix || W.sample >= P.spp) {  // never: a torn entry ends the wave, not the GPU
                flag_error(P, kErrPromTorn);
                return false;
            }
            lane_pixel(P, W.gid, W.x, W.y);
            W.seg0 = W.segs;
            W.slot = ~0u;
            W.active = true;
            begin_sample(P, F, W.x, W.y, W);
            diag_pixel_start(P, W.gid, 3ull);
            return true;
        }
        if (h >= t) __builtin_amdgcn_s_sleep(127);
        if (V.expired()) {
            valve_fire(P, kErrPromTimeout, 1u, V);
            return false;
        }
    }
}

// Persistent cost pre-pass (large scenes): its tail. Once the pixel queue is
// exhausted the pass runs on only until its last pixels' first samples end,
// and at 100k spheres a lane-mode segment of a nearly idle GPU takes
// milliseconds: the last ~20 % of the pass's time had most of the chip idle.
// So the pass counts the pixels it has finished (pre_done, one atomic per
// wave-iteration in which some ended), and once no more than pre_stop pixels
// are still in flight, every wave stops its pixels where they are: each takes
// the saturated key (the top bucket, as a pixel past the cost cap does) and
// the render traces it from sample 0. Those are the pixels whose first sample
// ran longest — the expensive ones — so the queue order they get is the right
// one, and no result changes (the render redoes them with the same ops).
__device__ __forceinline__ void pre_count(const KParams &P, uint64_t before, const Lane &L) {
    const uint32_t n = (uint32_t)__popcll(before & ~__ballot(L.active));
    if (n != 0u && (threadIdx.x & 63u) == 0u)
        __hip_atomic_fetch_add(P.pre_done, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Returns true when it stopped the wave's pixels (wave-uniform).
__device__ __forceinline__ bool pre_stop(const KParams &P, uint32_t npix, Lane &L) {
    const uint32_t done = (uint32_t)__builtin_amdgcn_readfirstlane(
        __hip_atomic_load(P.pre_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const uint64_t act = __ballot(L.active);
    if (act == 0ull || npix - min(done, npix) > P.pre_stop) return false;
    if (L.active) {  // the cost cap's record: saturated key, restart from sample 0 (seed NaN)
        P.cost_out[L.gid] = P.cost_capped;
        P.state[L.gid] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(0x7fc00000u));
        L.segs = L.seg0;
        L.active = false;
        diag_pixel_end(P, L.gid);
    }
    pre_count(P, act, L);
    return true;
}
// Render kernel (chain RNG), per-wave independent; sphere blocks are read
// with scalar loads (a block-wide LDS copy serves the coop and the resolve of
// scenes up to kCoopLds spheres). kPersist: the grid holds as many waves as the GPU keeps resident and
// lanes pull pixels from the (cost-ordered) queue until it is exhausted;
// otherwise an exact grid, one pixel per lane. kCost: the scheduling
// pre-pass (P.cost_out: per-pixel segments, P.state: the state to resume).
// Tile-major enumerations of a W x rows pixel grid: j in [0, tile_span) ->
// pixel index (row-major within a T x T tile, tiles row-major), or ~0u for a
// slot of a partial tile; T = 0: row-major, the identity. The cost sort
// uses them (RTX_QUEUE_TILE, below): spatially close rays share more of the
// layer grid's blocks. The exact grid can too (RTX_EXACT_TILE 8: a wave's 64
// lanes an 8 x 8 patch; an A/B option, flat at C2: S6s).
__host__ __device__ __forceinline__ uint32_t tile_span(uint32_t width, uint32_t rows, uint32_t T, uint32_t TY = 0u) {
    if (TY == 0u) TY = T;
    return T == 0u ? width * rows : ((width + T - 1u) / T) * ((rows + TY - 1u) / TY) * T * TY;
}
// (T x TY tiles; TY = 0: square)
__device__ __forceinline__ uint32_t tile_pixel(uint32_t j, uint32_t width, uint32_t rows, uint32_t T, uint32_t TY = 0u) {
    if (T == 0u) return j < width * rows ? j : ~0u;
    if (TY == 0u) TY = T;
    const uint32_t tx = (width + T - 1u) / T;
    const uint32_t t = j / (T * TY), u = j % (T * TY);
    const uint32_t x = (t % tx) * T + u % T, y = (t / tx) * TY + u / T;
    return (x < width && y < rows) ? y * width + x : ~0u;
}
#ifndef RTX_EXACT_TILE
#define RTX_EXACT_TILE 0
#endif
constexpr uint32_t kExactTile = RTX_EXACT_TILE;

template <bool kPersist, bool kCost = false, bool kPF = false, bool kLin = false>
__global__ void RTX_RENDER_BOUNDS_T2(kPF, kLin) k_render(const KParams P) {
    constexpr bool kCulled = kPF && RTX_CULL && !kLin;  // the culled scan (large scenes, not the linear mode)
    // dynamic LDS: [candidate list, list_bytes<kPF>][coop rays, kCoopBytes][coop LDS copy of the spheres]
    extern __shared__ __attribute__((aligned(16))) unsigned char s_mem[];
    uint32_t *list = reinterpret_cast<uint32_t *>(s_mem);
    constexpr uint32_t kLB = list_bytes<kPF>();
    float *coop_ws = reinterpret_cast<float *>(s_mem + kLB) + (threadIdx.x / 64) * (kCoopWaveBytes / 4);
    (void)coop_ws;
    // the coop's sphere data: a block-wide LDS copy for small scenes (SphLds)
    const bool coop_lds = P.scene.n <= kCoopLds;
    const SphLds sl = lds_copy(P.scene, reinterpret_cast<float *>(s_mem + kLB + kCoopBytes), coop_lds);
    const SphGlobal sg = sph_global(P.scene);
    // kPF scenes never fit the LDS copy: its place holds the scan's pack word
    uint32_t *pack = kPF ? reinterpret_cast<uint32_t *>(s_mem + kLB + kCoopBytes) : nullptr;
    const float *pf_tile = kPF && (RTX_PF_LDS || RTX_PF_RING) ? reinterpret_cast<const float *>(s_mem + kLB + kCoopBytes + 16) : nullptr;
    // promotion: the block's first wave to go idle serves the queue, the others leave
    __shared__ uint32_t s_server;
    const bool prom_on = kPersist && !kCost && P.prom != nullptr;
    if (kPF && threadIdx.x == 0) *pack = 0u;
    if (prom_on && threadIdx.x == 0) s_server = 0u;
    // "k_render runs" for k_trace's promotion service (take_promoted): one
    // plain store by one workgroup. A returning atomic by every workgroup
    // here, waited for at the barrier below, cost the C2 frame 4-7 ms
    // (43.7 vs 47.9-51 ms, profiles/R6d_ab_c2_bisect.jsonl).
    if (prom_on && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(&P.prom[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (coop_lds || kPF || prom_on) __syncthreads();
    const int last = (int)P.scene.n - 1;
    const Frame F = load_frame(P);
    const uint32_t npix = P.rows_local * P.width;
    const unsigned long long t_start = P.wave_times ? __builtin_amdgcn_s_memrealtime() : 0ull;
    Lane L;
    L.active = false;
    L.segs = 0;
    L.slot = ~0u;
    L.cb = L.ce = 0u;
    bool exhausted = !kPersist;
    if (!kPersist) {
        const uint32_t gid = tile_pixel(blockIdx.x * kRB + threadIdx.x, P.width, P.rows_local, kExactTile);
        if (gid < npix) start_pixel(P, F, gid, L);
    }
    // heavy slots [0, kh) of the queue (k_heavy_split; tier 1 = [0, k1)), normal slots [kh, npix)
    HeavyState H;
    H.kh = (kPersist && P.heavy) ? min(P.heavy[1], npix) : 0u;
    H.k1 = (kPersist && P.heavy) ? min(P.heavy[3], H.kh) : 0u;
    H.t1_done = H.k1 == 0u || P.trace_ext != 0u;  // tier 1: k_trace when it runs beside this kernel
    H.t2_done = H.k1 == H.kh;
    H.tier = 0;
    const uint32_t kh = H.kh;
    // the mean pixel's segments (dynamic priority's unit)
    const float dyn_m = (kPersist && P.cost_in && P.heavy) ? __uint_as_float(P.heavy[5]) : 0.0f;
    // promotion's exit count: the pixels this kernel owns (tier 1 is k_trace's when it runs beside it)
    const uint32_t owned = npix - (P.trace_ext != 0u ? H.k1 : 0u);
    uint32_t written = 0;  // pixels this wave wrote since it last reported
    unsigned long long last_beat = 0;  // the wave's last heartbeat (beat)
    Diag D;
    D.begin();
    for (;;) {
        if (!(H.t1_done && H.t2_done) && (H.tier != 0u || __ballot(L.active) == 0ull)) take_heavy(P, F, H, L);
        if (H.tier != 0u && __ballot(L.active) == 0ull) H.tier = 0;  // drained, no heavy slot left
        const bool heavy = H.tier != 0u;
        if (!heavy && !exhausted) exhausted = refill(P, F, kh, npix, L);
        if (kPersist && kCost && P.pre_done && exhausted && pre_stop(P, npix, L)) continue;
        const uint64_t act = __ballot(L.active);
        D.section(0);
        if (act == 0ull) {  // spp, depth > 0: idle after both queues => drained
            if (!prom_on) break;
            if (written != 0u && (threadIdx.x & 63u) == 0u)
                __hip_atomic_fetch_add(&P.prom[2], written, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            written = 0;
            uint32_t srv = 0;
            if ((threadIdx.x & 63u) == 0u) srv = atomicCAS(&s_server, 0u, threadIdx.x / 64u + 1u);
            srv = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)srv, 0, 64));
            if (srv != 0u && srv != threadIdx.x / 64u + 1u) break;  // another wave serves this block
            if (!take_promoted(P, F, npix, owned, false, L)) {
                // leaving: free the block's server slot, so that a wave of
                // this block that goes idle later can serve in its place
                if ((threadIdx.x & 63u) == 0u) atomicExch(&s_server, 0u);
                break;
            }
            L.active = (threadIdx.x & 63u) == 0u;  // one ray, traced by the whole wave (tier-1 coop)
            H.tier = 1;
            continue;
        }
        const uint64_t was_active = act;
        // still tracing: the servers' valve sees progress. Every tracing wave
        // beats, not only those that have seen the queue exhausted: a wave
        // whose lanes are all busy never refills and never learns it (R7e: a
        // 2 ms stress valve fired while only such waves were tracing)
        if (prom_on) beat(P, last_beat);
        D.iteration(act);
        if (heavy || (exhausted && (uint32_t)__popcll(act) <= P.coop_max)) {
            D.tail_iteration();
            // Frame tail: the few pixels left in this wave are its critical
            // path; trace their rays together, several lanes per ray.
            float my_best = __uint_as_float(0x7f800000u);
            bool my_seq = false;
            // this wave carries the frame's critical path: tier 1 > tier 2 > tail
            set_prio(H.tier == 1u ? P.prio_t1 : H.tier == 2u ? P.prio_t2 : (uint32_t)kTailPrio);
            unsigned long long *ctqp;
            unsigned long long *cp = D.coop_begin(H.tier, ctqp);
            bool promoted = false;
            int my_hit = kCulled
                             ? hit_world_groups_culled(P.scene, act, L.active, L.o, L.d, L.a, L.inv_a, kTMin, coop_ws,
                                                       my_best, my_seq)
                         : coop_lds ? hit_world_groups(P.scene, sl, act, L.active, L.o, L.d, L.a, L.inv_a, kTMin,
                                                       coop_ws, my_best, my_seq, cp, ctqp)
                                    : hit_world_groups(P.scene, sg, act, L.active, L.o, L.d, L.a, L.inv_a, kTMin,
                                                       coop_ws, my_best, my_seq, cp, ctqp);
            if (L.active) {
                if (my_seq) {  // (rare: the plain scan, so the kPF ping-pong's SGPRs stay out of this kernel)
                    my_best = __uint_as_float(0x7f800000u);
                    my_hit = hit_world_pre<false, !kPF>(P.scene, L.o, L.d, L.a, L.inv_a, kTMin, my_best, list);
                }
                // the tail's pixels may be promoted (tier-1 waves already
                // trace one ray with every lane; promoting tier-2 pixels
                // measured 1-6 ms slower at R = 2, 4, 8: profiles/R3r_*)
                promoted = shade<kCost>(P, F, L, min(my_hit, last), my_best,
                                        prom_on && exhausted && H.tier == 0u ? P.prom_min : 0u);
            }
            if (prom_on)
                written += (uint32_t)__popcll(act & ~__ballot(L.active)) - (uint32_t)__popcll(__ballot(promoted));
            if (kPersist && kCost && P.pre_done) pre_count(P, act, L);
            D.coop_end(cp, H.tier);
            if (H.tier == 0u) __builtin_amdgcn_s_setprio(0);  // a heavy wave keeps its priority
            D.section(3);
            continue;
        }
        // lane mode: a wave that holds one of the heaviest pixels of the
        // normal queue (its first prio_slots slots) runs at the top priority,
        // so its time per segment is not stretched by the SIMD's other waves
        if (P.cost_in) {
            set_prio(dyn_level(P, L, dyn_m));
        } else {
            set_prio(__ballot(L.active && L.slot < kh + P.prio_slots) != 0ull ? P.prio_hot : 0u);
        }
        bool promoted = false;
        D.rays(P, L.o, L.d, L.active, L.slot);
        if (kCulled) {  // large scenes: the culled scan (block bounds first, scan_culled)
            if (L.active) {
                float best = __uint_as_float(0x7f800000u);
                const int hit = hit_world_culled(P.scene, L.o, L.d, L.a, L.inv_a, kTMin, best, list);
                D.section(1);
                promoted = shade<kCost>(P, F, L, min(hit, last), best, prom_on && exhausted ? P.prom_min : 0u);
            }
        } else if ((RTX_PF_LDS || RTX_PF_RING) && kPF) {  // every lane of the wave fills the scan's LDS tile
            float best = __uint_as_float(0x7f800000u);
            auto ldc = [&P](uint32_t i) { return P.scene.cen[i]; };
            const int hit = hit_world_pre_ld<kPF, decltype(ldc), true>(P.scene, ldc, L.o, L.d, L.a, L.inv_a, kTMin,
                                                                       best, list, nullptr, 0, pf_tile, L.active);
            D.section(1);
            if (L.active) promoted = shade<kCost>(P, F, L, min(hit, last), best, prom_on && exhausted ? P.prom_min : 0u);
        } else if (L.active) {
            float best = __uint_as_float(0x7f800000u);
            // scenes that fit the coop's LDS copy resolve their candidates
            // from it (the same centre and radius floats as cen) instead of HBM/L2
            const int hit = (!kPF && coop_lds)  // kPF scenes (> kScanPfMin) never fit
                                ? hit_world_pre_ld<kPF>(P.scene, [sl](uint32_t i) { return sl.sphere(i); }, L.o, L.d,
                                                        L.a, L.inv_a, kTMin, best, list, nullptr, 0,
                                                        RTX_SCAN_LDS ? sl.pr : nullptr)
                                : hit_world_pre<kPF>(P.scene, L.o, L.d, L.a, L.inv_a, kTMin, best, list, pack);
            D.section(1);
            promoted = shade<kCost>(P, F, L, min(hit, last), best, prom_on && exhausted ? P.prom_min : 0u);
        }
        D.section(2);
        if (prom_on)  // pixels written this iteration (promoted ones are counted by whoever finishes them)
            written += (uint32_t)__popcll(was_active & ~__ballot(L.active)) - (uint32_t)__popcll(__ballot(promoted));
        if (kPersist && kCost && P.pre_done) pre_count(P, was_active, L);
    }
    D.finish(P);
    count_segments(P, L.segs);
    if (!kDiagAny && P.wave_times && (threadIdx.x & 63u) == 0u) {  // diagnostic only (rtx_debug_wave_times)
        const uint32_t w = blockIdx.x * (kRB / 64) + threadIdx.x / 64;
        P.wave_times[2 * w] = t_start;
        P.wave_times[2 * w + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

// Promotion service for the idle groups of a k_trace wave (`need`: the first
// lane of every idle group of size 2^lg): claims up to one entry per idle
// group in one CAS and loads each into its group's lanes (take_promoted's
// protocol and exit rule, k_trace's `helper` side). Returns the entries
// claimed, or -1 once the service is over for this wave: every pixel k_render
// owns is written, k_render has not started, or the valve fired. `blocking`
// (the wave has nothing else to trace): poll until an entry or the end;
// otherwise one look.
__device__ __forceinline__ int take_promoted_groups(const KParams &P, const Frame &F, uint32_t npix, uint32_t target,
                                                    uint64_t need, uint32_t lg, bool blocking, Lane &W) {
    const uint32_t lane = threadIdx.x & 63u;
    auto ld = [](const uint32_t *p) {
        return (uint32_t)__builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    };
    Valve V;
    V.start();
    uint32_t seen = ~0u, seen_beat = 0;
    const uint32_t nneed = (uint32_t)__popcll(need);
    // this lane's group among the idle ones (only meaningful in idle groups)
    const uint32_t rank = (uint32_t)__popcll(need & ((1ull << (lane & ~((1u << lg) - 1u))) - 1ull));
    for (;;) {
        const uint32_t done = ld(&P.prom[2]);
        if (done >= target || ld(&P.prom[3]) == 0u) return -1;
        const uint32_t bt = ld(&P.prom[4]);
        if (done != seen || bt != seen_beat) {  // progress: a pixel written or a heartbeat
            seen = done;
            seen_beat = bt;
            V.progress();
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        const uint32_t t = min(ld(&P.prom[0]), P.prom_cap);
        const uint32_t h = ld(&P.prom[1]);
        const uint32_t want = h < t ? min(t - h, nneed) : 0u;
        if (want != 0u) {
            uint32_t won = 0;
            if (lane == 0u) won = atomicCAS(&P.prom[1], h, h + want) == h ? 1u : 0u;
            won = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)won, 0, 64));
            if (won == 0u) continue;  // another server took them first
            bool torn = false, late = false;
            Valve E;  // each claimed entry's wait has its own clock from the claim (kErrPromEntryWait)
            E.start();
            if (!W.active && rank < want) {
                const uint32_t *e = P.prom_q + 8u * (h + rank);
                while (__hip_atomic_load(e + 7, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != P.epoch) {
                    __builtin_amdgcn_s_sleep(1);
                    if (E.expired()) {
                        late = true;
                        break;
                    }
                }
                __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the fields are read after the epoch matched
                W.gid = __hip_atomic_load(e + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                W.sample = __hip_atomic_load(e + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                W.seed = __uint_as_float(__hip_atomic_load(e + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                W.acc = mk3(__uint_as_float(__hip_atomic_load(e + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
                            __uint_as_float(__hip_atomic_load(e + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
                            __uint_as_float(__hip_atomic_load(e + 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
                late = late || __hip_atomic_load(e + 7, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != P.epoch;
                torn = !late && (W.gid >= npix || W.sample >= P.spp);
                if (!torn && !late) {
                    lane_pixel(P, W.gid, W.x, W.y);
                    W.seg0 = W.segs;
                    W.slot = ~0u;  // a promoted pixel: counted in prom[2] when written
                    W.active = true;
                    begin_sample(P, F, W.x, W.y, W);
                    diag_pixel_start(P, W.gid, 3ull);
                }
            }
            // never: a late or torn entry ends the wave's service, not the GPU
            const uint64_t lb = __ballot(late), tb = __ballot(torn);
            if ((lb | tb) != 0ull) {
                if (lb != 0ull) {
                    const uint32_t src = (uint32_t)__builtin_ctzll(lb);  // the record: the first late lane's wait
                    E.t0 = (uint32_t)__shfl((int)E.t0, (int)src, 64);
                    E.stalls = (uint32_t)__shfl((int)E.stalls, (int)src, 64);
                    valve_fire(P, kErrPromEntryWait, 2u, E);
                }
                if (tb != 0ull) flag_error(P, kErrPromTorn);
                return -1;
            }
            return (int)want;
        }
        if (!blocking) return 0;
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_sleep(127);
        if (V.expired()) {
            valve_fire(P, kErrPromTimeout, 2u, V);
            return -1;
        }
    }
}

// Tier 1 as its own kernel (the scheduled path, scenes up to kCoopLds
// spheres): workgroups of independent waves launched on the context's auxiliary
// stream beside k_render (launch_render), taking tier-1 slots ([0, k1) of the
// cost-ordered queue, k_heavy_split) and tracing each pixel with a group of
// lanes (trace_group_segment), at wave priority prio_t1. The very heaviest
// slots, [0, k0), go one per wave (the whole wave on one chain: the shortest
// time per segment); the rest 2^(6 - trace_lg) per wave (trace_group: the same
// chains for a fraction of the SIMD time). A group whose pixel ends takes the
// next slot; once tier 1 is exhausted the idle groups serve the promotion
// queue while k_render runs (take_promoted_groups), and a wave whose pixels
// fill at most half its groups regroups them into larger groups (regroup:
// shorter segments for the last chains). Its own register budget (up to 128
// VGPRs) keeps this state out of k_render, whose lane-mode loop it would
// otherwise crowd into scratch. k_render skips tier 1
// (KParams::trace_ext).
// Four independent waves per workgroup (no barrier after the copy): they share
// one LDS copy of the scene. One-wave workgroups, each with its own 10-13 KiB
// copy, took LDS the render's blocks needed: at R = 8 (7 k_trace waves per
// CU) only ~79 % of k_render's lanes were resident (profiles/R6r_pixel_timelines.jsonl).
constexpr uint32_t kTraceThreads = 256;
__global__ void __launch_bounds__(kTraceThreads, 4) k_trace(const KParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char s_mem[];
    const SphLds sl = lds_copy(P.scene, reinterpret_cast<float *>(s_mem), true, kTraceThreads);
    __syncthreads();
    const Frame F = load_frame(P);
    const uint32_t npix = P.rows_local * P.width;
    const uint32_t k1 = min(P.heavy[3], min(P.heavy[1], npix));
    const uint32_t k0 = min(P.heavy[4], k1);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t lg_many = min(max(P.trace_lg, 3u), 6u);
    set_prio(P.prio_t1);
    uint32_t lg = 6u;
    Lane W;
    W.active = false;
    W.segs = 0;
    W.seg0 = 0;
    W.slot = 0;
    uint32_t segs = 0;  // segments traced, counted by the first lane of each group
    bool t1_done = k1 == 0u;
    bool serve_done = P.prom == nullptr;
    unsigned long long last_beat = 0;  // the wave's last heartbeat (beat)
    for (;;) {
        uint64_t act = __ballot(W.active);
        if (act == 0ull && t1_done) lg = lg_many;  // an idle wave serves promotions in groups again
        if (!t1_done) {  // idle groups take tier-1 slots, one atomic per wave
            if (act == 0ull) {  // a wave without pixels picks its group size: solo slots one per wave
                const uint32_t next = (uint32_t)__builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(P.heavy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                lg = next < k0 ? 6u : lg_many;
            }
            const uint32_t g = 1u << lg;
            const uint64_t need = __ballot(!W.active && (lane & (g - 1u)) == 0u);
            if (need != 0ull) {
                const uint32_t n = (uint32_t)__popcll(need);
                uint32_t base = 0;
                if (lane == 0u) base = atomicAdd(P.heavy, n);  // the tier-1 counter
                base = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)base, 0, 64));
                const uint32_t rank = (uint32_t)__popcll(need & ((1ull << (lane & ~(g - 1u))) - 1ull));
                if (!W.active && base + rank < k1) {
                    start_pixel(P, F, P.perm[base + rank], W);
                    W.slot = base + rank;
                    diag_pixel_start(P, W.gid, 1ull);
                }
                if (base + n >= k1) t1_done = true;
                act = __ballot(W.active);
            }
        }
        if (t1_done && !serve_done) {  // then promoted pixels, while k_render runs
            const uint32_t g = 1u << lg;
            const uint64_t need = __ballot(!W.active && (lane & (g - 1u)) == 0u);
            if (need != 0ull) {
                set_prio(P.prio_t1);
                if (take_promoted_groups(P, F, npix, npix - k1, need, lg, act == 0ull, W) < 0) serve_done = true;
                set_prio(P.prio_t1);
                act = __ballot(W.active);
            }
        }
        if (act == 0ull) {
            if (t1_done && serve_done) break;
            continue;
        }
        if (t1_done && lg < 6u) {  // at most half the groups busy: fewer, larger groups
            uint32_t m = 0;
            for (uint32_t r = 0; r < (64u >> lg); ++r) m += (uint32_t)((act >> (r << lg)) & 1ull);
            if (2u * m <= (64u >> lg)) {
                const uint32_t nlg = 6u - (m <= 1u ? 0u : 32u - (uint32_t)__builtin_clz(m - 1u));
                regroup(W, lg, nlg, act);
                lg = nlg;
            }
        }
        bool ended;
        const bool first = (lane & ((1u << lg) - 1u)) == 0u;
        if (lg == 6u) {
            // one pixel in the whole wave: trace it to its end in a tight loop
            // (no group bookkeeping between segments: the per-segment latency
            // is this pixel's critical path)
            uint32_t n = 0;
            do {
                trace_group_segment<6>(P, F, sl, W, ended);
                ++n;
                if (P.prom) beat(P, last_beat);
            } while (!ended);
            if (first) segs += n;
        } else {
            if (P.prom) beat(P, last_beat);
            if (lg == 5u)  // wave-uniform; trace_group 1, 2, 4 or 8 (rtx_set_schedule)
                trace_group_segment<5>(P, F, sl, W, ended);
            else if (lg == 4u)
                trace_group_segment<4>(P, F, sl, W, ended);
            else  // 8 pixels per wave, 8 lanes each: a third of the issue per pixel-segment of 16-lane groups
                trace_group_segment<3>(P, F, sl, W, ended);
            if (W.active && first) segs++;
        }
        if (ended) {
            if (first) {
                write_pixel<false>(P, W);
                diag_pixel_end(P, W.gid);
                if (W.slot == ~0u)  // a promoted pixel: k_render's exit count
                    __hip_atomic_fetch_add(&P.prom[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            W.active = false;
        }
    }
    count_segments(P, segs);
}

// ---- cost-ordered pixel queue (LPT scheduling, see KSchedule) ------------
// One sample's segment count is a noisy estimate of a pixel's cost; the
// key is the sum over a (2R+1)^2 window of neighbouring pixels (clamped
// at the edges), which averages that noise over similar pixels.
constexpr int kLptRadius = 1;  // 3x3 window (radius 0 was 36 % slower, radius 2 5 % slower)
// sat_cap (row-split parts with a pre-pass cap, KTune::cap_split): a pixel
// the pre-pass stopped (cost kCostSaturated) takes the top bucket itself,
// and counts as sat_cap segments in its neighbours' windows (0: a stopped
// pixel's saturated cost saturates every window it is in, as for large
// scenes).
constexpr uint32_t kCostSaturated = 0xffffu;
__device__ __forceinline__ uint32_t cost_key(const uint32_t *cost, uint32_t i, uint32_t width, uint32_t rows,
                                             uint32_t cost_spp, uint32_t sat_cap) {
    if (sat_cap != 0u && cost[i] == kCostSaturated) return 0u;  // bucket 0 = most expensive
    const int x = (int)(i % width), y = (int)(i / width);
    uint32_t sum = 0;
    for (int dy = -kLptRadius; dy <= kLptRadius; ++dy) {
        const int yy = min(max(y + dy, 0), (int)rows - 1);
        for (int dx = -kLptRadius; dx <= kLptRadius; ++dx) {
            const int xx = min(max(x + dx, 0), (int)width - 1);
            const uint32_t c = cost[(uint32_t)yy * width + (uint32_t)xx];
            sum += (sat_cap != 0u && c == kCostSaturated) ? sat_cap : c;
        }
    }
    // scaled to 9 one-sample costs (the 3x3, 1-spp key the tiers were tuned on)
    const uint32_t win = (2 * kLptRadius + 1) * (2 * kLptRadius + 1) * cost_spp;
    if (win != 9u) sum = (sum * 9u + win / 2u) / win;
    return (kCostBuckets - 1u) - min(sum, kCostBuckets - 1u);  // bucket 0 = most expensive
}
constexpr uint32_t kSortPerThread = 16;
// The sort enumerates the pixels tile by tile (tile_pixel, RTX_QUEUE_TILE x
// RTX_QUEUE_TILE tiles; 0: row-major): a bucket then lists a tile's pixels
// together, so a wave's run of consecutive slots comes from a compact patch
// of the image (C2 37.7 -> 35.8 ms with the layer grid).
#ifndef RTX_QUEUE_TILE
#define RTX_QUEUE_TILE 16
#endif
constexpr uint32_t kQueueTile = RTX_QUEUE_TILE;
constexpr uint32_t kChunkShare = 16;  // the private runs of large scenes and medium shares (launch_render)

__global__ void __launch_bounds__(kBlock) k_cost_hist(const uint32_t *cost, uint32_t width, uint32_t rows,
                                                      uint32_t cost_spp, uint32_t sat_cap, uint32_t tile,
                                                      uint32_t tile_y, uint32_t *counts) {
    __shared__ uint32_t h[kCostBuckets];
    for (uint32_t b = threadIdx.x; b < kCostBuckets; b += kBlock) h[b] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * kBlock * kSortPerThread;
    for (uint32_t k = 0; k < kSortPerThread; ++k) {
        const uint32_t i = tile_pixel(base + k * kBlock + threadIdx.x, width, rows, tile, tile_y);
        if (i != ~0u) atomicAdd(&h[cost_key(cost, i, width, rows, cost_spp, sat_cap)], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < kCostBuckets; b += kBlock)
        if (h[b]) atomicAdd(&counts[b], h[b]);
}

// Positions: bucket start (prefix of the global counts) + a range the
// block reserves in the bucket + the element's rank inside the block: the
// enumeration's order (tile-major) within a bucket, blocks in any order.
// Per-pixel results do not depend on it.
__global__ void __launch_bounds__(kBlock) k_cost_scatter(const uint32_t *cost, uint32_t width, uint32_t rows,
                                                         uint32_t cost_spp, uint32_t sat_cap, uint32_t tile,
                                                         uint32_t tile_y,
                                                         const uint32_t *counts, uint32_t *cursors,
                                                         uint32_t *perm, uint32_t *inv) {
    __shared__ uint32_t h[kCostBuckets], start[kCostBuckets];
    for (uint32_t b = threadIdx.x; b < kCostBuckets; b += kBlock) h[b] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * kBlock * kSortPerThread;
    uint32_t rank[kSortPerThread], key[kSortPerThread];
    for (uint32_t k = 0; k < kSortPerThread; ++k) {
        const uint32_t i = tile_pixel(base + k * kBlock + threadIdx.x, width, rows, tile, tile_y);
        key[k] = i != ~0u ? cost_key(cost, i, width, rows, cost_spp, sat_cap) : 0u;
        rank[k] = i != ~0u ? atomicAdd(&h[key[k]], 1u) : 0u;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t pre = 0;
        for (uint32_t b = 0; b < kCostBuckets; ++b) {
            start[b] = pre;
            pre += counts[b];
        }
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < kCostBuckets; b += kBlock)
        if (h[b]) start[b] += atomicAdd(&cursors[b], h[b]);
    __syncthreads();
    for (uint32_t k = 0; k < kSortPerThread; ++k) {
        const uint32_t i = tile_pixel(base + k * kBlock + threadIdx.x, width, rows, tile, tile_y);
        if (i != ~0u) {
            const uint32_t g = start[key[k]] + rank[k];
            perm[g] = i;
            if (inv) inv[i] = g;  // coalesced: pixel i's queue slot (k_unpermute)
        }
    }
}

// Heavy-pixel split: with key k ~ a pixel's cost, a lane's share of the
// frame is W / lanes (W = sum of keys). Pixels whose key exceeds
// a1 times it form tier 1 (slots [0, k1): one pixel per wave,
// 64 lanes per ray). When there are fewer pixels than rho per
// resident lane (a small share of a frame, e.g. one GPU's rows of an 8-GPU
// split), the tier-1 bar rises to a1_small times the share
// and the pixels above a2_small times it (up to that bar) form tier
// 2 (slots [k1, kh), kHeavy2 per wave). Tiers and bars were chosen with
// tools/part_scaling.py on C2 split 1/2/4/8 ways (the defaults below);
// rtx_set_schedule (include/rtx.h) replaces them per context, and
// tools/heavy_sweep.py sweeps them through it. Writes kh to heavy[1] and
// k1 to heavy[3]. One thread: 256 buckets.
}  // namespace
KTune default_tune() {
    KTune t;
    t.a1 = kHeavy1Alpha;
    t.a1_small = kHeavy1AlphaSmall;
    t.a1_low = kHeavy1AlphaLow;
    t.a2_small = kHeavyAlpha;
    t.a2_medium = kHeavy2AlphaMedium;
    t.a2_large = kHeavy2AlphaLarge;
    t.rho = kHeavyRho;
    t.rho_low = kHeavyRhoLow;
    t.rho2 = kHeavyRho2;
    t.prio_frac = kPrioFracX100 / 100.0;
    t.occ_small = t.occ_low = t.occ_normal = 1.0;
    t.coop_max = (uint32_t)kCoopMax;
    t.coop_max_large = (uint32_t)kCoopMaxLarge;
    t.prio_t1 = 3;
    t.prio_t2 = 2;
    t.prio_hot = 3;
    t.chunk = 64;  // C2 35.9 -> 33.0 ms with the queue tiles (16 until S6u: 45.9 -> 44.5 ms then, R3w_*, R3x_*)
    t.trace_small = kTraceSmall;
    t.trace_low = kTraceLow;
    t.trace_medium = kTraceMedium;
    t.trace_large = kTraceLarge;
    t.prom_small = kPromSmall;
    t.prom_low = kPromLow;
    t.prom_medium = kPromMedium;
    t.prom_large = kPromLarge;
    t.prom_big = kPromBig;
    t.trace_group = kTraceGroup;
    t.trace_solo = kTraceSolo;
    t.cap_split = kCapSplit;
    t.dyn1 = kDynPrio1;
    t.dyn2 = kDynPrio2;
    t.dyn3 = kDynPrio3;
    return t;
}
namespace {
__global__ void k_heavy_split(const uint32_t *counts, uint32_t npix, uint32_t lanes, uint32_t spp, uint32_t *heavy,
                              const KTune t) {
    if (threadIdx.x != 0u) return;
    double w = 0.0;
    for (uint32_t b = 0; b < kCostBuckets; ++b) w += (double)counts[b] * (double)(kCostBuckets - 1u - b);
    const double share = w / (double)(lanes ? lanes : 1u);
    const bool small = (double)npix < t.rho * (double)lanes;
    // fewer than rho_low pixels per lane (a 4-way split of C2): tier 1
    // only above a1_low x share — one-ray waves are expensive, and
    // at this share there are many candidates that crowd the SIMDs
    const bool low = !small && (double)npix < t.rho_low * (double)lanes;
    const double a1 = small ? t.a1_small : low ? t.a1_low : t.a1;
    // a medium share (fewer than rho2 pixels per lane, e.g. a
    // 2- or 4-way split) also gets tier 2 above a2_medium x share
    const bool medium = !small && (double)npix < t.rho2 * (double)lanes;
    const double a2 = small ? t.a2_small : medium ? min(t.a2_medium, a1) : min(t.a2_large, a1);
    uint32_t kh = 0, k1 = 0, k0 = 0;
    for (uint32_t b = 0; b < kCostBuckets; ++b) {
        const double key = (double)(kCostBuckets - 1u - b);
        if (key > a2 * share) kh += counts[b];
        if (key > a1 * share) k1 += counts[b];
        if (key > t.trace_solo * share) k0 += counts[b];  // k_trace: one pixel per wave
    }
    heavy[1] = kh;
    heavy[3] = k1;
    heavy[4] = k0;
    // the mean pixel's segments at the full spp (keys: 9 one-sample costs; saturated keys count as the top bucket)
    heavy[5] = __float_as_uint((float)(w / (double)(npix ? npix : 1u) / 9.0 * (double)spp));
}

// ---- per-sample RNG (rtx_frame.rng_mode 1): one lane per (pixel, sample) --
// Every (pixel, sample) has its own seed (pixel_seed), so samples are
// independent and the north star's kernel shape applies: a lane traces ONE
// sample. A wave takes batches of consecutive pixels from the global queue
// (one atomic per batch); a batch's npx * spp items (pixel-major: item =
// po * spp + s) go to the wave's lanes as they free up, so lanes stay busy
// across path lengths (1..depth segments) without waiting for each other. A
// finished sample stores its colour (col * sky, or +0 for a black path) into
// the wave's scratch at [slot][s * npx + po] (float4); when all items of a
// batch are done, lane po folds its pixel's colours IN SAMPLE ORDER —
// acc = ((0 + c_0) + c_1) + ... — which is bit for bit the reference's
// accumulation (:304-312; adding +0 for a black sample leaves acc unchanged:
// acc starts at +0 and is never -0), and the batch's pixels are written with
// one coalesced store.
// kPsSlots batch slots per wave: lanes move on to new batches while earlier
// ones wait for a long path; a wave stalls only when every slot holds an
// unfinished, fully issued batch. Batches are ps_px pixels (<= ps_cap
// items; the host makes them smaller for a small frame share, so that every
// wave gets ~20 and the waves finish together). Scratch stays small
// (kPsSlots * ps_cap * 16 B per wave: in the 256 MB MALL), which measured
// faster than large batches (A/B in DESIGN.md §7). Once the queue is empty
// and a wave has at most kCoopMax samples left, it traces them with the
// group coop of the chain kernel (several lanes per ray), at a raised wave
// priority: the frame's last, longest paths end sooner.
#ifndef RTX_PS_ITEM_MAJOR  // per-sample scratch layout: 1 = item-major (37.6 vs 38.5 ms, 8.8 vs 13.5 GB per C2 frame: R3u), 0 = sample-major
#define RTX_PS_ITEM_MAJOR 1
#endif
constexpr int kPsSlots = 4;
constexpr uint32_t kPsStateBytes = (kRB / 64) * kPsSlots * 4 * sizeof(uint32_t);  // per block
struct PsLane {
    f3 o, d, col;
    float a, inv_a, seed;
    uint32_t bounce, segs;
    uint32_t slot;  // batch slot of the sample
    uint32_t sidx;  // s * npx + po: the sample's scratch index in its slot
    bool active;
};

__device__ __forceinline__ void ps_start(const KParams &P, const Frame &F, uint32_t px0, uint32_t npx,
                                         uint32_t slot, uint32_t item, PsLane &L) {
    const uint32_t po = item / P.spp;
    const uint32_t s = item - po * P.spp;
    uint32_t x, y;
    lane_pixel(P, px0 + po, x, y);
    L.seed = pixel_seed(P, x, y, s);
    f3 o, d;
    start_sample(F, x, y, L.seed, o, d);
    L.o = o;
    L.d = d;
    L.a = dir_len2(d);
    L.inv_a = 1.0f / L.a;
    L.col = mk3(1.0f, 1.0f, 1.0f);
    L.bounce = 0;
    L.slot = slot;
    L.sidx = RTX_PS_ITEM_MAJOR ? item : s * npx + po;
    L.active = true;
}

// Fold a completed batch of npx pixels from px0 (all lanes of the wave call
// it; lane po < npx owns pixel px0 + po) and write its pixels.
__device__ __forceinline__ void ps_fold(const KParams &P, uint32_t px0, uint32_t npx, const float4 *c) {
    // this wave's scratch stores complete before its loads below. Workgroup
    // scope is enough (the same wave; the CU's L1 is coherent within a
    // workgroup) and cheap: an agent-scope fence also writes back the L2.
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    const uint32_t po = threadIdx.x & 63u;
    if (po >= npx) return;
    f3 acc = mk3(0.0f, 0.0f, 0.0f);
    uint32_t s = 0;
    // sample s of pixel po: [s * npx + po] (sample-major), or [po * spp + s]
    // (item-major: the order the lanes take the items in)
    const uint32_t ss = RTX_PS_ITEM_MAJOR ? 1u : npx;
    if (RTX_PS_ITEM_MAJOR) c += po * P.spp;
    else c += po;
    for (; s + 8 <= P.spp; s += 8) {  // eight samples' loads in flight, adds in order
        float4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = c[(s + k) * ss];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc = acc + mk3(v[k].x, v[k].y, v[k].z);
    }
    for (; s < P.spp; ++s) {
        const float4 v = c[s * ss];
        acc = acc + mk3(v.x, v.y, v.z);
    }
    output_pixel(P, px0 + po, acc);
}

template <bool kPF, bool kLin = false>
__global__ void RTX_PS_BOUNDS_T(kPF) k_render_ps(const KParams P) {
    constexpr bool kCulled = kPF && RTX_CULL && !kLin;  // the culled scan (large scenes, not the linear mode)
    // dynamic LDS: [candidate list, list_bytes<kPF>][coop rays, kCoopBytes][batch slots, kPsStateBytes]
    //              [LDS copy of the spheres (n <= kCoopLds)]
    extern __shared__ __attribute__((aligned(16))) unsigned char s_mem[];
    uint32_t *list = reinterpret_cast<uint32_t *>(s_mem);
    constexpr uint32_t kLB = list_bytes<kPF>();
    float *coop_ws = reinterpret_cast<float *>(s_mem + kLB) + (threadIdx.x / 64) * (kCoopWaveBytes / 4);
    // this wave's batch slots: [k][0 px0, 1 npx, 2 items (0 = free), 3 items done]
    uint32_t *st = reinterpret_cast<uint32_t *>(s_mem + kLB + kCoopBytes) + (threadIdx.x / 64) * kPsSlots * 4;
    const bool sph_lds = !kPF && P.scene.n <= kCoopLds;
    const SphLds sl = lds_copy(P.scene, reinterpret_cast<float *>(s_mem + kLB + kCoopBytes + kPsStateBytes), sph_lds);
    const SphGlobal sg = sph_global(P.scene);
    const uint32_t lane = threadIdx.x & 63u;
    if (lane < kPsSlots * 4) st[lane] = 0u;
    __syncthreads();
    const int last = (int)P.scene.n - 1;
    const Frame F = load_frame(P);
    const uint32_t npix = P.rows_local * P.width;
    const uint32_t wave = blockIdx.x * (kRB / 64) + threadIdx.x / 64;
    float4 *scr = reinterpret_cast<float4 *>(P.ps_scratch) + (size_t)wave * kPsSlots * P.ps_cap;  // [slot][ps_cap]
    const unsigned long long t_start = P.wave_times ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const unsigned long long c_start = P.wave_times ? __builtin_amdgcn_s_memtime() : 0ull;
    PsLane L;
    L.active = false;
    L.segs = 0;
    // the slot being issued (wave-uniform): its slot index, first pixel, pixels, items, items issued
    uint32_t cur = 0, c_px0 = 0, c_npx = 0, c_total = 0, c_issued = 0;
    bool exhausted = false;
    for (;;) {
        // hand the idle lanes the next items: of batch `cur`, then of a new batch
        for (int pass = 0; pass < 2; ++pass) {
            const uint64_t idle = __ballot(!L.active);
            if (idle == 0ull) break;
            if (c_issued == c_total) {
                if (exhausted) break;
                const uint64_t freem = __ballot(lane < (uint32_t)kPsSlots && st[4 * lane + 2] == 0u);
                if (freem == 0ull) break;  // every slot waits for its last samples
                const uint32_t fk = (uint32_t)__builtin_ctzll(freem);
                uint32_t base = 0;
                if (lane == 0u) base = atomicAdd(P.queue, P.ps_px);
                base = (uint32_t)__shfl((int)base, 0, 64);
                if (base >= npix) {
                    exhausted = true;
                    break;
                }
                cur = fk;
                c_px0 = base;
                c_npx = min(P.ps_px, npix - base);
                c_total = c_npx * P.spp;
                c_issued = 0;
                if (lane == 0u) {
                    st[4 * fk + 0] = c_px0;
                    st[4 * fk + 1] = c_npx;
                    st[4 * fk + 3] = 0u;
                    st[4 * fk + 2] = c_total;
                }
            }
            const uint32_t take = min((uint32_t)__popcll(idle), c_total - c_issued);
            const uint32_t rank =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
            if (!L.active && rank < take) ps_start(P, F, c_px0, c_npx, cur, c_issued + rank, L);
            c_issued += take;
        }
        if (__ballot(L.active) == 0ull) break;  // queue exhausted and every batch folded
        bool ended = false;
        const uint64_t act = __ballot(L.active);
        float best = __uint_as_float(0x7f800000u);
        int hit = -1;
        if (exhausted && __popcll(act) <= kCoopMax) {  // the wave's last few samples: group coop
            __builtin_amdgcn_s_setprio(kTailPrio);
            bool seq = false;
            hit = kCulled  // (no breadth-first one-ray walk here: its registers cost this kernel 16 %, R9f)
                      ? hit_world_groups_culled<false>(P.scene, act, L.active, L.o, L.d, L.a, L.inv_a, kTMin, coop_ws,
                                                       best, seq)
                  : sph_lds ? hit_world_groups(P.scene, sl, act, L.active, L.o, L.d, L.a, L.inv_a, kTMin, coop_ws, best,
                                               seq)
                            : hit_world_groups(P.scene, sg, act, L.active, L.o, L.d, L.a, L.inv_a, kTMin, coop_ws, best,
                                               seq);
            if (L.active && seq) {  // a non-finite root in the group: the exact path
                best = __uint_as_float(0x7f800000u);
                hit = hit_world_pre<kPF>(P.scene, L.o, L.d, L.a, L.inv_a, kTMin, best, list);
            }
        } else if (L.active) {  // (the SGPR scan: the LDS tile measured slower here)
            hit = kCulled ? hit_world_culled(P.scene, L.o, L.d, L.a, L.inv_a, kTMin, best, list)
                  : sph_lds ? hit_world_pre_ld<kPF>(P.scene, [sl](uint32_t i) { return sl.sphere(i); }, L.o, L.d, L.a,
                                                    L.inv_a, kTMin, best, list)
                            : hit_world_pre<kPF>(P.scene, L.o, L.d, L.a, L.inv_a, kTMin, best, list);
        }
        if (L.active) {
            L.segs++;
            f3 c = mk3(0.0f, 0.0f, 0.0f);
            const int r = path_segment(P, L, min(hit, last), best, c);
            if (r != kSegContinue) {
                scr[(size_t)L.slot * P.ps_cap + L.sidx] = make_float4(c.x, c.y, c.z, 0.0f);  // +0: black path
                atomicAdd(&st[4 * L.slot + 3], 1u);
                L.active = false;
                ended = true;
            }
        }
        if (__ballot(ended) == 0ull) continue;
        // fold every batch whose samples are all done
        uint64_t full = __ballot(lane < (uint32_t)kPsSlots && st[4 * lane + 2] != 0u &&
                                 st[4 * lane + 3] == st[4 * lane + 2]);
        while (full != 0ull) {
            const uint32_t k = (uint32_t)__builtin_ctzll(full);
            full &= full - 1ull;
            ps_fold(P, st[4 * k + 0], st[4 * k + 1], scr + (size_t)k * P.ps_cap);
            if (lane == 0u) st[4 * k + 2] = 0u;
        }
    }
    uint32_t wsegs = L.segs;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) wsegs += __shfl_xor(wsegs, off, 64);
    count_segments(P, L.segs);
    // diagnostic only (rtx_debug_wave_times, armed with 2 x waves): per wave
    // (start, end) s_memrealtime, then (shader clocks, segments) in the upper half
    if (!RTX_DIAG_RAYS && P.wave_times && lane == 0u && wave < P.wave_cap / 2) {
        P.wave_times[2 * wave] = t_start;
        P.wave_times[2 * wave + 1] = __builtin_amdgcn_s_memrealtime();
        P.wave_times[P.wave_cap + 2 * wave] = __builtin_amdgcn_s_memtime() - c_start;
        P.wave_times[P.wave_cap + 2 * wave + 1] = wsegs;
    }
}

// spp == 0 or depth == 0: no segment is traced; the pixel is
// toGamma(0 / spp) (accColor stays 0; 0/0 = NaN for spp == 0, :312-313).
__global__ void __launch_bounds__(kBlock) k_render_trivial(const KParams P) {
    const uint32_t gid = blockIdx.x * kBlock + threadIdx.x;
    if (gid >= P.rows_local * P.width) return;
    Lane L;
    L.acc = mk3(0.0f, 0.0f, 0.0f);
    L.gid = gid;
    write_pixel(P, L);
}

// Gathered [nparts][max_rows][width] -> image [height][width].
__global__ void __launch_bounds__(kBlock) k_deinterleave(const float4 *__restrict__ g,
                                                         float4 *__restrict__ img, uint32_t width,
                                                         uint32_t height, uint32_t tile_rows,
                                                         uint32_t nparts, uint32_t max_rows) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= (uint64_t)width * height) return;
    const uint32_t y = (uint32_t)(i / width);
    const uint32_t x = (uint32_t)(i - (uint64_t)y * width);
    const uint32_t tile = y / tile_rows;
    const uint32_t part = tile % nparts;
    const uint32_t lr = (tile / nparts) * tile_rows + (y - tile * tile_rows);
    img[i] = g[((uint64_t)part * max_rows + lr) * width + x];
}

// The cost-ordered render's image, from its slot-ordered staging buffer to
// the linear framebuffer (ShaderCompute.hlsl:314's one texel per pixel, in
// pixel order): pixel i is stage[inv[i]], read gathered, stored coalesced.
// Only slots this launch staged are moved (w holds the launch's tag,
// KParams::stage_tag): a promoted pixel (stage w = 0) was written to out[i] by
// whoever finished it, and a slot a launch left unwritten (the valve fired:
// RTX_ERR_INCOMPLETE) keeps out[i] as it was, never another frame's pixel.
__global__ void __launch_bounds__(kBlock) k_unpermute(const float4 *__restrict__ stage, const uint32_t *__restrict__ inv,
                                                      uint32_t npix, uint32_t tag, float4 *__restrict__ out) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= npix) return;
    const float4 v = stage[inv[i]];
    if (__float_as_uint(v.w) == tag) out[i] = make_float4(v.x, v.y, v.z, 1.0f);
}

// One hit record of rtx_debug_hit_world (include/rtx.h): hit, t, p, normal,
// front_face, sphere index.
__device__ __forceinline__ void debug_record(const KScene &S, f3 o, f3 d, float best, int idx, float *r) {
    if (idx < 0) {
        for (int k = 0; k < 10; ++k) r[k] = 0.0f;
        r[9] = -1.0f;
        return;
    }
    const float4 sc = S.cen[idx];
    const f3 p = o + best * d;
    const float inv_r = 1.0f / sc.w;
    f3 nrm = inv_r * (p - mk3(sc.x, sc.y, sc.z));
    const bool ff = dot3(d, nrm) < 0.0f;
    if (!ff) nrm = -nrm;
    r[0] = 1.0f;
    r[1] = best;
    r[2] = p.x; r[3] = p.y; r[4] = p.z;
    r[5] = nrm.x; r[6] = nrm.y; r[7] = nrm.z;
    r[8] = ff ? 1.0f : 0.0f;
    r[9] = (float)idx;
}

// t_min > 0 and t_max >= t_min (rtx_debug_hit_world checks): the resolve
// orders roots by their bits (hit_key). start = kDebugCulled: the culled
// scan (k_render's lane mode for scenes with KScene::cpre), when the scene has it.
constexpr uint32_t kDebugCulled = 0xffffffffu;
__global__ void __launch_bounds__(kRB) k_debug_hit_world(const KScene S, const float *rays,
                                                            uint32_t nrays, float t_min,
                                                            float t_max, uint32_t start, float *out) {
    __shared__ uint32_t list[list_bytes<true>() > kListBytes ? list_bytes<true>() / sizeof(uint32_t)
                                                             : kListBytes / sizeof(uint32_t)];
    const uint32_t i = blockIdx.x * kRB + threadIdx.x;
    if (i >= nrays) return;
    const f3 o = mk3(rays[6 * i + 0], rays[6 * i + 1], rays[6 * i + 2]);
    const f3 d = mk3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
    const float a = dir_len2(d);
    const float inv_a = 1.0f / a;
    float best = t_max;
    const int idx =
        min((start == kDebugCulled && S.cpre)
                ? hit_world_culled(S, o, d, a, inv_a, t_min, best, list)
            : S.n_pad > kScanPfMin ? hit_world_pre<true>(S, o, d, a, inv_a, t_min, best, list, nullptr, start)
                                   : hit_world_pre<false>(S, o, d, a, inv_a, t_min, best, list, nullptr, start),
            (int)S.n - 1);
    debug_record(S, o, d, best, idx, out + 10 * (size_t)i);
}

// start = kDebugCulledCoop | q (q in 1..64): the culled group coop
// (hit_world_groups_culled, the large-scene tail / heavy tiers) with q rays
// per wave, i.e. 64 / 2^ceil(log2 q) lanes per ray (q > 32: two chunks of
// 32 rays at 2 lanes each); a ray whose group met a non-finite root takes
// the in-order path, as in the render. kDebugCulledCoopLane | q: the same
// with the per-lane walk (hit_world_groups_culled<false>: k_render_ps's
// form, whose one-ray case q = 1 the breadth-first selector never runs).
constexpr uint32_t kDebugCulledCoop = 0xffffff00u;
constexpr uint32_t kDebugCulledCoopLane = 0xfffffe00u;
template <bool kBfs>
__global__ void __launch_bounds__(kRB) k_debug_hit_world_coop(const KScene S, const float *rays, uint32_t nrays,
                                                              float t_min, float t_max, uint32_t q, float *out) {
    __shared__ uint32_t list[list_bytes<true>() / sizeof(uint32_t)];
    __shared__ float ws_all[(kRB / 64) * (kCoopWaveBytes / 4)];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x / 64u;
    const uint32_t i = (blockIdx.x * (kRB / 64u) + w) * q + lane;
    const bool active = lane < q && i < nrays;
    f3 o = mk3(0.0f, 0.0f, 0.0f), d = mk3(1.0f, 0.0f, 0.0f);
    if (active) {
        o = mk3(rays[6 * i + 0], rays[6 * i + 1], rays[6 * i + 2]);
        d = mk3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
    }
    const float a = dir_len2(d);
    const float inv_a = 1.0f / a;
    float best = t_max;
    bool seq = false;
    int idx = hit_world_groups_culled<kBfs>(S, __ballot(active), active, o, d, a, inv_a, t_min,
                                            ws_all + w * (kCoopWaveBytes / 4), best, seq);
    if (!active) return;
    if (seq) {
        best = t_max;
        idx = hit_world_pre<true>(S, o, d, a, inv_a, t_min, best, list);
    }
    debug_record(S, o, d, best, min(idx, (int)S.n - 1), out + 10 * (size_t)i);
}

// Issue-rate probe of hit_world's own instruction mix (rtx_debug_scan_rate,
// VERDICT r4 item 3): a full-occupancy grid of the render's shape (same
// workgroup size, register budget and LDS: list, coop slots, the scene's LDS
// copy) in which every lane takes one primary ray of the frame (pixel
// gid * 7919 mod npix: a spread over the image) and runs k_render's lane-mode
// hit_world on it `reps` times — the prefiltered scan and the resolve, nothing
// else. Its VALU issue rate over the launch (SQ_INSTS_VALU / SIMD-cycles) is
// what that mix sustains at the render's occupancy: the ceiling the render's
// scan section can reach. Scenes up to kCoopLds spheres (the headline's).
__global__ void RTX_RENDER_BOUNDS k_debug_scan_rate(const KParams P, uint32_t reps, unsigned long long *sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned char s_mem[];
    uint32_t *list = reinterpret_cast<uint32_t *>(s_mem);
    const SphLds sl = lds_copy(P.scene, reinterpret_cast<float *>(s_mem + kListBytes + kCoopBytes), true);
    __syncthreads();
    const uint32_t npix = P.rows_local * P.width;
    const uint32_t gid = blockIdx.x * kRB + threadIdx.x;
    const uint32_t px = (uint32_t)(((uint64_t)gid * 7919u) % npix);
    uint32_t x, y;
    lane_pixel(P, px, x, y);
    float seed = pixel_seed(P, x, y, 0);
    f3 o, d;
    start_sample(Frame{}, x, y, seed, o, d);
    const float a = dir_len2(d);
    const float inv_a = 1.0f / a;
    uint32_t acc = 0;
    for (uint32_t r = 0; r < reps; ++r) {
        float best = __uint_as_float(0x7f800000u);
        const int hit = hit_world_pre_ld<false>(P.scene, [sl](uint32_t i) { return sl.sphere(i); }, o, d, a, inv_a,
                                                kTMin, best, list, nullptr, 0, RTX_SCAN_LDS ? sl.pr : nullptr);
        acc += (uint32_t)hit ^ __float_as_uint(best);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += (uint32_t)__shfl_xor((int)acc, off, 64);
    if ((threadIdx.x & 63u) == 0u) atomicAdd(sink, (unsigned long long)acc);
}

__global__ void __launch_bounds__(kBlock) k_debug_math(int fn, const float *in0, const float *in1,
                                                       uint32_t n, float *out) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    if (fn == 12 || fn == 13) {  // diffuse direction: in0 = p[3n], in1 = (normal, rius)[6n]
        const f3 p = mk3(in0[3 * i], in0[3 * i + 1], in0[3 * i + 2]);
        const f3 nrm = mk3(in1[6 * i], in1[6 * i + 1], in1[6 * i + 2]);
        const f3 rius = mk3(in1[6 * i + 3], in1[6 * i + 4], in1[6 * i + 5]);
        const f3 dir = normalize3(lambert_guard(((p + nrm) + rius) - p, nrm, fn == 13));
        out[3 * i] = dir.x;
        out[3 * i + 1] = dir.y;
        out[3 * i + 2] = dir.z;
        return;
    }
    const float a = in0[i];
    const float b = in1 ? in1[i] : 0.0f;
    float seed = a;
    switch (fn) {
        case 0: out[i] = sqrt_rn(a); break;
        case 1: out[i] = a / b; break;
        case 2: { float s, c; sincos_rt(a, s, c); out[i] = s; } break;
        case 3: { float s, c; sincos_rt(a, s, c); out[i] = c; } break;
        case 4: out[i] = log2_rt(a); break;
        case 5: out[i] = exp2_rt(a); break;
        case 6: out[i] = pow_rt(a, b); break;
        case 7: out[i] = __uint_as_float(base_hash(__float_as_uint(a), __float_as_uint(b))); break;
        case 8: out[3 * i] = hash1(seed); out[3 * i + 1] = seed; out[3 * i + 2] = 0.0f; break;
        case 9: hash2(seed, out[3 * i], out[3 * i + 1]); out[3 * i + 2] = seed; break;
        case 10: { const f3 h = hash3(seed); out[3 * i] = h.x; out[3 * i + 1] = h.y; out[3 * i + 2] = h.z; } break;
        case 11: { const f3 r = random_in_unit_sphere(seed); out[3 * i] = r.x; out[3 * i + 1] = r.y; out[3 * i + 2] = r.z; } break;
        default: out[i] = 0.0f;
    }
}

inline uint32_t ceil_div(uint64_t a, uint32_t b) { return (uint32_t)((a + b - 1) / b); }

}  // namespace

// Workgroups the device keeps resident for `kern` (per-CU occupancy x CUs),
// queried once per (device, kernel, LDS size) and cached: the occupancy query
// costs host time inside every launch's timed region otherwise. Over-
// estimating is harmless: extra workgroups find the queue drained and exit.
static uint32_t resident_blocks(const void *kern, size_t lds) {
    struct Entry {
        int dev;
        const void *kern;
        size_t lds;
        uint32_t blocks;
    };
    static std::mutex mu;
    static std::vector<Entry> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 1024;
    {
        std::lock_guard<std::mutex> g(mu);
        for (const Entry &e : cache)
            if (e.dev == dev && e.kern == kern && e.lds == lds) return e.blocks;
    }
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 1024;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, (int)kRB, lds) != hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    const uint32_t blocks = (uint32_t)(cus * per_cu);
    std::lock_guard<std::mutex> g(mu);
    cache.push_back(Entry{dev, kern, lds, blocks});
    return blocks;
}

// Dynamic LDS above 64 KiB must be opted into per kernel.
static hipError_t allow_lds(const void *kern, size_t lds) {
    if (lds <= 65536) return hipSuccess;
    return hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

// k_render with the SGPR double-buffered scan for scenes whose `pre` array
// does not stay in the scalar cache (kScanPfMin).
static bool use_pf(const KScene &s) { return s.n_pad > kScanPfMin; }
// The linear-scan mode (rtx_set_scan_mode RTX_SCAN_LINEAR, or an RTX_CULL=0
// build): a large scene uploaded without the culled layout; its kernels scan
// every block of every segment (the reference's Hittable_list order of work,
// with the prefilter), through the per-wave LDS tile in the chain render.
static bool use_lin(const KScene &s) { return use_pf(s) && s.cpre == nullptr; }
template <bool kPersist, bool kCost>
static const void *render_fn(const KScene &s) {
    return !use_pf(s)   ? (const void *)k_render<kPersist, kCost, false>
           : use_lin(s) ? (const void *)k_render<kPersist, kCost, true, true>
                        : (const void *)k_render<kPersist, kCost, true>;
}
template <bool kPersist, bool kCost>
static void launch_k(const KScene &s, uint32_t blocks, size_t lds, hipStream_t stream, const KParams &a) {
    if (!use_pf(s))
        hipLaunchKernelGGL((k_render<kPersist, kCost, false>), dim3(blocks), dim3(kRB), lds, stream, a);
    else if (use_lin(s))
        hipLaunchKernelGGL((k_render<kPersist, kCost, true, true>), dim3(blocks), dim3(kRB), lds, stream, a);
    else
        hipLaunchKernelGGL((k_render<kPersist, kCost, true>), dim3(blocks), dim3(kRB), lds, stream, a);
}

// Dynamic LDS of the chain-RNG kernels: candidate lists + coop ray slots +
// the block's copy of the spheres for scenes up to kCoopLds.
static size_t render_lds(const KScene &s) {
    return (use_pf(s) ? list_bytes<true>() + 16 + (use_lin(s) ? kPfLdsBytes : 0u) : kListBytes) + kCoopBytes +  // kPF: the pack word (and the tile scan's tile)
           (s.n <= kCoopLds ? (size_t)coop_lds_bytes(s.n) : 0);
}

hipError_t launch_cost(const KParams &p, hipStream_t stream) {
    const uint64_t lanes = (uint64_t)p.rows_local * p.width;
    if (lanes == 0 || p.spp == 0 || p.depth == 0 || !p.cost_out) return hipErrorInvalidValue;
    const size_t lds = render_lds(p.scene);
    hipError_t e = allow_lds(render_fn<false, true>(p.scene), lds);
    if (e != hipSuccess) return e;
    launch_k<false, true>(p.scene, ceil_div(tile_span(p.width, p.rows_local, kExactTile), kRB), lds, stream, p);
    return hipGetLastError();
}

// Per-sample launches: items per batch slot (ps_cap = max(kPsItems, spp)); a
// batch is at most ps_px pixels, ps_px * spp <= ps_cap.
#ifndef RTX_PS_ITEMS
#define RTX_PS_ITEMS 512
#endif
constexpr uint32_t kPsItems = RTX_PS_ITEMS;
#ifndef RTX_PS_BPW
#define RTX_PS_BPW 40
#endif
constexpr uint32_t kPsBatchesPerWave = RTX_PS_BPW;
static size_t ps_lds(const KScene &s) {
    return (use_pf(s) ? list_bytes<true>() : kListBytes) + kCoopBytes + kPsStateBytes +
           (!use_pf(s) && s.n <= kCoopLds ? (size_t)coop_lds_bytes(s.n) : 0);
}
static const void *ps_fn(const KScene &s) {
    return !use_pf(s)   ? (const void *)k_render_ps<false>
           : use_lin(s) ? (const void *)k_render_ps<true, true>
                        : (const void *)k_render_ps<true>;
}
static uint32_t ps_cap_of(uint32_t spp) { return max(kPsItems, spp); }
// Every resident wave (an item is a sample, not a pixel: a frame share with
// fewer pixels than lanes still fills the GPU), fewer only for tiny frames.
static uint32_t ps_waves(const KParams &p) {
    const uint64_t items = (uint64_t)p.rows_local * p.width * p.spp;
    const uint32_t blocks = min(ceil_div(items, kRB), resident_blocks(ps_fn(p.scene), ps_lds(p.scene)));
    return blocks * (kRB / 64);
}
size_t ps_scratch_floats(const KParams &p) {
    if (p.rng_mode != 1u || p.spp == 0 || p.depth == 0 || (uint64_t)p.rows_local * p.width == 0) return 0;
    return (size_t)ps_waves(p) * kPsSlots * 4 * ps_cap_of(p.spp);
}
static hipError_t launch_ps(const KParams &p, const KSchedule &sched, hipStream_t stream) {
    const size_t lds = ps_lds(p.scene);
    hipError_t e = allow_lds(ps_fn(p.scene), lds);
    if (e != hipSuccess) return e;
    const uint32_t waves = ps_waves(p);
    KParams q = p;
    q.ps_cap = ps_cap_of(p.spp);
    q.ps_scratch = sched.ps_scratch;
    if (!q.ps_scratch || sched.ps_floats < (size_t)waves * kPsSlots * 4 * q.ps_cap) return hipErrorInvalidValue;
    // batches of <= ps_cap items, and about kPsBatchesPerWave of them per
    // wave for a small frame share (the waves then finish together)
    const uint64_t per_wave = (uint64_t)p.rows_local * p.width * p.spp / std::max(waves, 1u);
    const uint64_t items = std::min<uint64_t>(q.ps_cap, per_wave / kPsBatchesPerWave);
    q.ps_px = (uint32_t)std::max<uint64_t>(1u, std::min<uint64_t>(64u, items / p.spp));
    e = hipMemsetAsync(p.queue, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    const uint32_t blocks = waves / (kRB / 64);
    if (!use_pf(p.scene))
        hipLaunchKernelGGL(k_render_ps<false>, dim3(blocks), dim3(kRB), lds, stream, q);
    else if (use_lin(p.scene))
        hipLaunchKernelGGL((k_render_ps<true, true>), dim3(blocks), dim3(kRB), lds, stream, q);
    else
        hipLaunchKernelGGL(k_render_ps<true>, dim3(blocks), dim3(kRB), lds, stream, q);
    return hipGetLastError();
}

hipError_t launch_render(const KParams &p_in, const KSchedule &sched, hipStream_t stream) {
    const KTune &tune = sched.tune;  // validated by rtx_set_schedule
    KParams p = p_in;
    p.coop_max = min(max(p.scene.n <= kCoopLds ? tune.coop_max : tune.coop_max_large, 1u), 64u);
    p.prio_t1 = tune.prio_t1;
    p.prio_t2 = tune.prio_t2;
    p.prio_hot = tune.prio_hot;
    p.chunk = 0;
    const uint64_t lanes = (uint64_t)p.rows_local * p.width;
    if (lanes == 0) return hipSuccess;
    const uint32_t need = ceil_div(lanes, kRB);
    const uint32_t need_x = ceil_div(tile_span(p.width, p.rows_local, kExactTile), kRB);  // the exact grid's blocks
    if (p.spp == 0 || p.depth == 0) {
        hipLaunchKernelGGL(k_render_trivial, dim3(ceil_div(lanes, kBlock)), dim3(kBlock), 0, stream, p);
        return hipGetLastError();
    }
    if (p.rng_mode == 1u) return launch_ps(p, sched, stream);  // one lane per (pixel, sample)
    const bool pf = use_pf(p.scene);
    const size_t lds = render_lds(p.scene);
    hipError_t e = allow_lds(render_fn<true, false>(p.scene), lds);
    if (e == hipSuccess) e = allow_lds(render_fn<false, false>(p.scene), lds);
    if (e == hipSuccess) e = allow_lds(render_fn<false, true>(p.scene), lds);
    if (e == hipSuccess) e = allow_lds(render_fn<true, true>(p.scene), lds);
    if (e != hipSuccess) return e;
    if (!sched.cost || p.spp < kLptMinSpp) {
        launch_k<false, false>(p.scene, need_x, lds, stream, p);
        return hipGetLastError();
    }
    if (sched.nbuckets != kCostBuckets || sched.npix < lanes) return hipErrorInvalidValue;
    // 1. cost pre-pass: kCostSpp samples per pixel; records each pixel's
    // segments and its state (acc, seed) after them, which the render resumes
    KParams c = p;
    // large scenes: one sample — there a segment costs ~4 ms of wave time and
    // the pre-pass waits on its heaviest pixel's chain
    c.spp = min(p.spp, pf ? kCostSppLarge : kCostSpp);
    uint32_t split_cap = 0;
    {
        const uint32_t rb = resident_blocks(render_fn<true, false>(p.scene), lds);
        const bool whole = (double)lanes >= tune.rho2 * (double)min(need, rb) * kRB;  // a large part (the tiers' class)
        // a row-split share (small scenes) may cap too (cap_split): its stopped
        // pixels take the top bucket (tier 1), their neighbours count the cap
        split_cap = !whole && !pf ? min(tune.cap_split, 4096u) : 0u;
        c.cost_cap = whole ? (pf ? kCostCapLarge : kCostCap) : split_cap;
        c.cost_capped = (pf || split_cap != 0u) ? kCostSaturated : c.cost_cap;
    }
    c.chunk = 0;  // (private runs for the large-scene pre-pass: no faster)
    c.cost_out = sched.cost;
    c.state = sched.state;
    c.accum = nullptr;
    c.wave_times = nullptr;
    c.perm = nullptr;  // index order
    c.heavy = nullptr;
    c.prio_slots = 0;
    e = hipMemsetAsync(sched.buckets, 0, (2 * kCostBuckets + kSchedWords) * sizeof(uint32_t), stream);
    if (e == hipSuccess) e = hipMemsetAsync(p.queue, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    if (pf) {
        // large scenes: persistent lanes in index order (a lane whose pixel
        // ends takes the next one), so the pass does not wait on each wave's
        // slowest pixel — at 100k spheres an exact grid spent 27 % of the
        // C5 frame here; for small scenes the exact grid measured ~1 % faster
        const uint32_t pblocks = min(need, resident_blocks(render_fn<true, true>(p.scene), lds));
        // its tail: once at most pre_stop pixels are in flight they stop (pre_stop)
        if (kPreStopFrac > 0.0) {
            c.pre_done = sched.buckets + 2 * kCostBuckets + 6;  // heavy[6], zeroed above
            c.pre_stop = (uint32_t)(kPreStopFrac * (double)pblocks * kRB);
        }
        launch_k<true, true>(p.scene, pblocks, lds, stream, c);
    } else {
        launch_k<false, true>(p.scene, need_x, lds, stream, c);
    }
    // 2. counting sort by cost, descending
    // (in pixel tiles except for a small share: R = 8 12.7 vs 13.0 ms, S6r, S6v)
#ifndef RTX_QUEUE_TILE_ALL  // A/B: 1 = pixel tiles for every share size
#define RTX_QUEUE_TILE_ALL 0
#endif
#ifndef RTX_QUEUE_TILE_SPLIT  // A/B: a row-split part's tiles, this wide and one row tile (tile_rows) tall
#define RTX_QUEUE_TILE_SPLIT 0
#endif
    // a part's rows are runs of tile_rows image rows: its tiles are one run tall
    uint32_t qtile = RTX_QUEUE_TILE_ALL || (double)lanes >= tune.rho * (double)min(need, resident_blocks(render_fn<true, false>(p.scene), lds)) * kRB
                         ? kQueueTile
                         : 0u;
    uint32_t qtile_y = 0u;
    if (RTX_QUEUE_TILE_SPLIT != 0 && p.nparts > 1u && p.tile_rows != 0u) qtile = RTX_QUEUE_TILE_SPLIT, qtile_y = p.tile_rows;
    const uint32_t sblocks = ceil_div(tile_span(p.width, p.rows_local, qtile, qtile_y), kBlock * kSortPerThread);
    hipLaunchKernelGGL(k_cost_hist, dim3(sblocks), dim3(kBlock), 0, stream, sched.cost, p.width,
                       p.rows_local, c.spp, split_cap, qtile, qtile_y, sched.buckets);
    // 3. heavy-pixel split (from the histogram), the ordered queue, then
    // the persistent render over it
    uint32_t blocks = min(need, resident_blocks(render_fn<true, false>(p.scene), lds));
    {
        const double px_per_lane = (double)lanes / ((double)blocks * kRB);
        const double occ = px_per_lane < tune.rho ? tune.occ_small : px_per_lane < tune.rho_low ? tune.occ_low : tune.occ_normal;
        blocks = max(1u, (uint32_t)(blocks * occ + 0.5));
    }
    uint32_t *heavy = sched.buckets + 2 * kCostBuckets;
    hipLaunchKernelGGL(k_heavy_split, dim3(1), dim3(64), 0, stream, sched.buckets, (uint32_t)lanes, blocks * kRB, p.spp,
                       heavy, tune);
    hipLaunchKernelGGL(k_cost_scatter, dim3(sblocks), dim3(kBlock), 0, stream, sched.cost, p.width,
                       p.rows_local, c.spp, split_cap, qtile, qtile_y, sched.buckets, sched.buckets + kCostBuckets, sched.perm,
                       sched.stage ? sched.inv : nullptr);
    KParams q = p;
    q.cost_spp = c.spp;
    q.perm = sched.perm;
    q.out_slot = sched.stage;  // the image in queue-slot order, k_unpermute after the render
    q.stage_tag = sched.epoch;  // nonzero, new every launch: the staged pixels' w
    q.state = sched.state;
    q.prio_slots = (uint32_t)((double)blocks * kRB * tune.prio_frac);
    q.heavy = heavy;
    if (tune.dyn1 > 0.0) {  // dynamic lane-mode wave priority (rtx_schedule.prio_bar*)
        q.cost_in = sched.cost;
        q.dyn_bar[0] = (float)tune.dyn1;
        q.dyn_bar[1] = (float)tune.dyn2;
        q.dyn_bar[2] = (float)tune.dyn3;
    }
    // private queue runs per wave for a large part only (a whole frame: R = 2,
    // 4, 8 shares measured no better, profiles/R3x_parts.jsonl)
    // and small scenes only (at 100k spheres a pixel takes ~100 ms in lane
    // mode, and heavy pixels waited in busy waves' runs: C5 1.88 -> 2.05 s)
    // private runs of the queue (refill): refill_chunk slots for a small
    // scene's whole frame (C2 35.9 -> 33.0 ms at 64: S6t-S6u), at most
    // kChunkShare for a large scene (C5 128.7 -> 124.4 ms at 16; 64: 140) and
    // for a medium share (R = 2: 24.1 -> 22.4 ms at 16); none for smaller
    // shares (R = 4: 16.1 -> 16.9 ms with them)
    {
        const double ppl = (double)lanes / ((double)blocks * kRB);
        q.chunk = (!pf && ppl >= tune.rho2) ? min(tune.chunk, 4096u)
                  : ppl >= tune.rho_low     ? min(tune.chunk, kChunkShare)
                                            : 0u;
    }
    e = hipMemsetAsync(p.queue, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    // tier 1 in k_trace on the auxiliary stream (small scenes): its waves
    // are launched first and k_render leaves room for them (trace_waves / 4
    // fewer blocks), so whichever dispatches first, both are resident.
    uint32_t trace_waves = 0;
    if (sched.aux && !pf && p.scene.n <= kCoopLds) {
        const double px_per_lane = (double)lanes / ((double)blocks * kRB);
        const double frac = px_per_lane < tune.rho ? tune.trace_small : px_per_lane < tune.rho_low ? tune.trace_low
                            : px_per_lane < tune.rho2 ? tune.trace_medium : tune.trace_large;
        trace_waves = (uint32_t)(frac * blocks * (kRB / 64) + 0.5);
    }
    // promotion: served by idle k_render waves, and by k_trace after tier 1
    // when it runs. Large scenes have their own threshold (prom_big): there a
    // lane-mode segment is a 12.5k-block scan, so handing a far shorter
    // remaining chain to a whole wave pays (an earlier "1.86 -> 2.39 s" at
    // C5 was measured together with a 32-ray tail coop, R3u)
    {
        const double px_per_lane = (double)lanes / ((double)blocks * kRB);
        const double pm = p.scene.n > kCoopLds    ? tune.prom_big
                          : px_per_lane < tune.rho ? tune.prom_small : px_per_lane < tune.rho_low ? tune.prom_low
                          : px_per_lane < tune.rho2 ? tune.prom_medium : tune.prom_large;
        if (pm > 0.0 && sched.prom_q && sched.prom_cap > 0) {
            q.prom = sched.buckets + 2 * kCostBuckets + 8;  // zeroed with the buckets
            q.prom_q = sched.prom_q;
            q.prom_cap = sched.prom_cap;
            q.prom_min = (uint32_t)std::min<double>(pm, 4e9);
            q.epoch = sched.epoch;
        }
    }
    if (trace_waves > 0) {
        q.trace_ext = 1u;
        q.trace_lg = 6u - (uint32_t)__builtin_ctz(max(1u, min(tune.trace_group, 64u)));
        const size_t tlds = coop_lds_bytes(p.scene.n);
        e = hipEventRecord(sched.ev_fork, stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(sched.aux, sched.ev_fork, 0);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_trace, dim3((trace_waves + kTraceThreads / 64u - 1u) / (kTraceThreads / 64u)), dim3(kTraceThreads), tlds,
                           sched.aux, q);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipEventRecord(sched.ev_join, sched.aux);
        if (e != hipSuccess) return e;
        blocks = max(1u, blocks - (trace_waves + 3u) / 4u);
    }
    launch_k<true, false>(p.scene, blocks, lds, stream, q);
    e = hipGetLastError();
    if (e == hipSuccess && trace_waves > 0) e = hipStreamWaitEvent(stream, sched.ev_join, 0);
    if (e == hipSuccess && sched.stage) {
        hipLaunchKernelGGL(k_unpermute, dim3(ceil_div(lanes, kBlock)), dim3(kBlock), 0, stream, sched.stage, sched.inv,
                           (uint32_t)lanes, q.stage_tag, p.out);
        e = hipGetLastError();
    }
    return e;
}

hipError_t launch_deinterleave(const float4 *gathered, float4 *image, uint32_t width,
                               uint32_t height, uint32_t tile_rows, uint32_t nparts,
                               uint32_t max_rows, hipStream_t stream) {
    const uint64_t n = (uint64_t)width * height;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_deinterleave, dim3(ceil_div(n, kBlock)), dim3(kBlock), 0, stream, gathered,
                       image, width, height, tile_rows, nparts, max_rows);
    return hipGetLastError();
}

hipError_t launch_debug_hit_world(const KScene &s, const float *rays, uint32_t nrays, float t_min,
                                  float t_max, uint32_t start_block, float *out, hipStream_t stream) {
    if (nrays == 0) return hipSuccess;
    const uint32_t q = start_block & 0xffu;
    const uint32_t sel = start_block & ~0xffu;
    if ((sel == kDebugCulledCoop || sel == kDebugCulledCoopLane) && q >= 1u && q <= 64u && s.cpre) {
        const uint32_t waves = ceil_div(nrays, q);
        if (sel == kDebugCulledCoop)
            hipLaunchKernelGGL(k_debug_hit_world_coop<true>, dim3(ceil_div(waves, kRB / 64u)), dim3(kRB), 0, stream, s,
                               rays, nrays, t_min, t_max, q, out);
        else
            hipLaunchKernelGGL(k_debug_hit_world_coop<false>, dim3(ceil_div(waves, kRB / 64u)), dim3(kRB), 0, stream,
                               s, rays, nrays, t_min, t_max, q, out);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_debug_hit_world, dim3(ceil_div(nrays, kRB)), dim3(kRB), 0, stream, s,
                       rays, nrays, t_min, t_max, start_block, out);
    return hipGetLastError();
}

bool debug_scan_rate_supported(const KParams &p) {
    return p.scene.n <= kCoopLds && !use_pf(p.scene) && (uint64_t)p.rows_local * p.width != 0;
}

hipError_t launch_debug_scan_rate(const KParams &p, uint32_t reps, unsigned long long *sink, uint32_t *waves,
                                  hipStream_t stream) {
    if (!debug_scan_rate_supported(p)) return hipErrorInvalidValue;
    const size_t lds = kListBytes + kCoopBytes + (size_t)coop_lds_bytes(p.scene.n);
    const uint32_t blocks = resident_blocks((const void *)k_debug_scan_rate, lds);
    *waves = blocks * (kRB / 64);
    hipLaunchKernelGGL(k_debug_scan_rate, dim3(blocks), dim3(kRB), lds, stream, p, reps, sink);
    return hipGetLastError();
}

hipError_t launch_debug_math(int fn, const float *in0, const float *in1, uint32_t n, float *out,
                             hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_debug_math, dim3(ceil_div(n, kBlock)), dim3(kBlock), 0, stream, fn, in0, in1,
                       n, out);
    return hipGetLastError();
}

}  // namespace rtx
