// rtx_internal.h — kernel parameter block and launch entry points shared by
// rtx_kernels.hip (device code) and rtx_api.hip (C-ABI context glue).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rtx_grid.h"

namespace rtx {

// Device scene layout (all in HBM, read-only):
//   soa   float[n_pad*4]  AoSoA-8 blocks of 8 spheres, 128 B each:
//                         cx[8] cy[8] cz[8] -(r*r)[8] — the exact in-order
//                         fallback scan (scalar loads)
//   cen   float4[n]  center.xyz, radius  — read once per hit (normal)
//   mtype int   [n]  material code 0/1/2, 3 = "no scatter"
//   mval  float4[n]  albedo.rgb, fuzz-or-ir
// `soa` is padded to n_pad = roundup(n, kPad) spheres with copies of sphere
// n-1; a padded copy can only win where sphere n-1 itself would (same data,
// later index wins ties), so kernels clamp the winning index to n-1.
//   pre   float[n_pad*4]  AoSoA-8 like soa: cx[8] cy[8] cz[8] R[8], R the
//                         prefilter's inflated r^2 (rtx_prefilter.h) — the
//                         array every ray segment scans
// `smag` bounds |c| + r over the scene (rounded up), for the prefilter's
// per-ray overflow guard. Blocks [flat_lo, flat_hi) of `pre` hold spheres
// whose centres all have height flat_cy (the scan's 5-op test,
// rtx_prefilter.h line_test_q_flat).
struct KScene {
    const float *soa;
    const float *pre;
    const float4 *pre4;  // [n] (cx, cy, cz, R): the prefilter data per sphere (tail coop)
    const float4 *cen;
    const int *mtype;
    const float4 *mval;
    uint32_t n, n_pad;
    float smag;
    float flat_cy;             // centre height shared by every sphere of blocks [flat_lo, flat_hi)
    uint32_t flat_lo, flat_hi;  // the scene's longest run of such flat blocks (empty: 0, 0)
    // culled layout (the lane-mode scan of scenes with n_pad > kScanPfMin;
    // NULL otherwise): the spheres in a spatial order, blocked like pre, with
    // each block's bounding sphere (rtx_prefilter.h cull_bound)
    //   cpre  float[n_cpad*4]  AoSoA-8 like pre (cx cy cz R), position order
    //   cbnd  float[ceil(n_cpad/64)*32]  AoSoA-8 groups of 8 block bounds (cx cy cz R_b)
    //   cbnd2 float[ceil(n_cpad/512)*32] AoSoA-8: per super-group (64 blocks) its 8 group
    //                          bounds (each over the 64 spheres of a group of 8 blocks)
    //   cbnd3 float[ceil(n_cpad/4096)*32] AoSoA-8: per 512 blocks the 8 super-group bounds
    //                          (each over a super-group's 512 spheres)
    // A bound is flat — stored in the space stretched along y (rtx_prefilter.h
    // kCullSy) — iff its first block is >= cflat_lo.
    //   ccen  float4[n_cpad]   cen in position order (the resolve's sphere data)
    //   cperm uint32[n_cpad]   position -> scene index (a pad: a copy with R = -inf)
    // Blocks [cflat_lo, n_cpad/8) hold only spheres at height flat_cy.
    const float *cpre;
    const float *cbnd;
    const float *cbnd2;
    const float *cbnd3;
    const float4 *ccen;
    const uint32_t *cperm;
    uint32_t n_cpad, cflat_lo;
    // layer grid of the flat run (small scenes; rtx_grid.h): its LayerGrid,
    // then per cell the mask of the run's blocks it may need (NULL: none,
    // every block is scanned)
    const LayerGrid *grid;
};

#ifndef RTX_CULL  // A/B build: 0 = no culled layout (the large-scene lane-mode scan visits every block)
#define RTX_CULL 1
#endif
#ifndef RTX_GRID  // A/B build: 0 = no layer grid (every block of the flat layer is scanned, or culled)
#define RTX_GRID 1
#endif
#ifndef RTX_CULL_LEVELS  // bound levels above the blocks: 2 (groups, super-groups) or 3 (+ 512-block ranges)
#define RTX_CULL_LEVELS 3
#endif
// the flat section of the culled layout starts at a multiple of this many
// blocks: no bound test (8 entries) mixes flat and non-flat bounds
constexpr uint32_t kCullAlign = RTX_CULL_LEVELS >= 3 ? 512u : 64u;
#ifndef RTX_CULL_HALF  // culled scan: a bound wholly behind the origin fails too (rtx_prefilter.h HalfTest)
#define RTX_CULL_HALF 1
#endif
#ifndef RTX_CULL_HALF_SPHERES  // 1: also drop a flagged sphere wholly behind it (measured slower: R9s)
#define RTX_CULL_HALF_SPHERES 0
#endif
#ifndef RTX_CULL_BFS  // the one-ray culled coop walks the levels breadth first (0: each lane its subtree)
#define RTX_CULL_BFS 1
#endif
#ifndef RTX_SCAN_PF_MIN  // (A/B builds: 0 sends every scene to the kPF kernels)
#define RTX_SCAN_PF_MIN 1024
#endif
constexpr uint32_t kScanPfMin = RTX_SCAN_PF_MIN;  // scenes with n_pad above this take the kPF kernels (> 32 KiB of `pre`)

constexpr uint32_t kPad = 8;  // spheres per AoSoA block

constexpr uint32_t kFrameLambertGuard = 1u;  // = RTX_FRAME_LAMBERT_GUARD

// KParams::errors bits: a launch that sets one left pixels unwritten.
constexpr uint32_t kErrPromTimeout = 1u;    // a promotion server saw no progress for kPromValveTicks and left
constexpr uint32_t kErrPromTorn = 2u;       // a promotion entry held an out-of-range pixel or sample
constexpr uint32_t kErrPromEntryWait = 4u;  // a claimed promotion entry was not published within kPromValveTicks
constexpr uint32_t kErrKernarg = 8u;        // check build: a kernel's kernarg segment did not begin with its KParams

// The promotion valve (rtx_kernels.hip take_promoted): a server that has
// been polling for this long with no pixel written and no heartbeat leaves
// and flags the launch. s_memrealtime ticks (100 MHz). The stress build
// (Makefile) sets its own.
#ifndef RTX_PROM_VALVE_TICKS
#define RTX_PROM_VALVE_TICKS 1000000000ull  // 10 s
#endif
constexpr unsigned long long kPromValveTicks = RTX_PROM_VALVE_TICKS;
// KParams::err_diag: what the first server whose valve fired saw, one u64
// (rtx_api.hip check_errors prints it with the launch's queue counters):
//   bits 0-3 the error bit, 4-7 who (1 k_render server, 2 k_trace helper),
//   8-15 the server's own stalls (polls more than a beat period apart),
//   16-31 time since it last saw progress, 32-63 the heartbeat's age, both in
//   s_memrealtime >> 10 units (10.24 us)
constexpr uint32_t kErrDiagWords = 1;

// Per-launch constants (~ cbuffer b0 PerFrame + sceneValues of b1).
struct KParams {
    KScene scene;
    float4 *out;                   // part's rows, contiguous, row-major
    float4 *out_slot;              // cost-ordered render: the image by queue slot (k_unpermute), or NULL
    uint32_t stage_tag;            // ... the launch's tag in a staged pixel's w (k_unpermute moves only those)
    unsigned long long *counters;  // [0] += ray segments (hit_world calls)
    uint32_t *queue;               // pixel queue head (zeroed before each launch)
    uint32_t depth, spp;
    uint32_t width, rows_local;    // launch covers rows_local * width lanes
    uint32_t tile_rows, part, nparts;
    uint32_t rng_mode, frame_index;
    uint32_t flags;                // kFrame* bits (rtx_frame.flags)
    float org[3], hor[3], ver[3], llc[3];
    float img_w, img_h;
    float lens_u[3], lens_v[3], lens_r;  // thin lens (lens_r 0 = pinhole)
    float4 *accum;                 // progressive accumulation (NULL = plain frame)
    uint32_t accum_frames;         // frames in accum after this launch
    unsigned long long *wave_times;  // diagnostic: per-wave (start, end) s_memrealtime, or NULL
    uint32_t wave_cap;             // pairs in wave_times
    const uint32_t *perm;          // pixel queue order: slot -> local pixel (NULL = identity)
    uint32_t *cost_out;            // cost pre-pass: per-pixel segment count instead of colour
    uint32_t cost_spp;             // samples the pre-pass traced (the render resumes after them)
    uint32_t cost_cap;             // pre-pass: a pixel still tracing after this many segments stops (0: none)
    uint32_t cost_capped;          // ... and records this cost
    uint32_t *pre_done;            // persistent pre-pass: pixels finished (NULL: no early stop)
    uint32_t pre_stop;             // ... it stops its pixels once at most this many are in flight
    float4 *state;                 // per pixel (acc, seed) after cost_spp samples: written by the
                                   // pre-pass, resumed from by the persistent render (NULL = none)
    uint32_t prio_slots;           // normal-queue slots whose waves run at top priority
    uint32_t coop_max;             // queue exhausted: a wave with <= this many pixels traces them in group coop
    uint32_t prio_t1, prio_t2, prio_hot;  // wave priorities (0..3) of tier-1, tier-2 and hot lane-mode waves
    uint32_t trace_ext;            // tier 1 runs in k_trace beside k_render (k_render skips it)
    uint32_t chunk;                // refill: a wave's private run of this many queue slots (0 = one refill per need)
    // promotion (k_trace beside k_render): once its queue is empty, a lane-mode
    // wave hands a pixel whose projected remaining segments exceed prom_min
    // to k_trace at a sample boundary (rtx_kernels.hip, promote)
    uint32_t *prom;                // [0] entries claimed [1] entries taken [2] k_render-owned pixels written
                                   // [3] k_render has started (set by its workgroup 0)
                                   // [4] heartbeat: s_memrealtime >> 10 of a tracing wave (valve); NULL: off
    uint32_t *errors;              // launch error bits (kErr*), read back by rtx_sync / rtx_get_stats
    unsigned long long *err_diag;  // the first valve firing's record (kErrDiagWords; NULL: none)
    uint32_t *prom_q;              // [prom_cap][8] (gid, sample, seed, acc.xyz, -, epoch)
    uint32_t prom_cap, prom_min, epoch;
    uint32_t *heavy;               // [0] tier-1 counter [1] kh [2] tier-2 counter [3] k1 [4] k0
                                   // [5] mean segments per pixel at the full spp (float bits) (NULL = none)
    const uint32_t *cost_in;       // render: the pre-pass's per-pixel segments (dynamic wave priority; NULL = off)
    float dyn_bar[3];              // ... its bars (x heavy[5])
    uint32_t trace_lg;             // k_trace: log2(lanes per pixel) of its waves past the solo slots [0, k0)
    // per-sample RNG kernel (k_render_ps): per-wave sample-colour scratch
    // [wave][kPsSlots][ps_cap] float4, batches of at most ps_px pixels
    float *ps_scratch;
    uint32_t ps_px, ps_cap;
};

// Longest-processing-time-first scheduling for the persistent kernel: a
// pre-pass traces kCostSpp samples per pixel and records their segment
// count; a counting sort orders the pixel queue by that cost, descending,
// so the pixels that take longest start first and the frame does not end
// on a few expensive pixels started late.
// The chain render's schedule (include/rtx.h rtx_schedule; validated by
// rtx_set_schedule): heavy-pixel tier bars, share classes, hot-wave
// fraction, launch occupancy, tail-coop size. Doubles: k_heavy_split
// compares them with sums of cost keys.
struct KTune {
    double a1, a1_small, a1_low, a2_small, a2_medium, a2_large, rho, rho_low, rho2, prio_frac;
    double occ_small, occ_low, occ_normal;  // fraction of the resident waves launched for a small / low / larger share
    uint32_t coop_max;                      // KParams::coop_max (scenes with the coop's LDS copy)
    uint32_t coop_max_large;                // ... and without it (n > kCoopLds)
    uint32_t prio_t1, prio_t2, prio_hot;    // KParams::prio_*
    uint32_t chunk;                         // KParams::chunk for a part of at least rho2 pixels per lane
    double trace_small, trace_low, trace_medium, trace_large;  // k_trace waves / resident waves, by share class
    double prom_small, prom_low, prom_medium, prom_large;      // promotion threshold (projected segments; 0: off)
    double prom_big;                                           // ... for scenes without the coop's LDS copy
    uint32_t trace_group;                                      // k_trace: pixels per wave (1, 2, 4 or 8)
    double trace_solo;                                         // ... one per wave above this x share (k0)
    uint32_t cap_split;                                        // pre-pass cap of a row-split part (0: none)
    double dyn1, dyn2, dyn3;  // lane-mode wave priority 1/2/3 above these x the mean pixel (dyn1 0: static hot slots)
};
KTune default_tune();

struct KSchedule {
    uint32_t *cost;     // [npix]
    uint32_t *perm;     // [npix]
    float4 *state;      // [npix] (acc.xyz, seed) after the pre-pass's samples
    float4 *stage;      // [npix] the render's image by queue slot (NULL: written in place)
    uint32_t *inv;      // [npix] pixel -> queue slot (k_cost_scatter; k_unpermute)
    uint32_t *buckets;  // [2 * nbuckets + kSchedWords]: counts, cursors, heavy[8], prom[8] (zeroed per launch)
    uint32_t npix;      // capacity of cost / perm
    uint32_t nbuckets;  // must equal kCostBuckets of the kernel object
    float *ps_scratch;  // k_render_ps scratch (rng_mode 1), ps_floats floats
    size_t ps_floats;
    KTune tune;
    hipStream_t aux;    // k_trace's stream (NULL: tier 1 stays in k_render)
    hipEvent_t ev_fork, ev_join;
    uint32_t *prom_q;   // promotion queue storage, prom_cap entries of 8 words
    uint32_t prom_cap;
    uint32_t epoch;     // launch counter: a promotion entry is ready when its last word equals it
};
constexpr uint32_t kCostBuckets = 256;
// Scheduling words after the two bucket arrays (counts, cursors), zeroed per
// launch: heavy[8] (KParams::heavy; heavy[6]: the pre-pass's pre_done), then
// prom[8] (KParams::prom).
constexpr uint32_t kSchedWords = 16;
#ifndef RTX_COST_SPP
#define RTX_COST_SPP 2
#endif
constexpr uint32_t kCostSpp = RTX_COST_SPP;  // pre-pass samples per pixel (kept: the render resumes after them)
#ifndef RTX_COST_SPP_LARGE
#define RTX_COST_SPP_LARGE 1
#endif
constexpr uint32_t kCostSppLarge = RTX_COST_SPP_LARGE;  // ... for scenes above kScanPfMin spheres (C5: 1,997 vs 2,018 ms)
constexpr uint32_t kLptMinSpp = 8;  // below this the pre-pass costs more than it saves: exact grid
constexpr uint32_t kBlock = 256;    // threads per block of the auxiliary kernels (4 waves)

hipError_t launch_render(const KParams &p, const KSchedule &sched, hipStream_t stream);
// Floats of k_render_ps scratch a launch with these parameters needs (0 when
// it takes another kernel).
size_t ps_scratch_floats(const KParams &p);
hipError_t launch_cost(const KParams &p, hipStream_t stream);  // exact grid, p.cost_out set
hipError_t launch_deinterleave(const float4 *gathered, float4 *image, uint32_t width,
                               uint32_t height, uint32_t tile_rows, uint32_t nparts,
                               uint32_t max_rows, hipStream_t stream);
hipError_t launch_debug_hit_world(const KScene &s, const float *rays, uint32_t nrays,
                                  float t_min, float t_max, uint32_t start_block, float *out,
                                  hipStream_t stream);
// hit_world alone at the render's occupancy (rtx_debug_scan_rate); *waves: the grid's waves.
// Scenes that fit the coop's LDS copy (the C2 kernels), non-empty frames only:
bool debug_scan_rate_supported(const KParams &p);
hipError_t launch_debug_scan_rate(const KParams &p, uint32_t reps, unsigned long long *sink, uint32_t *waves,
                                  hipStream_t stream);
hipError_t launch_debug_math(int fn, const float *in0, const float *in1, uint32_t n,
                             float *out, hipStream_t stream);

}  // namespace rtx
