// rtx_api.hip — C-ABI context management for librtx.so (include/rtx.h).
//
// Replaces the D3D11 objects the reference's DxCSApp owns
// (CSVersion/DxCSApp.h:33-59): the IMMUTABLE WorldDef cbuffer becomes
// device arrays (rtx_upload_world), the DYNAMIC PerFrame cbuffer becomes
// kernel arguments (rtx_set_frame), the RWTexture2D UAV becomes a linear
// float4 framebuffer, Dispatch becomes rtx_render_rows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/rtx.h"
#include "rtx_internal.h"
#include "rtx_prefilter.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

int hip_fail(hipError_t e, const char *what) {
    return fail(RTX_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define RTX_HIP(call)                                   \
    do {                                                \
        hipError_t e_ = (call);                         \
        if (e_ != hipSuccess) return hip_fail(e_, #call); \
    } while (0)

struct EventPair {
    hipEvent_t start = nullptr, stop = nullptr;
};

// Launch timing: a ring of event pairs. When every pair is in use, the
// oldest launch's duration is folded into a running total if its stop event
// has completed (hipEventQuery, no wait); otherwise the ring doubles. A host
// that renders forever without rtx_stats_reset keeps as many pairs as it
// has launches in flight, and a launch never blocks on an older one.
constexpr size_t kEventRing = 64;  // initial ring size

// Device counter words (unsigned long long): [0] ray segments, [2] pixel-queue
// head (low half), [3] rtx_debug_pixel_cost's segments, [4] launch error bits
// (rtx::kErr*, low half; read back and cleared by check_errors), [1], [5] spare,
// [6, 6 + kErrDiagWords) the first promotion-valve firing's record
// (KParams::err_diag, rtx_internal.h).
constexpr size_t kErrWord = 4;
constexpr size_t kErrDiag = 6;
constexpr size_t kCounterWords = kErrDiag + rtx::kErrDiagWords;

}  // namespace

#ifndef RTX_FLAT
#define RTX_FLAT 1
#endif
#ifndef RTX_GRID_UPLOAD  // A/B build: 0 = no layer grid (every block of the flat run is scanned)
#define RTX_GRID_UPLOAD 1
#endif

struct rtx_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;  // own_stream or an external one
    // scene (device)
    float *d_soa = nullptr;
    float *d_pre = nullptr;  // prefilter blocks (rtx_prefilter.h)
    float4 *d_pre4 = nullptr;  // prefilter data per sphere (tail coop)
    float smag = 0.0f;
    float flat_cy = 0.0f;  // scene's flat run of `pre` blocks (rtx_internal.h KScene)
    uint32_t flat_lo = 0, flat_hi = 0;
    // culled layout (rtx_internal.h KScene; none: null)
    float *d_cpre = nullptr;
    float *d_cbnd = nullptr;
    float *d_cbnd2 = nullptr;
    float *d_cbnd3 = nullptr;
    uint32_t *d_cperm = nullptr;
    float4 *d_ccen = nullptr;
    uint32_t n_cpad = 0, cflat_lo = 0;
    // layer grid of the flat run (small scenes; rtx_grid.h; none: null):
    // its LayerGrid, then the cells' block masks
    rtx::LayerGrid *d_grid = nullptr;
    int scan_mode = RTX_SCAN_AUTO;  // rtx_set_scan_mode: applied by rtx_upload_world
    float4 *d_cen = nullptr;
    int *d_mtype = nullptr;
    float4 *d_mval = nullptr;
    uint32_t n = 0, n_pad = 0, depth = 0, spp = 0;
    bool have_world = false;
    // frame
    rtx_frame frame{};
    bool have_frame = false;
    // framebuffer
    float4 *d_fb = nullptr;
    size_t fb_pixels = 0;
    // progressive accumulation (linear sums) of accum_pixels pixels
    float4 *d_accum = nullptr;
    size_t accum_pixels = 0;
    uint32_t accum_frames = 0;
    // measurement
    unsigned long long *d_counters = nullptr;
    unsigned long long *d_wave_times = nullptr;  // diagnostic (rtx_debug_wave_times)
    size_t wave_times_cap = 0;
    // LPT scheduling scratch (persistent kernel): cost + perm per pixel
    uint32_t *d_sched = nullptr;
    size_t sched_pixels = 0;
    // per-sample RNG kernel's per-wave sample-colour scratch
    float *d_ps = nullptr;
    size_t ps_floats = 0;
    std::vector<EventPair> events = std::vector<EventPair>(kEventRing);  // ring: [ev_head, ev_head + ev_count)
    size_t ev_head = 0, ev_count = 0;
    rtx::KTune tune = rtx::default_tune();  // rtx_set_schedule
    hipStream_t aux_stream = nullptr;       // k_trace (tier 1 beside the render), created on first use
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    uint64_t epoch = 0;                     // render launches: promotion-queue entry epochs
    double ms_folded = 0.0;         // durations of launches whose pair was recycled
    uint64_t samples = 0;
    uint64_t launches = 0;
    bool n_changed = false;  // world resized since the last rtx_stats_reset
};

namespace {

int set_device(rtx_ctx *c) {
    RTX_HIP(hipSetDevice(c->device));
    return RTX_OK;
}

// After a stream synchronisation: the error bits the launches since the last
// check set (KParams::errors), reported once and cleared. A set bit means a
// launch left pixels unwritten (rtx_kernels.hip take_promoted).
int check_errors(rtx_ctx *c, const char *what) {
    unsigned long long w[kCounterWords - kErrWord];  // the error word, [5], the valve record
    RTX_HIP(hipMemcpyAsync(w, c->d_counters + kErrWord, sizeof(w), hipMemcpyDeviceToHost, c->stream));
    RTX_HIP(hipStreamSynchronize(c->stream));
    const unsigned long long bits = w[0];
    if (bits == 0) return RTX_OK;
    RTX_HIP(hipMemsetAsync(c->d_counters + kErrWord, 0, sizeof(w), c->stream));
    RTX_HIP(hipStreamSynchronize(c->stream));
    const double valve_ms = (double)rtx::kPromValveTicks * 1e-5;  // s_memrealtime: 100 MHz
    char buf[160];
    std::string why;
    if (bits & rtx::kErrPromTimeout) {
        std::snprintf(buf, sizeof buf, " a promotion server polled for %.0f ms seeing no pixel written and no "
                      "heartbeat, and left;", valve_ms);
        why += buf;
    }
    if (bits & rtx::kErrPromEntryWait) {
        std::snprintf(buf, sizeof buf, " a claimed promotion entry was not published within %.0f ms;", valve_ms);
        why += buf;
    }
    if (bits & rtx::kErrPromTorn) why += " a promotion entry was out of range;";
    if (bits & rtx::kErrKernarg) why += " a kernel's argument segment did not begin with its KParams (check build);";
    const unsigned long long d = w[kErrDiag - kErrWord];
    if (d != 0) {
        const unsigned lo = (unsigned)d, age = (unsigned)(d >> 32);
        std::snprintf(buf, sizeof buf, " first firing: bit %u by a %s server, %.2f ms since it saw progress, the "
                      "heartbeat %.2f ms old, %u stalls of the server itself;", lo & 0xfu,
                      ((lo >> 4) & 0xfu) == 2u ? "k_trace" : "k_render", (double)(lo >> 16) * 1.024e-2,
                      (double)age * 1.024e-2, (lo >> 8) & 0xffu);
        why += buf;
        // the last launch's queue counters (zeroed at its start, still in memory)
        uint32_t q[5] = {0, 0, 0, 0, 0};
        if (c->d_sched && c->sched_pixels &&
            hipMemcpy(q, c->d_sched + 2 * c->sched_pixels + 2 * rtx::kCostBuckets + 8, sizeof q,
                      hipMemcpyDeviceToHost) == hipSuccess) {
            std::snprintf(buf, sizeof buf, " last launch's queue: claimed %u, taken %u, k_render pixels written %u, "
                          "k_render started %u", q[0], q[1], q[2], q[3]);
            why += buf;
        }
    }
    return fail(RTX_ERR_INCOMPLETE, std::string(what) + ": a render launch left pixels unwritten:" + why);
}

void free_world(rtx_ctx *c) {
    (void)hipFree(c->d_soa);
    (void)hipFree(c->d_pre);
    (void)hipFree(c->d_pre4);
    (void)hipFree(c->d_cen);
    (void)hipFree(c->d_mtype);
    (void)hipFree(c->d_mval);
    (void)hipFree(c->d_cpre);
    (void)hipFree(c->d_cbnd);
    (void)hipFree(c->d_cbnd2);
    (void)hipFree(c->d_cbnd3);
    (void)hipFree(c->d_cperm);
    (void)hipFree(c->d_ccen);
    (void)hipFree(c->d_grid);
    c->d_grid = nullptr;
    c->d_cpre = c->d_cbnd = c->d_cbnd2 = c->d_cbnd3 = nullptr;
    c->d_cperm = nullptr;
    c->d_ccen = nullptr;
    c->n_cpad = c->cflat_lo = 0;
    c->d_soa = nullptr;
    c->d_pre = nullptr;
    c->d_pre4 = nullptr;
    c->d_cen = nullptr;
    c->d_mtype = nullptr;
    c->d_mval = nullptr;
    c->have_world = false;
}

rtx::KScene scene_of(const rtx_ctx *c) {
    rtx::KScene s;
    s.soa = c->d_soa;
    s.pre = c->d_pre;
    s.pre4 = c->d_pre4;
    s.smag = c->smag;
    s.flat_cy = c->flat_cy;
    s.flat_lo = c->flat_lo;
    s.flat_hi = c->flat_hi;
    s.cen = c->d_cen;
    s.mtype = c->d_mtype;
    s.mval = c->d_mval;
    s.n = c->n;
    s.n_pad = c->n_pad;
    s.cpre = c->d_cpre;
    s.cbnd = c->d_cbnd;
    s.cbnd2 = c->d_cbnd2;
    s.cbnd3 = c->d_cbnd3;
    s.cperm = c->d_cperm;
    s.ccen = c->d_ccen;
    s.n_cpad = c->n_cpad;
    s.cflat_lo = c->cflat_lo;
    s.grid = c->d_grid;
    return s;
}

}  // namespace

extern "C" {

int rtx_version(void) { return RTX_VERSION; }

#ifndef RTX_SRC_SHA
#define RTX_SRC_SHA "unknown"
#endif
// Build provenance: the hash of the sources this library was compiled from
// (Makefile SRC_SHA: sha256 over csrc/* and include/rtx.h, first 16 hex
// digits) and the offload target, so a run can show that the library it
// loaded is the one its tree's sources build.
// A variant build (Makefile variants/adhoc, tools/build_commit_variant.sh:
// other compile-time choices from the same sources) also names itself, so
// it is never mistaken for the product library.
#ifndef RTX_VARIANT
#define RTX_VARIANT "product"
#endif
const char *rtx_build_info(void) { return "src_sha16=" RTX_SRC_SHA " arch=gfx950 variant=" RTX_VARIANT; }

const char *rtx_last_error(void) { return g_last_error.c_str(); }

int rtx_device_count(int *count) {
    if (!count) return fail(RTX_ERR_INVALID, "rtx_device_count: null count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        return hip_fail(e, "hipGetDeviceCount");
    }
    *count = n;
    return RTX_OK;
}

int rtx_create(int hip_device, rtx_ctx **out) {
    if (!out) return fail(RTX_ERR_INVALID, "rtx_create: null out");
    *out = nullptr;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
    if (hip_device < 0 || hip_device >= ndev)
        return fail(RTX_ERR_INVALID, "rtx_create: device " + std::to_string(hip_device) +
                                         " out of range (" + std::to_string(ndev) + " devices)");
    rtx_ctx *c = new (std::nothrow) rtx_ctx();
    if (!c) return fail(RTX_ERR_NOMEM, "rtx_create: out of host memory");
    c->device = hip_device;
    int rc = set_device(c);
    if (rc != RTX_OK) {
        delete c;
        return rc;
    }
    e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return hip_fail(e, "hipStreamCreate");
    }
    c->stream = c->own_stream;
    e = hipMalloc(&c->d_counters, kCounterWords * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemsetAsync(c->d_counters, 0, kCounterWords * sizeof(unsigned long long), c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
        (void)hipStreamDestroy(c->own_stream);
        delete c;
        return hip_fail(e, "hipMalloc(counters)");
    }
    *out = c;
    return RTX_OK;
}

void rtx_destroy(rtx_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    free_world(c);
    (void)hipFree(c->d_fb);
    (void)hipFree(c->d_accum);
    (void)hipFree(c->d_counters);
    (void)hipFree(c->d_wave_times);
    (void)hipFree(c->d_sched);
    (void)hipFree(c->d_ps);
    for (auto &p : c->events) {
        if (p.start) (void)hipEventDestroy(p.start);
        if (p.stop) (void)hipEventDestroy(p.stop);
    }
    if (c->aux_stream) (void)hipStreamDestroy(c->aux_stream);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    (void)hipStreamDestroy(c->own_stream);
    delete c;
}

int rtx_set_stream(rtx_ctx *c, void *s) {
    if (!c) return fail(RTX_ERR_INVALID, "rtx_set_stream: null ctx");
    c->stream = reinterpret_cast<hipStream_t>(s);  // NULL: HIP's null stream (torch's default stream)
    return RTX_OK;
}

int rtx_use_own_stream(rtx_ctx *c) {
    if (!c) return fail(RTX_ERR_INVALID, "rtx_use_own_stream: null ctx");
    c->stream = c->own_stream;
    return RTX_OK;
}

int rtx_schedule_defaults(rtx_schedule *out) {
    if (!out) return fail(RTX_ERR_INVALID, "rtx_schedule_defaults: null out");
    const rtx::KTune t = rtx::default_tune();
    *out = rtx_schedule{};
    out->tier1_bar = (float)t.a1;
    out->tier1_bar_small = (float)t.a1_small;
    out->tier1_bar_low = (float)t.a1_low;
    out->tier2_bar_small = (float)t.a2_small;
    out->tier2_bar_medium = (float)t.a2_medium;
    out->tier2_bar = (float)std::min(t.a2_large, 1e30);
    out->small_share = (float)t.rho;
    out->low_share = (float)t.rho_low;
    out->medium_share = (float)t.rho2;
    out->hot_fraction = (float)t.prio_frac;
    out->occupancy_small = (float)t.occ_small;
    out->occupancy_low = (float)t.occ_low;
    out->occupancy_normal = (float)t.occ_normal;
    out->tail_coop_max = t.coop_max;
    out->tail_coop_max_large = t.coop_max_large;
    out->trace_small = (float)t.trace_small;
    out->trace_low = (float)t.trace_low;
    out->trace_medium = (float)t.trace_medium;
    out->trace_large = (float)t.trace_large;
    out->promote_small = (float)t.prom_small;
    out->promote_low = (float)t.prom_low;
    out->promote_medium = (float)t.prom_medium;
    out->promote_large = (float)t.prom_large;
    out->promote_big_scene = (float)t.prom_big;
    out->tier1_priority = t.prio_t1;
    out->tier2_priority = t.prio_t2;
    out->hot_priority = t.prio_hot;
    out->refill_chunk = t.chunk;
    out->trace_group = t.trace_group;
    out->trace_solo_bar = (float)std::min(t.trace_solo, 1e30);
    out->prepass_cap_split = t.cap_split;
    out->prio_bar1 = (float)t.dyn1;
    out->prio_bar2 = (float)t.dyn2;
    out->prio_bar3 = (float)t.dyn3;
    return RTX_OK;
}

int rtx_set_schedule(rtx_ctx *c, const rtx_schedule *s) {
    if (!c) return fail(RTX_ERR_INVALID, "rtx_set_schedule: null ctx");
    if (!s) {
        c->tune = rtx::default_tune();
        return RTX_OK;
    }
    const struct { const char *name; float v; } pos[] = {
        {"tier1_bar", s->tier1_bar},         {"tier1_bar_small", s->tier1_bar_small},
        {"tier1_bar_low", s->tier1_bar_low}, {"tier2_bar_small", s->tier2_bar_small},
        {"tier2_bar_medium", s->tier2_bar_medium}, {"tier2_bar", s->tier2_bar}, {"small_share", s->small_share},
        {"low_share", s->low_share},         {"medium_share", s->medium_share},
        {"trace_solo_bar", s->trace_solo_bar}};
    for (const auto &f : pos)
        if (!(f.v > 0.0f && f.v <= 1e30f))
            return fail(RTX_ERR_INVALID, std::string("rtx_set_schedule: ") + f.name + " must be finite and > 0");
    if (!(s->hot_fraction >= 0.0f && s->hot_fraction <= 1.0f))
        return fail(RTX_ERR_INVALID, "rtx_set_schedule: hot_fraction must be in [0, 1]");
    const float occ[] = {s->occupancy_small, s->occupancy_low, s->occupancy_normal};
    for (float o : occ)
        if (!(o > 0.0f && o <= 1.0f)) return fail(RTX_ERR_INVALID, "rtx_set_schedule: occupancies must be in (0, 1]");
    if (s->tail_coop_max < 1 || s->tail_coop_max > 64)
        return fail(RTX_ERR_INVALID, "rtx_set_schedule: tail_coop_max must be in 1..64");
    if (s->tail_coop_max_large < 1 || s->tail_coop_max_large > 64)
        return fail(RTX_ERR_INVALID, "rtx_set_schedule: tail_coop_max_large must be in 1..64");
    const float pr[] = {s->promote_small, s->promote_low, s->promote_medium, s->promote_large, s->promote_big_scene};
    for (float v : pr)
        if (!(v >= 0.0f && v <= 1e9f)) return fail(RTX_ERR_INVALID, "rtx_set_schedule: promote_* must be in [0, 1e9]");
    const float tr[] = {s->trace_small, s->trace_low, s->trace_medium, s->trace_large};
    for (float v : tr)
        if (!(v >= 0.0f && v <= 0.5f)) return fail(RTX_ERR_INVALID, "rtx_set_schedule: trace_* must be in [0, 0.5]");
    if (s->tier1_priority > 3 || s->tier2_priority > 3 || s->hot_priority > 3)
        return fail(RTX_ERR_INVALID, "rtx_set_schedule: priorities must be in 0..3");
    if (s->refill_chunk > 4096) return fail(RTX_ERR_INVALID, "rtx_set_schedule: refill_chunk must be in 0..4096");
    if (s->trace_group != 1 && s->trace_group != 2 && s->trace_group != 4 && s->trace_group != 8)
        return fail(RTX_ERR_INVALID, "rtx_set_schedule: trace_group must be 1, 2, 4 or 8");
    if (s->prepass_cap_split > 4096)
        return fail(RTX_ERR_INVALID, "rtx_set_schedule: prepass_cap_split must be in 0..4096");
    if (!(s->prio_bar1 == 0.0f || (s->prio_bar1 > 0.0f && s->prio_bar1 <= s->prio_bar2 &&
                                   s->prio_bar2 <= s->prio_bar3 && s->prio_bar3 <= 1e30f)))
        return fail(RTX_ERR_INVALID, "rtx_set_schedule: prio_bar1..3 must be 0 or 0 < bar1 <= bar2 <= bar3 <= 1e30");
    if (s->reserved != 0) return fail(RTX_ERR_INVALID, "rtx_set_schedule: reserved must be 0");
    rtx::KTune t;
    t.a1 = s->tier1_bar;
    t.a1_small = s->tier1_bar_small;
    t.a1_low = s->tier1_bar_low;
    t.a2_small = s->tier2_bar_small;
    t.a2_medium = s->tier2_bar_medium;
    t.a2_large = s->tier2_bar;
    t.rho = s->small_share;
    t.rho_low = s->low_share;
    t.rho2 = s->medium_share;
    t.prio_frac = s->hot_fraction;
    t.occ_small = s->occupancy_small;
    t.occ_low = s->occupancy_low;
    t.occ_normal = s->occupancy_normal;
    t.coop_max = s->tail_coop_max;
    t.coop_max_large = s->tail_coop_max_large;
    t.trace_small = s->trace_small;
    t.trace_low = s->trace_low;
    t.trace_medium = s->trace_medium;
    t.trace_large = s->trace_large;
    t.prom_small = s->promote_small;
    t.prom_low = s->promote_low;
    t.prom_medium = s->promote_medium;
    t.prom_large = s->promote_large;
    t.prom_big = s->promote_big_scene;
    t.prio_t1 = s->tier1_priority;
    t.prio_t2 = s->tier2_priority;
    t.prio_hot = s->hot_priority;
    t.chunk = s->refill_chunk;
    t.trace_group = s->trace_group;
    t.trace_solo = s->trace_solo_bar;
    t.cap_split = s->prepass_cap_split;
    t.dyn1 = s->prio_bar1;
    t.dyn2 = s->prio_bar1 > 0.0f ? s->prio_bar2 : 0.0f;
    t.dyn3 = s->prio_bar1 > 0.0f ? s->prio_bar3 : 0.0f;
    c->tune = t;
    return RTX_OK;
}

int rtx_get_schedule(rtx_ctx *c, rtx_schedule *out) {
    if (!c || !out) return fail(RTX_ERR_INVALID, "rtx_get_schedule: null argument");
    const rtx::KTune &t = c->tune;
    *out = rtx_schedule{};
    out->tier1_bar = (float)t.a1;
    out->tier1_bar_small = (float)t.a1_small;
    out->tier1_bar_low = (float)t.a1_low;
    out->tier2_bar_small = (float)t.a2_small;
    out->tier2_bar_medium = (float)t.a2_medium;
    out->tier2_bar = (float)std::min(t.a2_large, 1e30);
    out->small_share = (float)t.rho;
    out->low_share = (float)t.rho_low;
    out->medium_share = (float)t.rho2;
    out->hot_fraction = (float)t.prio_frac;
    out->occupancy_small = (float)t.occ_small;
    out->occupancy_low = (float)t.occ_low;
    out->occupancy_normal = (float)t.occ_normal;
    out->tail_coop_max = t.coop_max;
    out->tail_coop_max_large = t.coop_max_large;
    out->trace_small = (float)t.trace_small;
    out->trace_low = (float)t.trace_low;
    out->trace_medium = (float)t.trace_medium;
    out->trace_large = (float)t.trace_large;
    out->promote_small = (float)t.prom_small;
    out->promote_low = (float)t.prom_low;
    out->promote_medium = (float)t.prom_medium;
    out->promote_large = (float)t.prom_large;
    out->promote_big_scene = (float)t.prom_big;
    out->tier1_priority = t.prio_t1;
    out->tier2_priority = t.prio_t2;
    out->hot_priority = t.prio_hot;
    out->refill_chunk = t.chunk;
    out->trace_group = t.trace_group;
    out->trace_solo_bar = (float)std::min(t.trace_solo, 1e30);
    out->prepass_cap_split = t.cap_split;
    out->prio_bar1 = (float)t.dyn1;
    out->prio_bar2 = (float)t.dyn2;
    out->prio_bar3 = (float)t.dyn3;
    return RTX_OK;
}

// The culled layout (rtx_internal.h KScene, rtx_prefilter.h cull_bound):
// sections of spheres — large ones (r > 8x the median), the other non-flat
// ones, the flat ones (height flat_cy, when the scene has a flat run) — each
// in Morton order of its centres (x, z for the flat section; x, y, z
// otherwise) and padded to whole blocks with copies of its last sphere whose
// prefilter R is -inf: never flagged (Q = -inf), except by a lane outside the
// prefilter's safe region (thr = -inf flags everything), which then resolves
// the copy to the same key as the sphere itself — no result changes either way.
struct CullLayout {
    std::vector<float> pre, bnd, bnd2, bnd3;
    std::vector<uint32_t> perm;
    std::vector<uint8_t> pad;  // position holds a padding copy
    uint32_t flat_lo = 0;
};
static CullLayout build_cull(const rtx_world *w, const std::vector<float4> &pre4, bool has_flat, float flat_cy) {
    const uint32_t n = w->count;
    const float *S = w->spheres;
    std::vector<float> rs(n);
    for (uint32_t i = 0; i < n; ++i) rs[i] = std::fabs(S[4 * i + 3]);
    std::nth_element(rs.begin(), rs.begin() + n / 2, rs.end());
    const float big = 8.0f * rs[n / 2];
    std::vector<uint32_t> sec[3];
    for (uint32_t i = 0; i < n; ++i) {
        const bool fl = has_flat && __builtin_bit_cast(uint32_t, S[4 * i + 1]) == __builtin_bit_cast(uint32_t, flat_cy);
        sec[std::fabs(S[4 * i + 3]) > big ? 0 : fl ? 2 : 1].push_back(i);
    }
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) lo[k] = std::min(lo[k], (double)S[4 * i + k]), hi[k] = std::max(hi[k], (double)S[4 * i + k]);
    auto q = [&](uint32_t i, int k) -> uint64_t {
        const double span = hi[k] - lo[k];
        return span > 0.0 ? (uint64_t)std::min(1023.0, std::floor(((double)S[4 * i + k] - lo[k]) / span * 1024.0)) : 0;
    };
    auto morton = [&](uint32_t i, bool flat) {
        uint64_t key = 0;
        for (int bit = 0; bit < 10; ++bit) {
            if (flat)
                key |= ((q(i, 0) >> bit) & 1u) << (2 * bit) | ((q(i, 2) >> bit) & 1u) << (2 * bit + 1);
            else
                key |= ((q(i, 0) >> bit) & 1u) << (3 * bit) | ((q(i, 1) >> bit) & 1u) << (3 * bit + 1) |
                       ((q(i, 2) >> bit) & 1u) << (3 * bit + 2);
        }
        return key;
    };
    CullLayout L;
    for (int k = 0; k < 3; ++k) {
        if (sec[k].empty()) continue;
        std::stable_sort(sec[k].begin(), sec[k].end(),
                         [&](uint32_t a, uint32_t b) { return morton(a, k == 2) < morton(b, k == 2); });
        if (k == 2) {
            // the flat section starts at a multiple of kCullAlign blocks, so
            // that no bound test (8 entries of 1, 8 or 64 blocks) mixes flat
            // and non-flat bounds; the padding blocks' bounds never pass (R = -inf)
            while (!L.perm.empty() && (L.perm.size() / 8) % rtx::kCullAlign != 0) {
                const uint32_t last = L.perm.back();
                for (int i = 0; i < 8; ++i) L.perm.push_back(last), L.pad.push_back(1);
            }
            L.flat_lo = (uint32_t)L.perm.size() / 8;
        }
        for (uint32_t i : sec[k]) L.perm.push_back(i), L.pad.push_back(0);
        while (L.perm.size() % 8) L.perm.push_back(sec[k].back()), L.pad.push_back(1);
    }
    if (sec[2].empty()) L.flat_lo = (uint32_t)L.perm.size() / 8;
    const uint32_t np = (uint32_t)L.perm.size(), nblk = np / 8, ngrp = (nblk + 7) / 8;
    // the bound of positions [p0, p1): over their spheres; R = -inf when they are all padding
    auto bound_of = [&](uint32_t p0, uint32_t p1, bool fl) {
        std::vector<const float *> sp;
        bool all_pad = true;
        for (uint32_t p = p0; p < std::min(p1, np); ++p) sp.push_back(&S[4 * (size_t)L.perm[p]]), all_pad &= L.pad[p] != 0;
        rtx::CullBound cb = rtx::cull_bound(sp.data(), (int)sp.size(), fl, flat_cy, fl ? rtx::kCullSy : 1.0f);
        if (all_pad) cb.R = -INFINITY;
        return cb;
    };
    L.pre.assign(4 * (size_t)np, 0.0f);
    for (uint32_t p = 0; p < np; ++p) {
        const float4 v = pre4[L.perm[p]];
        float *blk = &L.pre[32 * (size_t)(p / 8)];
        blk[p % 8] = v.x, blk[8 + p % 8] = v.y, blk[16 + p % 8] = v.z, blk[24 + p % 8] = L.pad[p] ? -INFINITY : v.w;
    }
    L.bnd.assign(32 * (size_t)ngrp, 0.0f);
    for (uint32_t g = 0; g < ngrp; ++g)
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t b = 8 * g + j;
            float *gb = &L.bnd[32 * (size_t)g];
            if (b >= nblk) {  // past the last block: masked off by the kernel; flat height for a flat group
                gb[8 + j] = 8 * g >= L.flat_lo ? rtx::kCullSy * flat_cy : 0.0f;
                continue;
            }
            const rtx::CullBound cb = bound_of(8 * b, 8 * b + 8, b >= L.flat_lo);  // flat: stretched along y
            gb[j] = cb.cx, gb[8 + j] = cb.cy, gb[16 + j] = cb.cz, gb[24 + j] = cb.R;
        }
    // the top level: one bound over each group's 64 spheres, 8 groups per super-group
    const uint32_t nsg = (ngrp + 7) / 8;
    L.bnd2.assign(32 * (size_t)nsg, 0.0f);
    for (uint32_t s = 0; s < nsg; ++s)
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t g = 8 * s + j;
            float *gb = &L.bnd2[32 * (size_t)s];
            if (g >= ngrp) {
                gb[8 + j] = 64 * s >= L.flat_lo ? rtx::kCullSy * flat_cy : 0.0f;
                continue;
            }
            const rtx::CullBound cb = bound_of(64 * g, 64 * g + 64, 8 * g >= L.flat_lo);
            gb[j] = cb.cx, gb[8 + j] = cb.cy, gb[16 + j] = cb.cz, gb[24 + j] = cb.R;
        }
    // the third level: one bound over each super-group's 512 spheres, 8 per entry of bnd3
    const uint32_t nhg = (nsg + 7) / 8;
    L.bnd3.assign(32 * (size_t)nhg, 0.0f);
    for (uint32_t h = 0; h < nhg; ++h)
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t sg = 8 * h + j;
            float *gb = &L.bnd3[32 * (size_t)h];
            if (sg >= nsg) {
                gb[8 + j] = 512 * h >= L.flat_lo ? rtx::kCullSy * flat_cy : 0.0f;
                continue;
            }
            const rtx::CullBound cb = bound_of(512 * sg, 512 * sg + 512, 64 * sg >= L.flat_lo);
            gb[j] = cb.cx, gb[8 + j] = cb.cy, gb[16 + j] = cb.cz, gb[24 + j] = cb.R;
        }
    return L;
}

int rtx_upload_world(rtx_ctx *c, const rtx_world *w) {
    if (!c || !w) return fail(RTX_ERR_INVALID, "rtx_upload_world: null argument");
    if (w->reserved != 0) return fail(RTX_ERR_INVALID, "rtx_upload_world: reserved must be 0");
    if (w->count > 0 && (!w->spheres || !w->mat_types || !w->mat_values))
        return fail(RTX_ERR_INVALID, "rtx_upload_world: null array with count > 0");
    // Exactness bound of the kernel's all-miss test (rtx_kernels.hip,
    // RTX_ANYMAX): finite scene values of magnitude <= 1e15 keep every
    // ray-sphere discriminant of a finite ray free of fp32 overflow.
    for (uint32_t i = 0; i < w->count; ++i)
        for (int k = 0; k < 4; ++k) {
            const float v = w->spheres[4 * i + k];
            if (!(v >= -1e15f && v <= 1e15f))
                return fail(RTX_ERR_INVALID, "rtx_upload_world: sphere " + std::to_string(i) +
                                                 " has a non-finite or |value| > 1e15 component");
        }
    // The prefiltered scan's list entries hold a 24-bit local sphere index.
    if (w->count > (1u << 24) - rtx::kPad)
        return fail(RTX_ERR_INVALID, "rtx_upload_world: more than 16,777,208 spheres");
    int rc = set_device(c);
    if (rc) return rc;
    const uint32_t n = w->count;
    const uint32_t n_pad = (n + rtx::kPad - 1) / rtx::kPad * rtx::kPad;
    std::vector<float> soa(4 * (size_t)n_pad), pre(4 * (size_t)n_pad);
    double smag = 0.0;  // max |c| + |r|, for the prefilter's overflow guard
    std::vector<float4> cen(n), mval(n), pre4(n);
    std::vector<int> mtype(n);
    for (uint32_t i = 0; i < n_pad; ++i) {
        // padding: copies of sphere n-1 (see rtx::KScene)
        const uint32_t k = i < n ? i : n - 1;
        const float r = w->spheres[4 * k + 3];
        float *blk = &soa[32 * (size_t)(i / 8)];
        blk[i % 8] = w->spheres[4 * k + 0];
        blk[8 + i % 8] = w->spheres[4 * k + 1];
        blk[16 + i % 8] = w->spheres[4 * k + 2];
        const float r2 = r * r;
        blk[24 + i % 8] = -r2;
        float *pb = &pre[32 * (size_t)(i / 8)];
        pb[i % 8] = blk[i % 8];
        pb[8 + i % 8] = blk[8 + i % 8];
        pb[16 + i % 8] = blk[16 + i % 8];
        pb[24 + i % 8] = rtx::prefilter_R(blk[i % 8], blk[8 + i % 8], blk[16 + i % 8], r2);
        const double cx = blk[i % 8], cy = blk[8 + i % 8], cz = blk[16 + i % 8];
        smag = std::max(smag, std::sqrt(cx * cx + cy * cy + cz * cz) + std::fabs((double)r));
        if (i < n) pre4[i] = make_float4(pb[i % 8], pb[8 + i % 8], pb[16 + i % 8], pb[24 + i % 8]);
    }
    float smag_f = (float)smag;
    if ((double)smag_f < smag) smag_f = std::nextafter(smag_f, INFINITY);
    // The longest run of flat blocks (rtx_prefilter.h: all 8 centre heights
    // equal, bit for bit, and equal along the run): the scan's 5-op test.
    uint32_t flat_lo = 0, flat_hi = 0;
    float flat_cy = 0.0f;
    {
        auto bits = [&](uint32_t b, int k) { return __builtin_bit_cast(uint32_t, pre[32 * (size_t)b + 8 + k]); };
        auto flat = [&](uint32_t b) {
            for (int k = 1; k < 8; ++k)
                if (bits(b, k) != bits(b, 0)) return false;
            return true;
        };
        const uint32_t nblk = RTX_FLAT ? n_pad / 8 : 0;  // RTX_FLAT=0: A/B build without flat runs
        for (uint32_t b = 0; b < nblk;) {
            if (!flat(b)) {
                ++b;
                continue;
            }
            uint32_t e = b + 1;
            while (e < nblk && flat(e) && bits(e, 0) == bits(b, 0)) ++e;
            if (e - b > flat_hi - flat_lo) flat_lo = b, flat_hi = e, flat_cy = pre[32 * (size_t)b + 8];
            b = e;
        }
    }
    for (uint32_t i = 0; i < n; ++i) {
        cen[i] = make_float4(w->spheres[4 * i + 0], w->spheres[4 * i + 1], w->spheres[4 * i + 2],
                             w->spheres[4 * i + 3]);
        // The shader compares the float code with 0, 1, 2 (:209,219,229);
        // anything else does not scatter.
        const float t = w->mat_types[i];
        mtype[i] = (t == 0.0f) ? 0 : (t == 1.0f) ? 1 : (t == 2.0f) ? 2 : 3;
        mval[i] = make_float4(w->mat_values[4 * i + 0], w->mat_values[4 * i + 1],
                              w->mat_values[4 * i + 2], w->mat_values[4 * i + 3]);
    }
    CullLayout cl;
    const bool linear = c->scan_mode == RTX_SCAN_LINEAR;  // every block of every segment: no grid, no culled copy
    const bool cull = RTX_CULL && !linear && n_pad > rtx::kScanPfMin;  // the large-scene (kPF) kernels scan it
    if (cull) cl = build_cull(w, pre4, flat_hi > flat_lo, flat_cy);
    // the small-scene lane-mode scan's layer grid over the flat run (rtx_grid.h)
    rtx::LayerGrid grid{};
    std::vector<unsigned long long> gcell;
    const bool has_grid = RTX_GRID_UPLOAD && !linear && n_pad <= rtx::kScanPfMin && flat_hi > flat_lo &&
                          rtx::build_layer_grid(w->spheres, 8 * flat_lo, std::min(8 * flat_hi, n), grid, gcell);
    RTX_HIP(hipStreamSynchronize(c->stream));
    free_world(c);
    const size_t cap = n ? n : 1;
    RTX_HIP(hipMalloc(&c->d_soa, (n_pad ? 4 * (size_t)n_pad : 4) * sizeof(float)));
    RTX_HIP(hipMalloc(&c->d_pre, (n_pad ? 4 * (size_t)n_pad : 4) * sizeof(float)));
    RTX_HIP(hipMalloc(&c->d_pre4, cap * sizeof(float4)));
    RTX_HIP(hipMalloc(&c->d_cen, cap * sizeof(float4)));
    RTX_HIP(hipMalloc(&c->d_mtype, cap * sizeof(int)));
    RTX_HIP(hipMalloc(&c->d_mval, cap * sizeof(float4)));
    // All copies on the context stream (a non-blocking stream does not
    // order against the legacy null stream), then wait for them.
    if (n) {
        RTX_HIP(hipMemcpyAsync(c->d_soa, soa.data(), soa.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
        RTX_HIP(hipMemcpyAsync(c->d_pre, pre.data(), pre.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
        RTX_HIP(hipMemcpyAsync(c->d_pre4, pre4.data(), n * sizeof(float4), hipMemcpyHostToDevice, c->stream));
        RTX_HIP(hipMemcpyAsync(c->d_cen, cen.data(), n * sizeof(float4), hipMemcpyHostToDevice, c->stream));
        RTX_HIP(hipMemcpyAsync(c->d_mtype, mtype.data(), n * sizeof(int), hipMemcpyHostToDevice, c->stream));
        RTX_HIP(hipMemcpyAsync(c->d_mval, mval.data(), n * sizeof(float4), hipMemcpyHostToDevice, c->stream));
        RTX_HIP(hipStreamSynchronize(c->stream));
    }
    if (cull) {
        RTX_HIP(hipMalloc(&c->d_cpre, cl.pre.size() * sizeof(float)));
        RTX_HIP(hipMalloc(&c->d_cbnd, cl.bnd.size() * sizeof(float)));
        RTX_HIP(hipMalloc(&c->d_cbnd2, cl.bnd2.size() * sizeof(float)));
        RTX_HIP(hipMalloc(&c->d_cbnd3, cl.bnd3.size() * sizeof(float)));
        RTX_HIP(hipMemcpyAsync(c->d_cbnd3, cl.bnd3.data(), cl.bnd3.size() * sizeof(float), hipMemcpyHostToDevice,
                               c->stream));
        RTX_HIP(hipMemcpyAsync(c->d_cbnd2, cl.bnd2.data(), cl.bnd2.size() * sizeof(float), hipMemcpyHostToDevice,
                               c->stream));
        RTX_HIP(hipMalloc(&c->d_cperm, cl.perm.size() * sizeof(uint32_t)));
        RTX_HIP(hipMalloc(&c->d_ccen, cl.perm.size() * sizeof(float4)));
        std::vector<float4> ccen(cl.perm.size());
        for (size_t p = 0; p < ccen.size(); ++p) ccen[p] = cen[cl.perm[p]];
        RTX_HIP(hipMemcpyAsync(c->d_ccen, ccen.data(), ccen.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
        RTX_HIP(hipMemcpyAsync(c->d_cpre, cl.pre.data(), cl.pre.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
        RTX_HIP(hipMemcpyAsync(c->d_cbnd, cl.bnd.data(), cl.bnd.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
        RTX_HIP(hipMemcpyAsync(c->d_cperm, cl.perm.data(), cl.perm.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                               c->stream));
        RTX_HIP(hipStreamSynchronize(c->stream));
        c->n_cpad = (uint32_t)cl.perm.size();
        c->cflat_lo = cl.flat_lo;
    }
    if (has_grid) {
        static_assert(sizeof(rtx::LayerGrid) % 8 == 0, "the cells follow the LayerGrid, 8-byte aligned");
        std::vector<unsigned long long> buf(sizeof(rtx::LayerGrid) / 8 + gcell.size());
        std::memcpy(buf.data(), &grid, sizeof grid);
        std::memcpy(buf.data() + sizeof(rtx::LayerGrid) / 8, gcell.data(), gcell.size() * sizeof(unsigned long long));
        RTX_HIP(hipMalloc(&c->d_grid, buf.size() * sizeof(unsigned long long)));
        RTX_HIP(hipMemcpyAsync(c->d_grid, buf.data(), buf.size() * sizeof(unsigned long long), hipMemcpyHostToDevice,
                               c->stream));
        RTX_HIP(hipStreamSynchronize(c->stream));
    }
    if (c->n != n) c->n_changed = true;
    c->n = n;
    c->n_pad = n_pad;
    c->smag = smag_f;
    c->flat_cy = flat_cy;
    c->flat_lo = flat_lo;
    c->flat_hi = flat_hi;
    c->depth = w->depth;
    c->spp = w->spp;
    c->have_world = true;
    return RTX_OK;
}

int rtx_set_scan_mode(rtx_ctx *c, int mode) {
    if (!c) return fail(RTX_ERR_INVALID, "rtx_set_scan_mode: null ctx");
    if (mode != RTX_SCAN_AUTO && mode != RTX_SCAN_LINEAR) return fail(RTX_ERR_INVALID, "rtx_set_scan_mode: unknown mode");
    c->scan_mode = mode;
    return RTX_OK;
}

int rtx_set_frame(rtx_ctx *c, const rtx_frame *f) {
    if (!c || !f) return fail(RTX_ERR_INVALID, "rtx_set_frame: null argument");
    if (f->width == 0 || f->height == 0)
        return fail(RTX_ERR_INVALID, "rtx_set_frame: zero width or height");
    if (f->rng_mode > 1) return fail(RTX_ERR_INVALID, "rtx_set_frame: unknown rng_mode");
    if ((f->flags & ~(uint32_t)RTX_FRAME_LAMBERT_GUARD) != 0 || f->reserved != 0)
        return fail(RTX_ERR_INVALID, "rtx_set_frame: unknown flags or nonzero reserved");
    if (!(f->lens_u[3] >= 0.0f)) return fail(RTX_ERR_INVALID, "rtx_set_frame: negative lens radius");
    if ((uint64_t)f->width * f->height > (1ull << 31))
        return fail(RTX_ERR_INVALID, "rtx_set_frame: more than 2^31 pixels");
    c->frame = *f;
    c->have_frame = true;
    return RTX_OK;
}

uint32_t rtx_part_rows(uint32_t height, uint32_t tile_rows, uint32_t part, uint32_t nparts) {
    if (tile_rows == 0 || nparts == 0 || part >= nparts) return 0;
    const uint32_t tiles = (height + tile_rows - 1) / tile_rows;
    if (part >= tiles) return 0;
    const uint32_t my_tiles = (tiles - part + nparts - 1) / nparts;  // tiles part, part+nparts, ...
    uint32_t rows = my_tiles * tile_rows;
    const uint32_t last_tile = part + (my_tiles - 1) * nparts;
    if (last_tile == tiles - 1) rows -= tiles * tile_rows - height;  // ragged final tile
    return rows;
}

static int render_impl(rtx_ctx *c, uint32_t tile_rows, uint32_t part, uint32_t nparts, void *d_out,
                       float4 *accum, uint32_t accum_frames, uint32_t frame_index);

// Scheduling scratch (words): cost[npix] perm[npix] buckets[2K + kSchedWords], then the
// per-pixel pre-pass state (float4, 16-byte aligned).
static size_t sched_state_off(size_t npix) { return (2 * npix + 2 * rtx::kCostBuckets + rtx::kSchedWords + 3) & ~(size_t)3; }
constexpr uint32_t kPromCap = 65536;  // promotion queue entries (8 words each)

int rtx_render_rows(rtx_ctx *c, uint32_t tile_rows, uint32_t part, uint32_t nparts, void *d_out) {
    if (!c) return fail(RTX_ERR_INVALID, "rtx_render_rows: null ctx");
    return render_impl(c, tile_rows, part, nparts, d_out, nullptr, 0, c->frame.frame_index);
}

int rtx_accumulate(rtx_ctx *c, int reset) {
    if (!c) return fail(RTX_ERR_INVALID, "rtx_accumulate: null ctx");
    if (!c->have_frame) return fail(RTX_ERR_STATE, "rtx_accumulate: no frame set");
    int rc = set_device(c);
    if (rc) return rc;
    const size_t px = (size_t)c->frame.width * c->frame.height;
    // a frame of another size restarts the accumulation (the accumulator is
    // indexed by pixel: it must hold exactly width*height sums)
    if (reset || c->accum_frames == 0 || !c->d_accum || c->accum_pixels != px) {
        if (!c->d_accum || c->accum_pixels != px) {
            RTX_HIP(hipStreamSynchronize(c->stream));
            (void)hipFree(c->d_accum);
            c->d_accum = nullptr;
            c->accum_pixels = 0;
            RTX_HIP(hipMalloc(&c->d_accum, px * sizeof(float4)));
            c->accum_pixels = px;
        }
        RTX_HIP(hipMemsetAsync(c->d_accum, 0, px * sizeof(float4), c->stream));
        c->accum_frames = 0;
    }
    rc = render_impl(c, 1, 0, 1, nullptr, c->d_accum, c->accum_frames + 1, c->accum_frames);
    if (rc == RTX_OK) c->accum_frames++;
    return rc;
}

uint32_t rtx_accumulated_frames(rtx_ctx *c) { return c ? c->accum_frames : 0; }

static rtx::KParams make_params(const rtx_ctx *c, uint32_t rows, uint32_t tile_rows, uint32_t part,
                                uint32_t nparts, float4 *out, float4 *accum, uint32_t accum_frames,
                                uint32_t frame_index) {
    const rtx_frame &f = c->frame;
    rtx::KParams p{};
    p.scene = scene_of(c);
    p.out = out;
    p.counters = c->d_counters;
    p.queue = reinterpret_cast<uint32_t *>(c->d_counters + 2);
    p.errors = reinterpret_cast<uint32_t *>(c->d_counters + kErrWord);
    p.err_diag = c->d_counters + kErrDiag;
    p.depth = c->depth;
    p.spp = c->spp;
    p.width = f.width;
    p.rows_local = rows;
    p.tile_rows = tile_rows;
    p.part = part;
    p.nparts = nparts;
    p.rng_mode = f.rng_mode;
    p.frame_index = frame_index;
    p.flags = f.flags;
    p.accum = accum;
    p.accum_frames = accum_frames;
    for (int k = 0; k < 3; ++k) {
        p.lens_u[k] = f.lens_u[k];
        p.lens_v[k] = f.lens_v[k];
    }
    p.lens_r = f.lens_u[3];
    p.wave_times = c->d_wave_times;
    p.wave_cap = (uint32_t)std::min<size_t>(c->wave_times_cap, 0xffffffffu);
    for (int k = 0; k < 3; ++k) {
        p.org[k] = f.origin[k];
        p.hor[k] = f.horizontal[k];
        p.ver[k] = f.vertical[k];
        p.llc[k] = f.lower_left[k];
    }
    p.img_w = f.img_w;
    p.img_h = f.img_h;
    return p;
}

static int render_impl(rtx_ctx *c, uint32_t tile_rows, uint32_t part, uint32_t nparts, void *d_out,
                       float4 *accum, uint32_t accum_frames, uint32_t frame_index) {
    if (!c->have_world) return fail(RTX_ERR_STATE, "rtx_render_rows: no world uploaded");
    if (!c->have_frame) return fail(RTX_ERR_STATE, "rtx_render_rows: no frame set");
    if (tile_rows == 0 || nparts == 0 || part >= nparts)
        return fail(RTX_ERR_INVALID, "rtx_render_rows: bad partition");
    int rc = set_device(c);
    if (rc) return rc;
    const rtx_frame &f = c->frame;
    const uint32_t rows = rtx_part_rows(f.height, tile_rows, part, nparts);
    float4 *out = reinterpret_cast<float4 *>(d_out);
    if (!out) {
        if (nparts != 1) return fail(RTX_ERR_INVALID, "rtx_render_rows: d_out NULL needs nparts == 1");
        const size_t px = (size_t)f.width * f.height;
        if (c->fb_pixels != px) {
            RTX_HIP(hipStreamSynchronize(c->stream));
            (void)hipFree(c->d_fb);
            c->d_fb = nullptr;
            c->fb_pixels = 0;
            RTX_HIP(hipMalloc(&c->d_fb, px * sizeof(float4)));
            c->fb_pixels = px;
        }
        out = c->d_fb;
    }
    rtx::KParams p = make_params(c, rows, tile_rows, part, nparts, out, accum, accum_frames, frame_index);

    if (c->ev_count == c->events.size()) {
        EventPair &old = c->events[c->ev_head];
        const hipError_t q = hipEventQuery(old.stop);
        if (q == hipSuccess) {  // recycle the oldest pair: fold its duration
            float t = 0.0f;
            RTX_HIP(hipEventElapsedTime(&t, old.start, old.stop));
            c->ms_folded += t;
            c->ev_head = (c->ev_head + 1) % c->events.size();
            c->ev_count--;
        } else if (q == hipErrorNotReady) {  // still running: grow the ring, no wait
            std::vector<EventPair> grown(2 * c->events.size());
            for (size_t i = 0; i < c->ev_count; ++i) grown[i] = c->events[(c->ev_head + i) % c->events.size()];
            c->events.swap(grown);
            c->ev_head = 0;
        } else {
            return hip_fail(q, "hipEventQuery");
        }
    }
    EventPair &ev = c->events[(c->ev_head + c->ev_count) % c->events.size()];
    if (!ev.start) RTX_HIP(hipEventCreate(&ev.start));
    if (!ev.stop) RTX_HIP(hipEventCreate(&ev.stop));
    RTX_HIP(hipEventRecord(ev.start, c->stream));
    const size_t npix = (size_t)rows * f.width;
    if (c->sched_pixels < npix) {
        RTX_HIP(hipStreamSynchronize(c->stream));
        (void)hipFree(c->d_sched);
        c->d_sched = nullptr;
        c->sched_pixels = 0;
        // cost, perm, buckets; then 16-byte aligned per-pixel state
        // ... the promotion queue, then the slot-ordered image staging (float4) and the inverse permutation
        RTX_HIP(hipMalloc(&c->d_sched,
                          (sched_state_off(npix) + 4 * npix + 8 * (size_t)kPromCap + 5 * npix) * sizeof(uint32_t)));
        // the promotion queue's epoch words start below every launch's epoch
        RTX_HIP(hipMemsetAsync(c->d_sched + sched_state_off(npix) + 4 * npix, 0,
                               8 * (size_t)kPromCap * sizeof(uint32_t), c->stream));
        c->sched_pixels = npix;
    }
    const size_t ps_need = rtx::ps_scratch_floats(p);
    if (ps_need > c->ps_floats) {
        RTX_HIP(hipStreamSynchronize(c->stream));
        (void)hipFree(c->d_ps);
        c->d_ps = nullptr;
        c->ps_floats = 0;
        RTX_HIP(hipMalloc(&c->d_ps, ps_need * sizeof(float)));
        c->ps_floats = ps_need;
    }
    rtx::KSchedule sched;
    sched.ps_scratch = c->d_ps;
    sched.ps_floats = c->ps_floats;
    sched.cost = c->d_sched;
    sched.perm = c->d_sched + c->sched_pixels;
    sched.buckets = c->d_sched + 2 * c->sched_pixels;
    sched.state = reinterpret_cast<float4 *>(c->d_sched + sched_state_off(c->sched_pixels));
    sched.npix = (uint32_t)c->sched_pixels;
    sched.nbuckets = rtx::kCostBuckets;
    sched.tune = c->tune;
    if (!c->aux_stream) {
        RTX_HIP(hipStreamCreateWithFlags(&c->aux_stream, hipStreamNonBlocking));
        RTX_HIP(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
        RTX_HIP(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
    }
    sched.aux = c->aux_stream;
    sched.prom_q = c->d_sched + sched_state_off(c->sched_pixels) + 4 * c->sched_pixels;
    sched.prom_cap = kPromCap;
    sched.stage = reinterpret_cast<float4 *>(sched.prom_q + 8 * (size_t)kPromCap);  // 16-byte aligned
    sched.inv = sched.prom_q + 8 * (size_t)kPromCap + 4 * c->sched_pixels;
    sched.epoch = (uint32_t)++c->epoch;
    sched.ev_fork = c->ev_fork;
    sched.ev_join = c->ev_join;
    hipError_t e = rtx::launch_render(p, sched, c->stream);
    if (e != hipSuccess) return hip_fail(e, "launch_render");
    RTX_HIP(hipEventRecord(ev.stop, c->stream));
    c->ev_count++;
    c->launches++;
    c->samples += (uint64_t)rows * f.width * c->spp;
    return RTX_OK;
}

int rtx_render(rtx_ctx *c) { return rtx_render_rows(c, 1, 0, 1, nullptr); }

int rtx_deinterleave_rows(rtx_ctx *c, const void *d_gathered, uint32_t width, uint32_t height,
                          uint32_t tile_rows, uint32_t nparts, void *d_image) {
    if (!c || !d_gathered || !d_image) return fail(RTX_ERR_INVALID, "rtx_deinterleave_rows: null argument");
    if (tile_rows == 0 || nparts == 0) return fail(RTX_ERR_INVALID, "rtx_deinterleave_rows: bad partition");
    int rc = set_device(c);
    if (rc) return rc;
    const uint32_t max_rows = rtx_part_rows(height, tile_rows, 0, nparts);  // part 0 is largest
    hipError_t e = rtx::launch_deinterleave(reinterpret_cast<const float4 *>(d_gathered),
                                            reinterpret_cast<float4 *>(d_image), width, height,
                                            tile_rows, nparts, max_rows, c->stream);
    if (e != hipSuccess) return hip_fail(e, "launch_deinterleave");
    return RTX_OK;
}

int rtx_sync(rtx_ctx *c) {
    if (!c) return fail(RTX_ERR_INVALID, "rtx_sync: null ctx");
    int rc = set_device(c);
    if (rc) return rc;
    RTX_HIP(hipStreamSynchronize(c->stream));
    return check_errors(c, "rtx_sync");
}

void *rtx_framebuffer(rtx_ctx *c) { return c ? c->d_fb : nullptr; }

int rtx_download(rtx_ctx *c, float *host, size_t bytes) {
    if (!c || !host) return fail(RTX_ERR_INVALID, "rtx_download: null argument");
    if (!c->d_fb) return fail(RTX_ERR_STATE, "rtx_download: nothing rendered into the context framebuffer");
    if (bytes != c->fb_pixels * sizeof(float4))
        return fail(RTX_ERR_INVALID, "rtx_download: bytes != width*height*16");
    int rc = set_device(c);
    if (rc) return rc;
    RTX_HIP(hipMemcpyAsync(host, c->d_fb, bytes, hipMemcpyDeviceToHost, c->stream));
    RTX_HIP(hipStreamSynchronize(c->stream));
    return check_errors(c, "rtx_download");
}

int rtx_stats_reset(rtx_ctx *c) {
    if (!c) return fail(RTX_ERR_INVALID, "rtx_stats_reset: null ctx");
    int rc = set_device(c);
    if (rc) return rc;
    rc = check_errors(c, "rtx_stats_reset");  // an unreported error of earlier launches
    RTX_HIP(hipMemsetAsync(c->d_counters, 0, kCounterWords * sizeof(unsigned long long), c->stream));
    RTX_HIP(hipStreamSynchronize(c->stream));
    c->ev_head = 0;
    c->ev_count = 0;
    c->ms_folded = 0.0;
    c->samples = 0;
    c->launches = 0;
    c->n_changed = false;
    return rc;
}

int rtx_get_stats(rtx_ctx *c, rtx_stats *out) {
    if (!c || !out) return fail(RTX_ERR_INVALID, "rtx_get_stats: null argument");
    if (c->n_changed) return fail(RTX_ERR_STATE, "rtx_get_stats: world changed since rtx_stats_reset");
    int rc = set_device(c);
    if (rc) return rc;
    RTX_HIP(hipStreamSynchronize(c->stream));
    rc = check_errors(c, "rtx_get_stats");
    if (rc) return rc;
    unsigned long long h[4];
    RTX_HIP(hipMemcpyAsync(h, c->d_counters, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    RTX_HIP(hipStreamSynchronize(c->stream));
    double ms = c->ms_folded;
    for (size_t i = 0; i < c->ev_count; ++i) {
        const EventPair &p = c->events[(c->ev_head + i) % c->events.size()];
        float t = 0.0f;
        RTX_HIP(hipEventElapsedTime(&t, p.start, p.stop));
        ms += t;
    }
    out->kernel_ms = ms;
    out->launches = c->launches;
    out->samples = c->samples;
    out->segments = h[0];
    out->sphere_tests = h[0] * (uint64_t)c->n;
    return RTX_OK;
}

int rtx_alloc(rtx_ctx *c, size_t bytes, void **d_ptr) {
    if (!c || !d_ptr) return fail(RTX_ERR_INVALID, "rtx_alloc: null argument");
    *d_ptr = nullptr;
    int rc = set_device(c);
    if (rc) return rc;
    hipError_t e = hipMalloc(d_ptr, bytes ? bytes : 1);
    if (e == hipErrorOutOfMemory) return fail(RTX_ERR_NOMEM, "rtx_alloc: out of device memory");
    if (e != hipSuccess) return hip_fail(e, "hipMalloc");
    return RTX_OK;
}

int rtx_free(rtx_ctx *c, void *d_ptr) {
    if (!c) return fail(RTX_ERR_INVALID, "rtx_free: null ctx");
    if (!d_ptr) return RTX_OK;
    int rc = set_device(c);
    if (rc) return rc;
    RTX_HIP(hipStreamSynchronize(c->stream));
    RTX_HIP(hipFree(d_ptr));
    return RTX_OK;
}

int rtx_copy_to_host(rtx_ctx *c, void *host, const void *d_src, size_t bytes) {
    if (!c || ((!host || !d_src) && bytes)) return fail(RTX_ERR_INVALID, "rtx_copy_to_host: null argument");
    if (!bytes) return RTX_OK;
    int rc = set_device(c);
    if (rc) return rc;
    RTX_HIP(hipMemcpyAsync(host, d_src, bytes, hipMemcpyDeviceToHost, c->stream));
    RTX_HIP(hipStreamSynchronize(c->stream));
    return RTX_OK;
}

int rtx_copy_to_device(rtx_ctx *c, void *d_dst, const void *host, size_t bytes) {
    if (!c || ((!host || !d_dst) && bytes)) return fail(RTX_ERR_INVALID, "rtx_copy_to_device: null argument");
    if (!bytes) return RTX_OK;
    int rc = set_device(c);
    if (rc) return rc;
    RTX_HIP(hipMemcpyAsync(d_dst, host, bytes, hipMemcpyHostToDevice, c->stream));
    RTX_HIP(hipStreamSynchronize(c->stream));
    return RTX_OK;
}

int rtx_debug_pixel_cost(rtx_ctx *c, uint32_t spp, uint32_t *host_cost) {
    if (!c || !host_cost) return fail(RTX_ERR_INVALID, "rtx_debug_pixel_cost: null argument");
    if (!c->have_world || !c->have_frame) return fail(RTX_ERR_STATE, "rtx_debug_pixel_cost: no world/frame");
    int rc = set_device(c);
    if (rc) return rc;
    const rtx_frame &f = c->frame;
    const size_t npix = (size_t)f.width * f.height;
    uint32_t *d = nullptr;
    RTX_HIP(hipMalloc(&d, npix * sizeof(uint32_t)));
    rtx::KParams p = make_params(c, f.height, 1, 0, 1, nullptr, nullptr, 0, f.frame_index);
    if (spp) p.spp = spp;
    p.cost_out = d;
    p.counters = c->d_counters + 3;
    p.wave_times = nullptr;
    hipError_t e = rtx::launch_cost(p, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(host_cost, d, npix * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return hip_fail(e, "rtx_debug_pixel_cost");
    return RTX_OK;
}

int rtx_debug_wave_times(rtx_ctx *c, size_t max_waves, unsigned long long *host_pairs) {
    if (!c) return fail(RTX_ERR_INVALID, "rtx_debug_wave_times: null ctx");
    int rc = set_device(c);
    if (rc) return rc;
    if (max_waves != c->wave_times_cap) {  // (re)arm: allocate and enable recording
        RTX_HIP(hipStreamSynchronize(c->stream));
        (void)hipFree(c->d_wave_times);
        c->d_wave_times = nullptr;
        c->wave_times_cap = 0;
        if (max_waves) {
            RTX_HIP(hipMalloc(&c->d_wave_times, max_waves * 2 * sizeof(unsigned long long)));
            RTX_HIP(hipMemsetAsync(c->d_wave_times, 0, max_waves * 2 * sizeof(unsigned long long), c->stream));
            c->wave_times_cap = max_waves;
        }
        return RTX_OK;
    }
    if (host_pairs && max_waves) {
        RTX_HIP(hipMemcpyAsync(host_pairs, c->d_wave_times, max_waves * 2 * sizeof(unsigned long long),
                               hipMemcpyDeviceToHost, c->stream));
        RTX_HIP(hipStreamSynchronize(c->stream));
    }
    return RTX_OK;
}

int rtx_debug_hit_world_from(rtx_ctx *c, const float *rays, uint32_t nrays, float t_min, float t_max,
                             uint32_t start_block, float *out) {
    if (!c || (nrays && (!rays || !out))) return fail(RTX_ERR_INVALID, "rtx_debug_hit_world: null argument");
    if (!c->have_world) return fail(RTX_ERR_STATE, "rtx_debug_hit_world: no world uploaded");
    // the resolve compares roots by their bit patterns (rtx_kernels.hip
    // hit_key), which order like the values only for roots > 0
    if (!(t_min > 0.0f && t_min <= 3.4e38f))
        return fail(RTX_ERR_INVALID, "rtx_debug_hit_world: t_min must be finite and > 0");
    if (t_max != t_max) return fail(RTX_ERR_INVALID, "rtx_debug_hit_world: t_max is NaN");
    if (nrays == 0) return RTX_OK;
    if (t_max < t_min) {  // no root lies in [t_min, t_max]: every ray misses
        for (size_t i = 0; i < (size_t)nrays; ++i) {
            for (int k = 0; k < 9; ++k) out[10 * i + k] = 0.0f;
            out[10 * i + 9] = -1.0f;
        }
        return RTX_OK;
    }
    int rc = set_device(c);
    if (rc) return rc;
    float *d_rays = nullptr, *d_out = nullptr;
    RTX_HIP(hipMalloc(&d_rays, (size_t)nrays * 6 * sizeof(float)));
    hipError_t e = hipMalloc(&d_out, (size_t)nrays * 10 * sizeof(float));
    if (e == hipSuccess) e = hipMemcpyAsync(d_rays, rays, (size_t)nrays * 6 * sizeof(float), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess)
        e = rtx::launch_debug_hit_world(scene_of(c), d_rays, nrays, t_min, t_max, start_block, d_out, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(out, d_out, (size_t)nrays * 10 * sizeof(float), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d_rays);
    (void)hipFree(d_out);
    if (e != hipSuccess) return hip_fail(e, "rtx_debug_hit_world");
    return RTX_OK;
}

int rtx_debug_hit_world(rtx_ctx *c, const float *rays, uint32_t nrays, float t_min, float t_max, float *out) {
    return rtx_debug_hit_world_from(c, rays, nrays, t_min, t_max, 0, out);
}

int rtx_debug_scan_rate(rtx_ctx *c, uint32_t reps, float *ms, unsigned long long *wave_segments) {
    if (!c || !ms || !wave_segments) return fail(RTX_ERR_INVALID, "rtx_debug_scan_rate: null argument");
    if (!c->have_world) return fail(RTX_ERR_STATE, "rtx_debug_scan_rate: no world uploaded");
    if (!c->have_frame) return fail(RTX_ERR_STATE, "rtx_debug_scan_rate: no frame set");
    int rc = set_device(c);
    if (rc) return rc;
    const rtx_frame &f = c->frame;
    rtx::KParams p = make_params(c, f.height, 1, 0, 1, nullptr, nullptr, 0, f.frame_index);
    if (!rtx::debug_scan_rate_supported(p))  // refused before any HIP call: every HIP error below is hip_fail's
        return fail(RTX_ERR_INVALID, "rtx_debug_scan_rate: scenes up to 640 spheres and a non-empty frame only");
    unsigned long long *sink = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    uint32_t waves = 0;
    RTX_HIP(hipMalloc(&sink, sizeof(unsigned long long)));
    hipError_t e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) e = hipMemsetAsync(sink, 0, sizeof(unsigned long long), c->stream);
    if (e == hipSuccess) e = hipEventRecord(e0, c->stream);
    if (e == hipSuccess) e = rtx::launch_debug_scan_rate(p, reps, sink, &waves, c->stream);
    if (e == hipSuccess) e = hipEventRecord(e1, c->stream);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipEventElapsedTime(ms, e0, e1);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(sink);
    if (e != hipSuccess) return hip_fail(e, "rtx_debug_scan_rate");
    *wave_segments = (unsigned long long)waves * reps;
    return RTX_OK;
}

int rtx_debug_math(rtx_ctx *c, int fn, const float *in0, const float *in1, uint32_t n, float *out) {
    if (!c || (n && (!in0 || !out))) return fail(RTX_ERR_INVALID, "rtx_debug_math: null argument");
    if (fn < RTX_FN_SQRT || fn > RTX_FN_LAMBERT_DIR_GUARD)
        return fail(RTX_ERR_INVALID, "rtx_debug_math: unknown fn");
    const bool vec = fn >= RTX_FN_LAMBERT_DIR;  // in0 = p[3n], in1 = (normal, rius)[6n]
    if (vec && n && !in1) return fail(RTX_ERR_INVALID, "rtx_debug_math: lambert functions need in1");
    if (n == 0) return RTX_OK;
    int rc = set_device(c);
    if (rc) return rc;
    float *d0 = nullptr, *d1 = nullptr, *dout = nullptr;
    const size_t outn = (size_t)n * 3;
    const size_t n0 = vec ? (size_t)n * 3 : (size_t)n, n1 = vec ? (size_t)n * 6 : (size_t)n;
    RTX_HIP(hipMalloc(&d0, n0 * sizeof(float)));
    hipError_t e = hipMalloc(&dout, outn * sizeof(float));
    if (e == hipSuccess && in1) e = hipMalloc(&d1, n1 * sizeof(float));
    if (e == hipSuccess) e = hipMemcpyAsync(d0, in0, n0 * sizeof(float), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess && in1) e = hipMemcpyAsync(d1, in1, n1 * sizeof(float), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(dout, 0, outn * sizeof(float), c->stream);
    if (e == hipSuccess) e = rtx::launch_debug_math(fn, d0, d1, n, dout, c->stream);
    const size_t copy_n = (fn >= RTX_FN_HASH1) ? outn : (size_t)n;
    if (e == hipSuccess) e = hipMemcpyAsync(out, dout, copy_n * sizeof(float), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d0);
    (void)hipFree(d1);
    (void)hipFree(dout);
    if (e != hipSuccess) return hip_fail(e, "rtx_debug_math");
    return RTX_OK;
}

}  // extern "C"
