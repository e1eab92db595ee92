/*
 * rtx.h — C-ABI of the MI355X-native sphere path tracer (librtx.so).
 *
 * This is the drop-in boundary for the reference's GPU path. In
 * Brochu/RayTrace-WE-GPU the host app (CSVersion/DxCSApp.cpp) talks to the
 * GPU through D3D11 objects owned by CDx11Base (CSVersion/Dx11Base.h:11-40):
 *   - cbuffer b1 `WorldDef`   (DxCSApp.cpp:64-71, ShaderCompute.hlsl:12-19),
 *     IMMUTABLE, uploaded once in LoadContent (DxCSApp.cpp:393-413);
 *   - cbuffer b0 `PerFrame`   (DxCSApp.cpp:30-37, ShaderCompute.hlsl:3-10),
 *     DYNAMIC, Map/memcpy/Unmap every Update (DxCSApp.cpp:481-496);
 *   - UAV slot 0 RWTexture2D<float4> (DxCSApp.cpp:326-356, :519) written by
 *     `CSMain` (ShaderCompute.hlsl:291-315);
 *   - Dispatch(32,32,1) (DxCSApp.cpp:524).
 * Every entry point below names the reference call it replaces.
 *
 * Conventions: plain C types only; no exceptions cross the ABI; every
 * function returns RTX_OK (0) or a negative RTX_ERR_* code and then
 * rtx_last_error() (thread-local) describes the failure. A context is bound
 * to one HIP device and is not thread-safe (the reference drives one D3D11
 * immediate context from the UI thread). Framebuffers are linear
 * float4[rows * width], row 0 = image bottom (the reference's DTid.y,
 * ShaderCompute.hlsl:306-307 with the display quad's texcoords,
 * DxCSApp.cpp:297-303).
 */
#ifndef RTX_H_
#define RTX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define RTX_API __attribute__((visibility("default")))
#else
#define RTX_API
#endif

#define RTX_VERSION 145 /* 1.4.5 */
/* ABI notes.
 *  1.4.5: schedule defaults tier1_bar_low 2.0 -> 1.8, promote_low 300 ->
 *         500 (the R = 4 share with the layer grid, S6k-S6l) and
 *         refill_chunk 16 -> 64 (the queue in pixel tiles, S6t-S6u); private
 *         runs (at most 16 slots) also for large scenes and medium shares;
 *         no layout change.
 *  1.4.4: rtx_set_scan_mode (RTX_SCAN_AUTO / RTX_SCAN_LINEAR; a new entry
 *         point, no layout change).
 *  1.4.3: RTX_DEBUG_CULLED_COOP_LANE(q) (the culled coop's per-lane walk);
 *         RTX_ERR_INCOMPLETE's message names which promotion wait fired and
 *         what the server saw (no layout change).
 *  1.4.2: rtx_debug_hit_world_from's start_block RTX_DEBUG_CULLED and
 *         RTX_DEBUG_CULLED_COOP(q) (the culled scan, lane mode and group
 *         coop; no layout change).
 *  1.4.1: rtx_debug_scan_rate (a diagnostic; no layout change).
 *  1.4.0: rtx_schedule.prio_bar1..3 (after prepass_cap_split, before
 *         `reserved`): dynamic lane-mode wave priority; the struct grew by
 *         12 bytes.
 *  1.3.0: rtx_schedule.trace_solo_bar (after promote_big_scene),
 *         trace_group and prepass_cap_split (after refill_chunk): the
 *         struct grew by 12 bytes;
 *         rtx_build_info; RTX_ERR_INCOMPLETE: rtx_sync, rtx_download, rtx_get_stats and
 *         rtx_stats_reset report a render launch that left pixels unwritten
 *         (the promotion service's safety valve fired) instead of returning
 *         the image as if it were complete.
 *  1.2.0: rtx_schedule.promote_big_scene (after promote_large) and
 *         refill_chunk (before `reserved`): the struct grew by 8 bytes.
 *  1.1.0: rtx_schedule_defaults / rtx_set_schedule / rtx_get_schedule (the
 *         chain-RNG schedule, formerly an undocumented environment variable
 *         of the library: the library now reads no environment);
 *         rtx_debug_hit_world_from; rtx_debug_hit_world rejects t_min <= 0.
 *  1.0.x: rtx_set_stream(ctx, NULL) selects HIP's null (legacy default)
 *         stream, which implicitly synchronises with every blocking stream;
 *         the context's own non-blocking stream is rtx_use_own_stream. (The
 *         first 1.0 builds treated NULL as "own stream".) */

enum {
    RTX_OK = 0,
    RTX_ERR_INVALID = -1, /* bad argument (null pointer, size mismatch, ...) */
    RTX_ERR_HIP = -2,     /* a HIP runtime call failed */
    RTX_ERR_STATE = -3,   /* call out of order (no world / no frame yet) */
    RTX_ERR_NOMEM = -4,   /* host or device allocation failed */
    RTX_ERR_INCOMPLETE = -5 /* a render launch since the last check left pixels
                               unwritten (reported once, by the next rtx_sync,
                               rtx_download, rtx_get_stats or rtx_stats_reset) */
};

/* Material type codes, as the reference stores them in WorldDef::matTypes
 * (DxCSApp.cpp:11-17 SetFloat4Cmpt; ShaderCompute.hlsl:209,219,229). */
enum { RTX_MAT_LAMBERT = 0, RTX_MAT_METAL = 1, RTX_MAT_DIELECTRIC = 2 };

/* RNG modes. CHAIN is the reference: ONE fp32 seed per pixel carried through
 * all samples (ShaderCompute.hlsl:295, 304-309). PER_SAMPLE re-seeds every
 * (pixel, sample) so samples are independent of each other (needed to split
 * one pixel's samples across lanes/GPUs); it is an extension, not reference
 * behaviour. */
enum { RTX_RNG_CHAIN = 0, RTX_RNG_PER_SAMPLE = 1 };

/* rtx_frame.flags. RTX_FRAME_LAMBERT_GUARD (an extension):
 * a diffuse scatter direction whose three components are all below 1e-9 in
 * magnitude is replaced by the normal before it is normalised — the guard of
 * the pixel-shader prototype's lambert (Shader_RT.fx:219-225) with the
 * compute shader's own unused near_zero (ShaderCompute.hlsl:70-74). The
 * compute shader has no guard (:209-217) and normalises a zero vector to
 * NaN; 0 keeps that. */
enum { RTX_FRAME_LAMBERT_GUARD = 1 };

/* Scene (~ cbuffer b1 WorldDef, DxCSApp.cpp:64-71). Arrays are read during
 * rtx_upload_world and copied; the caller keeps ownership. Unlike the
 * reference's fixed 512-sphere cbuffer the count is unbounded. */
typedef struct rtx_world {
    uint32_t count;           /* sceneValues.x : number of spheres           */
    uint32_t depth;           /* sceneValues.y : max ray segments per sample */
    uint32_t spp;             /* sceneValues.z : samples per pixel           */
    uint32_t reserved;        /* must be 0                                   */
    const float *spheres;     /* 4*count : center.xyz, radius  (spheres[])   */
    const float *mat_types;   /* count   : RTX_MAT_* as float  (matTypes[])  */
    const float *mat_values;  /* 4*count : albedo.rgb, fuzz-or-ir (matValues[]) */
} rtx_world;

/* Per-frame constants (~ cbuffer b0 PerFrame, DxCSApp.cpp:30-37). The four
 * rows are the reference's viewVals as the shader reads them
 * (ShaderCompute.hlsl:122-123): origin, horizontal, vertical, lower-left. */
typedef struct rtx_frame {
    float origin[4];          /* viewVals[0] */
    float horizontal[4];      /* viewVals[1] */
    float vertical[4];        /* viewVals[2] */
    float lower_left[4];      /* viewVals[3] */
    float img_w;              /* img_dim.x = perspectiveVals.w               (ShaderCompute.hlsl:294) */
    float img_h;              /* img_dim.y = perspectiveVals.w / perspectiveVals.y */
    uint32_t width;           /* framebuffer width in pixels  (texture Width,  DxCSApp.cpp:331) */
    uint32_t height;          /* framebuffer height in pixels (texture Height, DxCSApp.cpp:330) */
    uint32_t rng_mode;        /* RTX_RNG_*; 0 = reference                     */
    uint32_t frame_index;     /* seed offset for progressive frames; 0 = reference (time unused, :296) */
    uint32_t flags;           /* RTX_FRAME_* bits; 0 = reference              */
    uint32_t reserved;        /* must be 0 */
    /* Thin-lens defocus (an extension: the reference's compute
     * shader passes aperture but ignores it, DxCSApp.cpp:179 /
     * ShaderCompute.hlsl:118-127). lens_u/lens_v = camera u/v axes, lens_u[3]
     * = lens radius (aperture/2); 0 = pinhole (reference behaviour). Per
     * sample: rd = radius * random_in_unit_disk (ShaderCompute.hlsl:50-57),
     * offset = u*rd.x + v*rd.y, origin += offset, dir -= offset
     * (Shader_RT.fx:288-298). */
    float lens_u[4];
    float lens_v[4];
} rtx_frame;

/* Counters of the last launches since rtx_stats_reset (measurement, §8d). */
typedef struct rtx_stats {
    double kernel_ms;         /* summed HIP-event duration of the render kernels */
    uint64_t launches;        /* render kernel launches                          */
    uint64_t samples;         /* pixel-samples traced (pixels * spp)             */
    uint64_t segments;        /* hit_world calls (ray segments)                  */
    uint64_t sphere_tests;    /* segments * sphere count (ray-sphere tests)      */
} rtx_stats;

typedef struct rtx_ctx rtx_ctx;

/* ---- library / device ------------------------------------------------- */
RTX_API int rtx_version(void);
/* Build provenance (1.3.0): "src_sha16=<hash of the sources the library was
 * compiled from> arch=gfx950" (static string). */
RTX_API const char *rtx_build_info(void);
/* Thread-local text of the last failure on this thread ("" if none). */
RTX_API const char *rtx_last_error(void);
/* Number of visible HIP devices. */
RTX_API int rtx_device_count(int *count);

/* ---- context lifecycle (~ CDx11Base::Initialize / Terminate) ------------
 * rtx_create replaces D3D11CreateDeviceAndSwapChain (CSVersion/Dx11Base.cpp:75)
 * + the resource creation in LoadContent; rtx_destroy replaces
 * CDx11Base::Terminate -> DxCSApp::UnloadContent (Dx11Base.cpp:134-152,
 * DxCSApp.cpp:420-456). */
RTX_API int rtx_create(int hip_device, rtx_ctx **out);
RTX_API void rtx_destroy(rtx_ctx *ctx);
/* Use an external hipStream_t (e.g. torch's current stream) for every later
 * launch and copy. NULL is HIP's null (legacy default) stream — the handle
 * torch reports for its default stream — so that work orders with the
 * caller's other work on it. */
RTX_API int rtx_set_stream(rtx_ctx *ctx, void *hip_stream);
/* Back to the context's own non-blocking stream (the state after rtx_create). */
RTX_API int rtx_use_own_stream(rtx_ctx *ctx);

/* ---- schedule of the chain-RNG render ------------------
 * The reference's RNG chain makes a pixel's samples sequential, so the render
 * schedules PIXELS: a 2-spp cost pre-pass gives every pixel a cost key (its
 * 3x3 neighbourhood's segments), the persistent render takes pixels most
 * expensive first, and the heaviest are traced by groups of lanes. With
 * share = (sum of the keys) / (resident lanes) and "pixels per lane" = the
 * part's pixels / resident lanes:
 *   - tier 1 (one pixel per wave, 64 lanes per ray): keys above
 *     tier1_bar x share; for a SMALL part (pixels per lane < small_share,
 *     e.g. one rank of an 8-way split) tier1_bar_small, for a LOW part
 *     (< low_share) tier1_bar_low;
 *   - tier 2 (eight pixels per wave): a small part's keys above
 *     tier2_bar_small x share, a MEDIUM part's (< medium_share) above
 *     tier2_bar_medium x share, a larger part's above tier2_bar x share
 *     (tier-2 bars above the tier-1 bar select no tier 2);
 *   - hot_fraction x resident lanes of the normal queue's first slots run at
 *     wave priority hot_priority; tier-1 waves at tier1_priority, tier-2
 *     waves at tier2_priority (s_setprio 0..3: issue arbitration among the
 *     waves of a SIMD);
 *   - occupancy_*: the fraction of the resident waves launched for a small /
 *     low / larger part;
 *   - tail_coop_max: once the queue is empty a wave with at most this many
 *     pixels left traces them with several lanes per ray (1..64);
 *     tail_coop_max_large for scenes above 640 spheres (no LDS copy of the
 *     scene: the group's sphere reads go to L2/HBM);
 *   - trace_*: for scenes up to 640 spheres tier 1 runs in its own kernel
 *     beside the render (one pixel per wave, all 64 lanes on its ray), with
 *     this fraction of the resident waves for a small / low / medium /
 *     larger part (0: tier 1 stays in the render kernel); trace_group
 *     pixels per wave of it (each traced by 64 / trace_group lanes: more
 *     chains for about the same issue, a little longer per segment), except
 *     keys above trace_solo_bar x share, traced one per wave; the kernel also
 *     serves the promotion queue once tier 1 is done;
 *   - promote_*: once the pixel queue is empty, a lane whose pixel is
 *     projected to need more than this many further ray segments hands it
 *     over at a sample boundary to a wave with nothing else to do (an idle
 *     render wave, or the tier-1 kernel), which traces it with all 64 lanes
 *     (0: never); promote_big_scene replaces them for scenes above 640
 *     spheres (no LDS copy: a segment is a long scan there, so a far
 *     shorter remaining chain is worth handing to a whole wave);
 *   - refill_chunk: for a part of at least medium_share pixels per lane (a
 *     whole frame) of a scene up to 1,024 spheres, each wave takes its pixels
 *     from a private run of this many consecutive slots of the cost-ordered
 *     queue (at most 16 for a larger scene or a part of low_share to
 *     medium_share pixels per lane; none below), re-stocked when
 *     empty, so its lanes hold pixels from few runs (coherent rays) rather
 *     than one slot per refill from wherever the queue head is; the last
 *     eighth of the queue is taken slot by slot;
 *   - prio_bar1..3: a lane-mode wave runs at priority 1, 2 or 3 while some
 *     lane's pixel is projected (its segments per sample so far, the cost
 *     pre-pass's included, times the samples left) to need more than
 *     prio_barK x the mean pixel's segments (the pre-pass's estimate), else
 *     at 0: the longest remaining chains get the SIMDs' issue, whatever their
 *     key said; prio_bar1 = 0 selects the static scheme instead (hot_fraction
 *     of the queue's first slots at hot_priority).
 * Results never depend on the schedule (every pixel's operations are the
 * same whichever lanes trace it); only the time does. The defaults are the
 * measured best. A context starts with the defaults. */
typedef struct rtx_schedule {
    float tier1_bar;          /* default 1.7 */
    float tier1_bar_small;    /* default 1.6 */
    float tier1_bar_low;      /* default 1.8 (2.0 before 1.4.5) */
    float tier2_bar_small;    /* default 2.0 */
    float tier2_bar_medium;   /* default 1e30 (none; 1.2 in earlier builds) */
    float tier2_bar;          /* default 1e30 (no tier 2 for a larger part) */
    float small_share;        /* default 1.2 pixels per resident lane */
    float low_share;          /* default 2.5 */
    float medium_share;       /* default 3.5 */
    float hot_fraction;       /* default 0.2 */
    float occupancy_small;    /* default 1.0; each occupancy in (0, 1] */
    float occupancy_low;      /* default 1.0 */
    float occupancy_normal;   /* default 1.0 */
    float trace_small;        /* default 0.35; each trace_* in [0, 0.5] */
    float trace_low;          /* default 0.3 */
    float trace_medium;       /* default 0.15 */
    float trace_large;        /* default 0 */
    float promote_small;      /* default 400; each promote_* in [0, 1e9] */
    float promote_low;        /* default 500 (300 before 1.4.5) */
    float promote_medium;     /* default 400 */
    float promote_large;      /* default 400 */
    float promote_big_scene;  /* default 60: every part of a scene above 640 spheres */
    float trace_solo_bar;     /* default 6: tier-1 keys above this x share are traced one pixel per wave
                                 even when trace_group > 1 */
    uint32_t tail_coop_max;   /* default 32 */
    uint32_t tail_coop_max_large; /* default 8: the same for scenes above 640 spheres */
    uint32_t tier1_priority;  /* default 3 */
    uint32_t tier2_priority;  /* default 2 */
    uint32_t hot_priority;    /* default 3 */
    uint32_t refill_chunk;    /* default 64 (16 before 1.4.5); 0..4096 (0, 1: one refill per need) */
    uint32_t trace_group;     /* default 4: tier-1 pixels per wave of the tier-1 kernel (1, 2, 4 or 8; 8 since 1.4.1) */
    uint32_t prepass_cap_split; /* default 0 (none): a row-split part's cost pre-pass stops a pixel past this
                                   many segments (0..4096); it goes to the top of the queue (tier 1) and the
                                   render traces it from sample 0 */
    float prio_bar1;          /* default 0.5 (0: static hot slots, hot_fraction / hot_priority) */
    float prio_bar2;          /* default 1.0 */
    float prio_bar3;          /* default 1.5 */
    uint32_t reserved;        /* must be 0 */
} rtx_schedule;
/* The library's defaults (no context, no GPU). */
RTX_API int rtx_schedule_defaults(rtx_schedule *out);
/* Validates and installs a schedule for later launches of `ctx` (NULL =
 * the defaults): bars and shares finite and > 0, hot_fraction in [0, 1],
 * occupancies in (0, 1], trace_* in [0, 0.5], promote_* in [0, 1e9],
 * tail_coop_max and tail_coop_max_large in 1..64,
 * priorities in 0..3, refill_chunk in 0..4096, trace_group 1, 2, 4 or 8,
 * trace_solo_bar > 0, prepass_cap_split in 0..4096, prio_bar1 = 0 or
 * 0 < prio_bar1 <= prio_bar2 <= prio_bar3 <= 1e30, reserved 0. */
RTX_API int rtx_set_schedule(rtx_ctx *ctx, const rtx_schedule *schedule);
RTX_API int rtx_get_schedule(rtx_ctx *ctx, rtx_schedule *out);

/* ---- scene / frame upload ----------------------------------------------
 * ~ CreateBuffer(WorldDef, IMMUTABLE) (DxCSApp.cpp:393-413). */
RTX_API int rtx_upload_world(rtx_ctx *ctx, const rtx_world *world);
/* How hit_world finds its candidates (the answer is the reference's in both):
 * RTX_SCAN_AUTO (the default): the flat layer's blocks through the layer grid
 * (scenes up to 1,024 spheres) and the culled scan over a spatially ordered
 * copy (larger scenes); RTX_SCAN_LINEAR: every block of the scene for every
 * ray segment, in Hittable_list order (Hittable_list.cpp:3-20,
 * ShaderCompute.hlsl:194), with the prefilter — large scenes stream it
 * through a per-wave LDS tile of 64 blocks. Takes effect at the next
 * rtx_upload_world. */
enum { RTX_SCAN_AUTO = 0, RTX_SCAN_LINEAR = 1 };
RTX_API int rtx_set_scan_mode(rtx_ctx *ctx, int mode);
/* ~ Map(WRITE_DISCARD)/memcpy/Unmap of PerFrame (DxCSApp.cpp:494-496).
 * Host-side only: constants travel as kernel arguments. */
RTX_API int rtx_set_frame(rtx_ctx *ctx, const rtx_frame *frame);

/* ---- render (~ Dispatch(32,32,1), DxCSApp.cpp:524) ------------------------
 * Renders the rows owned by partition `part` of `nparts`: image rows are
 * cut into tiles of `tile_rows` rows and tile k belongs to part k % nparts
 * (interleaved row tiles). The part's rows are written in
 * ascending order, contiguously, to d_out (device pointer, at least
 * rtx_part_rows(...) * width float4s). d_out == NULL renders into the
 * context's own framebuffer (whole image only: part 0 of 1).
 * Asynchronous on the context stream. */
RTX_API int rtx_render_rows(rtx_ctx *ctx, uint32_t tile_rows, uint32_t part,
                            uint32_t nparts, void *d_out);
/* Whole frame into the context framebuffer (= rtx_render_rows(ctx,1,0,1,NULL)). */
RTX_API int rtx_render(rtx_ctx *ctx);
/* Progressive accumulation (the reference's intended
 * interactive mode: sampleCount/currSamples DxCSApp.cpp:491-492, frame loop
 * CSVersion/main.cpp:51-52, seed hook ShaderCompute.hlsl:296). reset != 0
 * clears the accumulator. Each call renders one frame of spp samples per
 * pixel with frame_index = frames accumulated so far (distinct seeds), adds
 * each pixel's linear sample sum into a float4 accumulator, and writes
 * toGamma(sum / (frames * spp)) into the context framebuffer. */
RTX_API int rtx_accumulate(rtx_ctx *ctx, int reset);
/* Frames accumulated since the last reset. */
RTX_API uint32_t rtx_accumulated_frames(rtx_ctx *ctx);
/* Rows owned by `part` (host arithmetic, no GPU). */
RTX_API uint32_t rtx_part_rows(uint32_t height, uint32_t tile_rows, uint32_t part,
                               uint32_t nparts);
/* Gathered buffer [nparts][max_rows][width] (each part's rows, padded to
 * the largest part) -> image [height][width] in global row order. Device
 * pointers; asynchronous on the context stream. */
RTX_API int rtx_deinterleave_rows(rtx_ctx *ctx, const void *d_gathered,
                                  uint32_t width, uint32_t height,
                                  uint32_t tile_rows, uint32_t nparts,
                                  void *d_image);
/* Wait for all work on the context stream (~ the implicit sync of Present,
 * DxCSApp.cpp:551); RTX_ERR_INCOMPLETE if a launch left pixels unwritten. */
RTX_API int rtx_sync(rtx_ctx *ctx);
/* Device pointer of the context framebuffer (width*height float4) or NULL. */
RTX_API void *rtx_framebuffer(rtx_ctx *ctx);
/* Copy the context framebuffer to host memory (synchronous). The reference
 * never reads results back; this is the image-output contract (§8f-1). */
RTX_API int rtx_download(rtx_ctx *ctx, float *host_rgba, size_t bytes);

/* ---- device buffers (for callers without their own allocator) ----------
 * Ordered on the context stream; copies are synchronous. d_ptr from
 * rtx_alloc may be passed as d_out / d_gathered / d_image above. */
RTX_API int rtx_alloc(rtx_ctx *ctx, size_t bytes, void **d_ptr);
RTX_API int rtx_free(rtx_ctx *ctx, void *d_ptr);
RTX_API int rtx_copy_to_host(rtx_ctx *ctx, void *host, const void *d_src, size_t bytes);
RTX_API int rtx_copy_to_device(rtx_ctx *ctx, void *d_dst, const void *host, size_t bytes);

/* ---- measurement ------------------------------------------------------ */
RTX_API int rtx_stats_reset(rtx_ctx *ctx);
/* Synchronises the stream, then reports counters since the last reset. */
RTX_API int rtx_get_stats(rtx_ctx *ctx, rtx_stats *out);

/* ---- host-side producers (no GPU) ----------------------------------------
 * WorldDef::random_world (DxCSApp.cpp:72-134) with MSVC rand() (unseeded,
 * DxCSApp.cpp:6-9) emulated bit-exactly. grid_half_extent 9 = reference
 * (326 spheres), 11 = RTIOW final scene (486). At most `capacity` spheres
 * are written (the generator stops there); *count receives the number
 * written. Arrays: spheres 4*capacity, mat_types capacity, mat_values
 * 4*capacity. */
RTX_API int rtx_scene_random_world(int32_t grid_half_extent, uint32_t capacity,
                                   float *spheres, float *mat_types,
                                   float *mat_values, uint32_t *count);
/* WorldDef::test_world (DxCSApp.cpp:136-157): 4 spheres. */
RTX_API int rtx_scene_test_world(float *spheres, float *mat_types,
                                 float *mat_values, uint32_t *count);
/* The pixel-shader prototype's scene (Shader_RT.fx:300-335): 7 spheres
 * (ground, 3 small Lambert, glass, Lambert, metal); arrays of capacity 7. */
RTX_API int rtx_scene_ps_world(float *spheres, float *mat_types,
                               float *mat_values, uint32_t *count);
/* PerFrame::ComputeViewVals (DxCSApp.cpp:39-61) + the focus distance of
 * DxCSApp::Update (DxCSApp.cpp:488) with focus_dist <= 0 meaning
 * |from - at|. Fills the four view rows, img_w = width_px,
 * img_h = width_px / aspect (ShaderCompute.hlsl:294) and width/height. */
RTX_API int rtx_camera_look_at(const float from[3], const float at[3],
                               const float vup[3], float vfov_deg, float aspect,
                               float aperture, float focus_dist,
                               uint32_t width_px, uint32_t height_px,
                               rtx_frame *out);
/* Enable thin-lens defocus on a frame from rtx_camera_look_at: lens
 * radius = aperture / 2 (focus distance is already in the frame rows). */
RTX_API int rtx_camera_set_aperture(rtx_frame *frame, float aperture);
/* Camera(width, height) of the CPU library (Camera.h:9-21). */
RTX_API int rtx_camera_simple(uint32_t width_px, uint32_t height_px, rtx_frame *out);
/* Adapters from the reference's exact cbuffer byte layouts: WorldDef
 * (18,448 B, DxCSApp.cpp:64-71) and PerFrame (112 B, DxCSApp.cpp:30-37,
 * viewVals stored transposed, :60). The world adapter writes into
 * caller arrays of capacity 512 like rtx_scene_random_world. */
RTX_API int rtx_world_from_worlddef(const void *worlddef_bytes, size_t nbytes,
                                    float *spheres, float *mat_types,
                                    float *mat_values, rtx_world *out);
RTX_API int rtx_frame_from_perframe(const void *perframe_bytes, size_t nbytes,
                                    uint32_t width_px, uint32_t height_px,
                                    rtx_frame *out);

/* ---- debug entry points: the hot-path building blocks run on the GPU ----
 * (used by the parity tests; same device code as the render kernel).
 * rays: nrays * 6 floats (origin.xyz, dir.xyz) host memory. out: nrays * 10
 * floats: hit(0/1), t, p.xyz, normal.xyz, front_face(0/1), sphere index.
 * Uses the uploaded world. Synchronous. ~ hit_world, ShaderCompute.hlsl:188-205. */
RTX_API int rtx_debug_hit_world(rtx_ctx *ctx, const float *rays, uint32_t nrays,
                                float t_min, float t_max, float *out);
/* Requirements of both: t_min finite and > 0 (the render's 0.001; the
 * kernel orders candidate roots by their bit patterns, which order like the
 * values only for positive roots), t_max not NaN. t_max < t_min: no ray
 * hits (no root lies in [t_min, t_max]).
 * rtx_debug_hit_world_from: the same, with the prefiltered scan starting at
 * 8-sphere block start_block % ceil(count / 8) and wrapping round — the
 * start the large-scene kernels take from their workgroup's position word
 * (DESIGN.md §3 "pack start"); the result is the in-order scan's for every
 * start (ties between spheres on either side of the wrap included).
 * start_block = RTX_DEBUG_CULLED: for a world of more than 1,024 spheres
 * (after padding to 8), the culled scan the render's lane mode runs on such
 * scenes (a spatially ordered copy of the spheres whose 8-sphere blocks are
 * skipped when no lane's line passes their bounding sphere, DESIGN.md §3e
 * "culled scan"); smaller worlds scan from block
 * RTX_DEBUG_CULLED % ceil(count / 8) as above. */
#define RTX_DEBUG_CULLED 0xFFFFFFFFu
/* start_block = RTX_DEBUG_CULLED_COOP(q), q in 1..64, for the same worlds:
 * the culled scan split over a wave's lanes as the render's frame tail and
 * heavy tiers run it, q rays per wave (64 / 2^ceil(log2 q) lanes per ray). */
#define RTX_DEBUG_CULLED_COOP(q) (0xFFFFFF00u | (unsigned)(q))
/* start_block = RTX_DEBUG_CULLED_COOP_LANE(q): the same split with each lane
 * walking its own subtree (the per-sample kernel's form; RTX_DEBUG_CULLED_COOP
 * walks one ray's levels breadth first). */
#define RTX_DEBUG_CULLED_COOP_LANE(q) (0xFFFFFE00u | (unsigned)(q))
RTX_API int rtx_debug_hit_world_from(rtx_ctx *ctx, const float *rays, uint32_t nrays,
                                     float t_min, float t_max, uint32_t start_block,
                                     float *out);
/* Evaluates device math function `fn` (RTX_FN_*) elementwise on host
 * arrays (in0, in1 may be unused); out receives n floats (hash functions
 * write 1, 2 or 3 floats per element: out must hold 3*n). The diffuse
 * direction functions take n cases: in0 = p[3n], in1 = (normal, rius)[6n],
 * out = normalize(((p + normal) + rius) - p)[3n] (ShaderCompute.hlsl:
 * 211-212), unguarded or with RTX_FRAME_LAMBERT_GUARD. Synchronous. */
enum {
    RTX_FN_SQRT = 0, RTX_FN_DIV = 1, RTX_FN_SIN = 2, RTX_FN_COS = 3,
    RTX_FN_LOG2 = 4, RTX_FN_EXP2 = 5, RTX_FN_POW = 6, RTX_FN_BASEHASH = 7,
    RTX_FN_HASH1 = 8, RTX_FN_HASH2 = 9, RTX_FN_HASH3 = 10, RTX_FN_RIUS = 11,
    RTX_FN_LAMBERT_DIR = 12, RTX_FN_LAMBERT_DIR_GUARD = 13
};
RTX_API int rtx_debug_math(rtx_ctx *ctx, int fn, const float *in0,
                           const float *in1, uint32_t n, float *out);
/* Wave timeline diagnostic: a call with a new max_waves (> 0) arms
 * recording of every render wave's (start, end) s_memrealtime (100 MHz)
 * into a device buffer of that many waves (0 disarms); a call with the same
 * max_waves and host_pairs != NULL copies the pairs back (synchronous). */
RTX_API int rtx_debug_wave_times(rtx_ctx *ctx, size_t max_waves, unsigned long long *host_pairs);
/* Per-pixel cost diagnostic: traces the whole current frame with `spp`
 * samples per pixel (0 = the world's spp), one lane per pixel, and writes
 * each pixel's ray-segment count (hit_world calls) into host_cost
 * (width * height uint32, row 0 = image bottom). Does not touch the
 * framebuffer or the stats. Synchronous. */
RTX_API int rtx_debug_pixel_cost(rtx_ctx *ctx, uint32_t spp, uint32_t *host_cost);
/* Issue-rate probe of hit_world's instruction mix (ABI 1.4.1): a
 * full-occupancy grid shaped like the render (same workgroups, register
 * budget and LDS) in which every lane runs the render's lane-mode hit_world
 * (prefiltered scan + resolve, ShaderCompute.hlsl:188-205) `reps` times on
 * one primary ray of the current frame, and nothing else. *ms: the launch's
 * HIP-event time; *wave_segments: waves x reps (one wave-segment = 64 ray
 * segments' hit_world). A profiler's SQ_INSTS_VALU over this launch gives
 * the VALU issue rate the scan-and-resolve mix sustains on its own — the
 * ceiling for the render's hit_world section. Scenes up to 640 spheres (the
 * render's LDS-copy scenes); needs a world and a frame. Synchronous. */
RTX_API int rtx_debug_scan_rate(rtx_ctx *ctx, uint32_t reps, float *ms, unsigned long long *wave_segments);

#ifdef __cplusplus
}
#endif
#endif /* RTX_H_ */
