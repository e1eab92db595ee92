/*
 * rtx_oracle.h — CPU oracle for the path-tracing hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so, and only as the checker / the timed CPU baseline.
 *
 * Two restatements of the reference algorithm:
 *   - fp32 "twin": the op-for-op restatement of the HIP kernel's arithmetic
 *     spec, itself following CSVersion/ShaderCompute.hlsl and
 *     Sphere.cpp / Hittable_list.cpp / Camera.h. GPU output must equal it
 *     bit for bit.
 *   - fp64 "reference geometry": Sphere::hit / Hittable_list::hit /
 *     Camera::get_ray exactly as the reference's double-precision CPU
 *     library computes them (Sphere.cpp:3-32, Hittable_list.cpp:3-20,
 *     Camera.h:9-26, Vec3.h, Ray.h, Hittable.h). Pinned against golden
 *     vectors produced by compiling those reference files (oracle/_ref).
 * Struct layouts equal include/rtx.h's rtx_world / rtx_frame.
 */
#ifndef RTX_ORACLE_H_
#define RTX_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_world {
    uint32_t count, depth, spp, reserved;
    const float *spheres;    /* 4*count: center.xyz, radius */
    const float *mat_types;  /* count */
    const float *mat_values; /* 4*count */
} or_world;

typedef struct or_frame {
    float origin[4], horizontal[4], vertical[4], lower_left[4];
    float img_w, img_h;
    uint32_t width, height, rng_mode, frame_index, flags, reserved; /* flags: RTX_FRAME_* */
    float lens_u[4], lens_v[4]; /* thin lens: axes, lens_u[3] = radius (0 = pinhole) */
} or_frame;

/* Render the listed global image rows (ys[0..nys)) into out
 * (nys * width * 4 floats, row order of ys). precision 32 = fp32 twin,
 * 64 = fp64 geometry/shading with the same fp32 RNG chain. nthreads >= 1.
 * *segments (optional) receives the number of hit_world calls. */
int or_render_rows(const or_world *w, const or_frame *f, const uint32_t *ys, uint32_t nys,
                   float *out, int nthreads, int precision, uint64_t *segments);
/* As or_render_rows (precision 32) but out receives each pixel's LINEAR
 * sample sum (accColor before /spp and toGamma), w = 1: the per-frame
 * contribution of progressive accumulation (rtx_accumulate). */
int or_render_rows_linear(const or_world *w, const or_frame *f, const uint32_t *ys, uint32_t nys,
                          float *out, int nthreads, uint64_t *segments);

/* hit_world for a batch of rays (6 floats / 6 doubles each). out: 10 per
 * ray: hit, t, p.xyz, normal.xyz, front_face, index (same as
 * rtx_debug_hit_world). */
int or_hit_world_f32(const or_world *w, const float *rays, uint32_t n, float t_min, float t_max,
                     float *out);
int or_hit_world_f64(const double *spheres /* 4*count */, uint32_t count, const double *rays,
                     uint32_t n, double t_min, double t_max, double *out);
/* Camera(width, height).get_ray(u, v) in double (Camera.h:9-26). out: 6 per (u,v). */
int or_camera_simple_rays_f64(uint32_t width, uint32_t height, const double *uv, uint32_t n,
                              double *out);

/* Elementwise math of the twin spec; fn codes = RTX_FN_* of include/rtx.h
 * (12/13, the diffuse direction: in0 = p[3n], in1 = (normal, rius)[6n]). */
int or_math(int fn, const float *in0, const float *in1, uint32_t n, float *out);
uint32_t or_base_hash(uint32_t x, uint32_t y);

/* Scene and camera producers (DxCSApp.cpp:39-61, 72-157; Camera.h:9-21). */
int or_random_world(int32_t ext, uint32_t capacity, float *spheres, float *mat_types,
                    float *mat_values, uint32_t *count);
int or_test_world(float *spheres, float *mat_types, float *mat_values, uint32_t *count);
int or_camera_look_at(const float from[3], const float at[3], const float vup[3], float vfov,
                      float aspect, float focus_dist, uint32_t width, uint32_t height,
                      or_frame *out);
int or_camera_simple(uint32_t width, uint32_t height, or_frame *out);

#ifdef __cplusplus
}
#endif
#endif
