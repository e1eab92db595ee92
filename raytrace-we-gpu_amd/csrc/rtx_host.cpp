// rtx_host.cpp — host-side producers of the reference's GPU inputs
// (no GPU calls): the WorldDef scene builders and the PerFrame camera of
// CSVersion/DxCSApp.cpp, plus adapters from the reference's exact cbuffer
// byte layouts.
#include <cmath>
#include <cstring>

#include "../../include/rtx.h"

namespace {

// MSVC CRT rand(): 32-bit LCG, state starts at 1 when never seeded
// (DxCSApp.cpp:6-9 calls rand() without srand). RAND_MAX = 32767.
struct MsvcRand {
    uint32_t state = 1u;
    int next() {
        state = state * 214013u + 2531011u;
        return (int)((state >> 16) & 0x7fffu);
    }
    // random(): static_cast<float>(rand()) / static_cast<float>(RAND_MAX)
    float random() { return (float)next() / 32767.0f; }
};

struct Writer {
    float *sph, *mt, *mv;
    uint32_t cap, count = 0;
    bool put(float cx, float cy, float cz, float r, float type, float a0, float a1, float a2,
             float a3) {
        if (count >= cap) return false;
        sph[4 * count + 0] = cx;
        sph[4 * count + 1] = cy;
        sph[4 * count + 2] = cz;
        sph[4 * count + 3] = r;
        mt[count] = type;
        mv[4 * count + 0] = a0;
        mv[4 * count + 1] = a1;
        mv[4 * count + 2] = a2;
        mv[4 * count + 3] = a3;
        ++count;
        return true;
    }
};

// XMVector3Normalize / XMVector3Cross / length in fp32 (XNAMath SSE order:
// ((x*x + y*y) + z*z), V / sqrt(.)).
struct V3 {
    float x, y, z;
};
V3 sub(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
V3 scale(V3 a, float s) { return V3{a.x * s, a.y * s, a.z * s}; }
float len3(V3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
V3 norm3(V3 a) {
    const float l = len3(a);
    return V3{a.x / l, a.y / l, a.z / l};
}
V3 cross3(V3 a, V3 b) {
    return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

void set_row(float r[4], V3 v, float w) {
    r[0] = v.x;
    r[1] = v.y;
    r[2] = v.z;
    r[3] = w;
}

}  // namespace

extern "C" {

// WorldDef::random_world, DxCSApp.cpp:72-134.
int rtx_scene_random_world(int32_t ext, uint32_t capacity, float *spheres, float *mat_types,
                           float *mat_values, uint32_t *count) {
    if (!spheres || !mat_types || !mat_values || !count || ext < 0) return RTX_ERR_INVALID;
    Writer w{spheres, mat_types, mat_values, capacity};
    MsvcRand rng;
    // Four fixed spheres (:74-93).
    w.put(0.0f, -1000.0f, 0.0f, 1000.0f, 0.0f, 0.5f, 0.5f, 0.5f, 1.0f);
    w.put(0.0f, 1.0f, 0.0f, 1.0f, 2.0f, 0.0f, 0.0f, 0.0f, 1.5f);
    w.put(-4.0f, 1.0f, 0.0f, 1.0f, 0.0f, 0.4f, 0.2f, 0.1f, 1.0f);
    w.put(4.0f, 1.0f, 0.0f, 1.0f, 1.0f, 0.7f, 0.6f, 0.5f, 0.0f);
    for (int a = -ext; a < ext && w.count < capacity; ++a) {
        for (int b = -ext; b < ext && w.count < capacity; ++b) {
            const float mat_choice = rng.random();
            // { a + 0.9*random(), 0.2, b + 0.9*random() }: double arithmetic,
            // braced-init evaluates left to right, stored as float.
            const float cx = (float)((double)a + 0.9 * (double)rng.random());
            const float cz = (float)((double)b + 0.9 * (double)rng.random());
            const float cy = 0.2f;
            // XMVector3Length(center - ref) > 0.9 (:103); no center lies
            // within 1.5e-2 of the cut, so fp32 vs fp64 cannot matter.
            const double dx = (double)cx - 4.0, dy = (double)cy - 0.2f, dz = (double)cz;
            if (std::sqrt(dx * dx + dy * dy + dz * dz) > 0.9) {
                if ((double)mat_choice < 0.8) {  // Diffuse: albedo random()*random() (:110)
                    const float r0 = rng.random(), r1 = rng.random();
                    const float g0 = rng.random(), g1 = rng.random();
                    const float b0 = rng.random(), b1 = rng.random();
                    w.put(cx, cy, cz, 0.2f, 0.0f, r0 * r1, g0 * g1, b0 * b1, 0.0f);
                } else if ((double)mat_choice < 0.95) {  // Metal: random()/2 + 1, fuzz 0 (:118)
                    const float r = rng.random() / 2.0f + 1.0f;
                    const float g = rng.random() / 2.0f + 1.0f;
                    const float bb = rng.random() / 2.0f + 1.0f;
                    w.put(cx, cy, cz, 0.2f, 1.0f, r, g, bb, 0.0f);
                } else {  // Glass ir 1.5 (:126)
                    w.put(cx, cy, cz, 0.2f, 2.0f, 0.0f, 0.0f, 0.0f, 1.5f);
                }
            }
        }
    }
    *count = w.count;
    return RTX_OK;
}

// WorldDef::test_world, DxCSApp.cpp:136-157.
int rtx_scene_test_world(float *spheres, float *mat_types, float *mat_values, uint32_t *count) {
    if (!spheres || !mat_types || !mat_values || !count) return RTX_ERR_INVALID;
    Writer w{spheres, mat_types, mat_values, 4};
    w.put(0.0f, -1000.5f, -1.0f, 1000.0f, 0.0f, 0.5f, 0.5f, 0.5f, 1.0f);
    w.put(0.0f, 0.0f, -1.0f, 0.5f, 0.0f, 0.2f, 0.4f, 0.8f, 1.0f);
    w.put(1.0f, 0.0f, -1.0f, 0.5f, 1.0f, 0.8f, 0.4f, 0.2f, 0.0f);
    w.put(-1.0f, 0.0f, -1.0f, 0.5f, 2.0f, 0.5f, 0.5f, 0.5f, 1.5f);
    *count = w.count;
    return RTX_OK;
}

// The pixel-shader prototype's scene (Shader_RT.fx:300-335, its
// random_world, whose loop was never finished: ":310 TODO: debug why loops +
// randoms don't work"): the ground, three small Lambert spheres and the
// three big ones. Materials in this library's encoding (mat_values .w =
// fuzz or ir; the prototype's -1 placeholders kept where unused). Rendered
// with the compute shader's material semantics (the prototype's own
// hemisphere sampling and by-value RNG are out of scope).
int rtx_scene_ps_world(float *spheres, float *mat_types, float *mat_values, uint32_t *count) {
    if (!spheres || !mat_types || !mat_values || !count) return RTX_ERR_INVALID;
    Writer w{spheres, mat_types, mat_values, 7};
    w.put(0.0f, -1000.0f, 0.0f, 1000.0f, 0.0f, 0.5f, 0.5f, 0.5f, -1.0f);  // :306 AddLambert
    w.put(3.0f, 0.2f, 1.5f, 0.2f, 0.0f, 0.2f, 0.2f, 0.8f, -1.0f);         // :311
    w.put(4.5f, 0.2f, 1.0f, 0.2f, 0.0f, 0.2f, 0.8f, 0.2f, -1.0f);         // :315
    w.put(4.5f, 0.2f, 2.0f, 0.2f, 0.0f, 0.8f, 0.3f, 0.2f, -1.0f);         // :319
    w.put(0.0f, 1.0f, 0.0f, 1.0f, 2.0f, 1.0f, 1.0f, 1.0f, 1.5f);          // :323 AddDielectric
    w.put(-4.0f, 1.0f, 0.0f, 1.0f, 0.0f, 0.4f, 0.2f, 0.1f, -1.0f);        // :326
    w.put(4.0f, 1.0f, 0.0f, 1.0f, 1.0f, 0.7f, 0.6f, 0.5f, 0.0f);          // :329 AddMetal, fuzz 0
    *count = w.count;
    return RTX_OK;
}

// PerFrame::ComputeViewVals (DxCSApp.cpp:39-61) with the focus distance of
// DxCSApp::Update (:488). The aperture is passed but unused, as in the
// reference (:179; get_ray ignores it, ShaderCompute.hlsl:118-127).
int rtx_camera_look_at(const float from[3], const float at[3], const float vup[3], float vfov,
                       float aspect, float aperture, float focus_dist, uint32_t width_px,
                       uint32_t height_px, rtx_frame *out) {
    (void)aperture;
    if (!from || !at || !vup || !out || width_px == 0 || height_px == 0 || !(aspect > 0.0f))
        return RTX_ERR_INVALID;
    const V3 f{from[0], from[1], from[2]}, a{at[0], at[1], at[2]}, up{vup[0], vup[1], vup[2]};
    if (!(focus_dist > 0.0f)) focus_dist = len3(sub(f, a));  // XMVector4Length(camPos - camLookAt)
    // deg2rad: deg * pi / 180.0 in double, returned as float (:19-22).
    const float theta = (float)((double)vfov * 3.1415926535897932385 / 180.0);
    const float h = std::tan(theta / 2.0f);
    const float view_h = (float)(2.0 * (double)h);
    const float view_w = aspect * view_h;
    const V3 w = norm3(sub(f, a));
    const V3 u = norm3(cross3(up, w));
    const V3 v = cross3(w, u);
    const V3 horizontal = scale(u, focus_dist * view_w);
    const V3 vertical = scale(v, focus_dist * view_h);
    const V3 llc = sub(sub(sub(f, scale(horizontal, 0.5f)), scale(vertical, 0.5f)), scale(w, focus_dist));
    std::memset(out, 0, sizeof(*out));
    set_row(out->origin, f, 1.0f);
    set_row(out->horizontal, horizontal, 0.0f);
    set_row(out->vertical, vertical, 0.0f);
    set_row(out->lower_left, llc, 1.0f);
    set_row(out->lens_u, u, 0.0f);  // lens radius 0: pinhole, as the reference shader
    set_row(out->lens_v, v, 0.0f);
    out->img_w = (float)width_px;              // perspectiveVals.w
    out->img_h = (float)width_px / aspect;     // perspectiveVals.w / perspectiveVals.y
    out->width = width_px;
    out->height = height_px;
    return RTX_OK;
}

// Camera(width, height) of the CPU library (Camera.h:9-21), in double,
// rounded to float: origin 0, horizontal (2*aspect,0,0), vertical (0,2,0),
// lower_left = origin - H/2 - V/2 - (0,0,1).
int rtx_camera_simple(uint32_t width_px, uint32_t height_px, rtx_frame *out) {
    if (!out || width_px == 0 || height_px == 0) return RTX_ERR_INVALID;
    const double aspect = (double)width_px / height_px;
    const double vh = 2.0, vw = aspect * vh;
    std::memset(out, 0, sizeof(*out));
    out->origin[3] = 1.0f;
    out->horizontal[0] = (float)vw;
    out->vertical[1] = (float)vh;
    out->lower_left[0] = (float)(0.0 - vw / 2);
    out->lower_left[1] = (float)(0.0 - vh / 2);
    out->lower_left[2] = (float)(0.0 - 1.0);
    out->lower_left[3] = 1.0f;
    out->lens_u[0] = 1.0f;  // Camera.h basis: u = +x, v = +y, pinhole
    out->lens_v[1] = 1.0f;
    out->img_w = (float)width_px;
    out->img_h = (float)height_px;
    out->width = width_px;
    out->height = height_px;
    return RTX_OK;
}

int rtx_camera_set_aperture(rtx_frame *frame, float aperture) {
    if (!frame || !(aperture >= 0.0f)) return RTX_ERR_INVALID;
    frame->lens_u[3] = aperture / 2.0f;  // f4w.w = aperture / 2 (DXRayTrace.cpp:52-57)
    return RTX_OK;
}

// WorldDef byte layout (DxCSApp.cpp:64-71): float4 sceneValues;
// float4 spheres[512]; float4 matTypes[128] (4 per float4,
// SetFloat4Cmpt :11-17); float4 matValues[512] = 18,448 bytes.
int rtx_world_from_worlddef(const void *bytes, size_t nbytes, float *spheres, float *mat_types,
                            float *mat_values, rtx_world *out) {
    if (!bytes || !spheres || !mat_types || !mat_values || !out) return RTX_ERR_INVALID;
    if (nbytes != 18448) return RTX_ERR_INVALID;
    const float *f = static_cast<const float *>(bytes);
    const float cnt = f[0], depth = f[1], spp = f[2];
    if (!(cnt >= 0.0f && cnt <= 512.0f) || !(depth >= 0.0f) || !(spp >= 0.0f)) return RTX_ERR_INVALID;
    // The shader loops `for (int i = 0; i < sceneValues.x; ++i)` (:194).
    const uint32_t n = (uint32_t)std::ceil(cnt);
    const float *sph = f + 4;
    const float *mt = f + 4 + 4 * 512;
    const float *mv = f + 4 + 4 * 512 + 4 * 128;
    for (uint32_t i = 0; i < n; ++i) {
        for (int k = 0; k < 4; ++k) {
            spheres[4 * i + k] = sph[4 * i + k];
            mat_values[4 * i + k] = mv[4 * i + k];
        }
        mat_types[i] = mt[i];  // matTypes[i/4][i%4] == flat index i
    }
    std::memset(out, 0, sizeof(*out));
    out->count = n;
    out->depth = (uint32_t)std::ceil(depth);
    out->spp = (uint32_t)std::ceil(spp);
    out->spheres = spheres;
    out->mat_types = mat_types;
    out->mat_values = mat_values;
    return RTX_OK;
}

// PerFrame byte layout (DxCSApp.cpp:30-37): float4 time; float4
// perspectiveVals {vfov, aspect, aperture, width}; float4 currSamples;
// XMMATRIX viewVals stored transposed (:60) = 112 bytes.
int rtx_frame_from_perframe(const void *bytes, size_t nbytes, uint32_t width_px, uint32_t height_px,
                            rtx_frame *out) {
    if (!bytes || !out || nbytes != 112 || width_px == 0 || height_px == 0) return RTX_ERR_INVALID;
    const float *f = static_cast<const float *>(bytes);
    const float *persp = f + 4;
    const float *m = f + 12;  // m[4*j + i] = viewVals^T row j comp i = row i comp j
    std::memset(out, 0, sizeof(*out));
    float *rows[4] = {out->origin, out->horizontal, out->vertical, out->lower_left};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) rows[i][j] = m[4 * j + i];
    out->img_w = persp[3];
    out->img_h = persp[3] / persp[1];
    out->width = width_px;
    out->height = height_px;
    return RTX_OK;
}

}  // extern "C"
