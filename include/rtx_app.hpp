// rtx_app.hpp — C++ host surface mirroring the reference's app plug-in
// interface, driven through the rtx C-ABI instead of D3D11.
//
//   RtxBase   ~ CDx11Base (CSVersion/Dx11Base.h:11-40): Initialize /
//               Terminate + pure virtual LoadContent / UnloadContent /
//               Update / Render.
//   RtxCSApp  ~ DxCSApp  (CSVersion/DxCSApp.h:12-60, DxCSApp.cpp:160-552):
//               LoadContent builds WorldDef::random_world and uploads it
//               (DxCSApp.cpp:199-418); Update computes PerFrame's camera
//               (:458-497); Render launches the path tracer (:499-552).
// Errors: bool returns like the reference (false + rtx_last_error()).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "rtx.h"

namespace rtx {

class RtxBase {
public:
    RtxBase() = default;
    virtual ~RtxBase();
    RtxBase(const RtxBase &) = delete;
    RtxBase &operator=(const RtxBase &) = delete;

    // ~ CDx11Base::Initialize(HWND, HINSTANCE) (CSVersion/Dx11Base.cpp:23-132):
    // creates the device context, then calls LoadContent.
    bool Initialize(int hip_device);
    // ~ CDx11Base::Terminate (CSVersion/Dx11Base.cpp:134-152).
    void Terminate();

    virtual bool LoadContent() = 0;
    virtual void UnloadContent() = 0;
    virtual void Update() = 0;
    virtual void Render() = 0;

    rtx_ctx *context() const { return m_ctx; }
    const std::string &last_error() const { return m_error; }

protected:
    rtx_ctx *m_ctx = nullptr;
    std::string m_error;
};

enum class SceneKind { RandomWorld, TestWorld, PsWorld };

struct AppConfig {
    uint32_t width = 1024, height = 576;   // texture size, DxCSApp.cpp:330-331
    uint32_t spp = 60, depth = 50;         // sceneValues, DxCSApp.cpp:133
    SceneKind scene = SceneKind::RandomWorld;
    int32_t grid_half_extent = 9;          // random_world grid, DxCSApp.cpp:95-97
    uint32_t max_spheres = 0;              // 0 = no cap
    float cam_pos[3] = {13.0f, 2.0f, 3.0f};   // DxCSApp.cpp:176
    float cam_look_at[3] = {0.0f, 0.0f, 0.0f};
    float up[3] = {0.0f, 1.0f, 0.0f};
    float vfov = 20.0f;                    // perspectiveVals, DxCSApp.cpp:179
    float aspect = 16.0f / 9.0f;
    float aperture = 2.0f;
    bool simple_camera = false;            // Camera.h instead of ComputeViewVals
    float lens_aperture = 0.0f;            // > 0: thin lens (extension, §8f-3); 0 = reference pinhole
    uint32_t rng_mode = RTX_RNG_CHAIN;
    bool lambert_guard = false;            // RTX_FRAME_LAMBERT_GUARD (extension, §8f-4); false = reference
    // Drive the library through the reference's own cbuffer bytes: LoadContent
    // fills a WorldDef (random_world, at most 512 spheres) and hands it to
    // rtx_world_from_worlddef; Update fills a PerFrame and hands it to
    // rtx_frame_from_perframe — DxCSApp's data path byte for byte.
    bool cbuffers = false;
};

// The reference's constant-buffer byte layouts (HLSL packing: float4 rows).
// WorldDef, DxCSApp.cpp:64-71: sceneValues {count, depth, spp, -1};
// spheres[512] (centre, radius); matTypes[128], four codes per float4
// (SetFloat4Cmpt, :11-17); matValues[512].
struct WorldDefBytes {
    float scene_values[4];
    float spheres[512][4];
    float mat_types[128][4];
    float mat_values[512][4];
};
static_assert(sizeof(WorldDefBytes) == 18448, "WorldDef is 18,448 bytes");
// PerFrame, DxCSApp.cpp:30-37: time, perspectiveVals {vfov, aspect,
// aperture, width}, currSamples, viewVals (4x4, stored transposed, :60).
struct PerFrameBytes {
    float time[4];
    float perspective_vals[4];
    float curr_samples[4];
    float view_vals[16];
};
static_assert(sizeof(PerFrameBytes) == 112, "PerFrame is 112 bytes");
// WorldDef::random_world into the cbuffer layout (DxCSApp.cpp:72-134); false
// if the scene does not fit its 512 slots.
bool fill_worlddef(const AppConfig &cfg, WorldDefBytes &out);
// DxCSApp::Update's PerFrame (DxCSApp.cpp:481-492): perspectiveVals,
// ComputeViewVals with focus_dist = |camPos - camLookAt|, currSamples.
bool fill_perframe(const AppConfig &cfg, float sample_count, PerFrameBytes &out);

class RtxCSApp : public RtxBase {
public:
    explicit RtxCSApp(const AppConfig &cfg = AppConfig());
    ~RtxCSApp() override;

    bool LoadContent() override;
    void UnloadContent() override;
    void Update() override;
    void Render() override;

    // Image output contract (§8f-1): the framebuffer, row 0 = image bottom.
    bool Download(std::vector<float> &rgba);
    const AppConfig &config() const { return m_cfg; }
    uint32_t sphere_count() const { return m_count; }
    bool ok() const { return m_ok; }

private:
    AppConfig m_cfg;
    std::vector<float> m_spheres, m_mat_types, m_mat_values;
    uint32_t m_count = 0;
    rtx_frame m_frame{};
    uint32_t m_frame_count = 0;  // ~ sampleCount, DxCSApp.cpp:491
    bool m_ok = true;
};

// PFM (float RGB, rows stored bottom-to-top = our row order) and binary
// PPM (8-bit, top-to-bottom: rows flipped, values clamped to [0,1]).
bool write_pfm(const std::string &path, const float *rgba, uint32_t w, uint32_t h);
bool write_ppm(const std::string &path, const float *rgba, uint32_t w, uint32_t h);

}  // namespace rtx
