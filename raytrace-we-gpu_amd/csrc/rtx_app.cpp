// rtx_app.cpp — RtxBase / RtxCSApp: the reference's CDx11Base / DxCSApp
// entry-point surface (LoadContent / Update / Render / UnloadContent) over
// the rtx C-ABI. See include/rtx_app.hpp.
#include "../../include/rtx_app.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>

namespace rtx {

// Derived classes call Terminate() in their own destructor (UnloadContent
// is virtual); the base only releases a context still held.
RtxBase::~RtxBase() {
    if (m_ctx) rtx_destroy(m_ctx);
}

bool RtxBase::Initialize(int hip_device) {
    if (m_ctx) return true;
    if (rtx_create(hip_device, &m_ctx) != RTX_OK) {
        m_error = rtx_last_error();
        m_ctx = nullptr;
        return false;
    }
    return LoadContent();
}

void RtxBase::Terminate() {
    if (!m_ctx) return;
    UnloadContent();
    rtx_destroy(m_ctx);
    m_ctx = nullptr;
}

RtxCSApp::RtxCSApp(const AppConfig &cfg) : m_cfg(cfg) {}

bool fill_worlddef(const AppConfig &cfg, WorldDefBytes &out) {
    std::memset(&out, 0, sizeof(out));
    float sph[4 * 512], mt[512], mv[4 * 512];
    uint32_t n = 0;
    if (rtx_scene_random_world(cfg.grid_half_extent, 512, sph, mt, mv, &n) != RTX_OK) return false;
    const uint64_t full = 4ull + 4ull * (uint64_t)cfg.grid_half_extent * cfg.grid_half_extent;
    if (full > 512) return false;  // the cbuffer holds 512 spheres (DxCSApp.cpp:67)
    for (uint32_t i = 0; i < n; ++i) {
        for (int k = 0; k < 4; ++k) {
            out.spheres[i][k] = sph[4 * i + k];
            out.mat_values[i][k] = mv[4 * i + k];
        }
        out.mat_types[i / 4][i % 4] = mt[i];  // SetFloat4Cmpt(matTypes[i/4], i%4, .)
    }
    out.scene_values[0] = (float)n;  // { count, 50, 60, -1 } (:133)
    out.scene_values[1] = (float)cfg.depth;
    out.scene_values[2] = (float)cfg.spp;
    out.scene_values[3] = -1.0f;
    return true;
}

bool fill_perframe(const AppConfig &cfg, float sample_count, PerFrameBytes &out) {
    std::memset(&out, 0, sizeof(out));
    const float persp[4] = {cfg.vfov, cfg.aspect, cfg.aperture, (float)cfg.width};  // :179
    rtx_frame f{};
    // ComputeViewVals(camPos, camLookAt, upDir, vfov, aspect, aperture, focus_dist) (:488-489)
    if (rtx_camera_look_at(cfg.cam_pos, cfg.cam_look_at, cfg.up, persp[0], persp[1], persp[2], 0.0f, cfg.width,
                           cfg.height, &f) != RTX_OK)
        return false;
    std::memcpy(out.perspective_vals, persp, sizeof(persp));
    const float *rows[4] = {f.origin, f.horizontal, f.vertical, f.lower_left};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) out.view_vals[4 * j + i] = rows[i][j];  // XMMatrixTranspose (:60)
    for (int k = 0; k < 4; ++k) out.curr_samples[k] = sample_count;       // (:491-492)
    return true;
}

RtxCSApp::~RtxCSApp() { Terminate(); }

bool RtxCSApp::LoadContent() {
    if (m_cfg.cbuffers) {  // the reference's WorldDef bytes through the adapter
        WorldDefBytes wd;
        rtx_world w{};
        m_spheres.assign(4 * 512, 0.0f);
        m_mat_types.assign(512, 0.0f);
        m_mat_values.assign(4 * 512, 0.0f);
        if (m_cfg.scene != SceneKind::RandomWorld || !fill_worlddef(m_cfg, wd) ||
            rtx_world_from_worlddef(&wd, sizeof(wd), m_spheres.data(), m_mat_types.data(), m_mat_values.data(),
                                    &w) != RTX_OK) {
            m_error = "WorldDef: only random_world scenes of at most 512 spheres fit the cbuffer";
            return m_ok = false;
        }
        m_count = w.count;
        if (rtx_upload_world(m_ctx, &w) != RTX_OK) {  // CreateBuffer(WorldDef, IMMUTABLE) (:393-413)
            m_error = rtx_last_error();
            return m_ok = false;
        }
        return m_ok = true;
    }
    // WorldDef w; WorldDef::random_world(w);  (DxCSApp.cpp:401-402)
    uint32_t cap = m_cfg.scene == SceneKind::PsWorld ? 7 : 4;
    if (m_cfg.scene == SceneKind::RandomWorld) {
        const uint64_t full = 4ull + 4ull * (uint64_t)m_cfg.grid_half_extent * m_cfg.grid_half_extent;
        cap = (uint32_t)std::min<uint64_t>(full, m_cfg.max_spheres ? m_cfg.max_spheres : full);
    }
    m_spheres.assign(4 * (size_t)cap, 0.0f);
    m_mat_types.assign(cap, 0.0f);
    m_mat_values.assign(4 * (size_t)cap, 0.0f);
    int rc = (m_cfg.scene == SceneKind::RandomWorld)
                 ? rtx_scene_random_world(m_cfg.grid_half_extent, cap, m_spheres.data(),
                                          m_mat_types.data(), m_mat_values.data(), &m_count)
                 : (m_cfg.scene == SceneKind::PsWorld)
                       ? rtx_scene_ps_world(m_spheres.data(), m_mat_types.data(), m_mat_values.data(), &m_count)
                       : rtx_scene_test_world(m_spheres.data(), m_mat_types.data(), m_mat_values.data(),
                                              &m_count);
    if (rc != RTX_OK) {
        m_error = "scene generation failed";
        return m_ok = false;
    }
    rtx_world w{};
    w.count = m_count;
    w.depth = m_cfg.depth;
    w.spp = m_cfg.spp;
    w.spheres = m_spheres.data();
    w.mat_types = m_mat_types.data();
    w.mat_values = m_mat_values.data();
    // CreateBuffer(WorldDef, IMMUTABLE)  (DxCSApp.cpp:393-413)
    if (rtx_upload_world(m_ctx, &w) != RTX_OK) {
        m_error = rtx_last_error();
        return m_ok = false;
    }
    return m_ok = true;
}

void RtxCSApp::UnloadContent() {
    // Device resources belong to the context; RtxBase::Terminate destroys it.
    m_spheres.clear();
    m_mat_types.clear();
    m_mat_values.clear();
}

void RtxCSApp::Update() {
    // focus_dist = |camPos - camLookAt|; ComputeViewVals; sampleCount++
    // (DxCSApp.cpp:488-492), then the PerFrame upload (:494-496).
    int rc;
    if (m_cfg.cbuffers) {  // the reference's PerFrame bytes through the adapter
        PerFrameBytes pf;
        rc = fill_perframe(m_cfg, (float)(m_frame_count + 1), pf)
                 ? rtx_frame_from_perframe(&pf, sizeof(pf), m_cfg.width, m_cfg.height, &m_frame)
                 : RTX_ERR_INVALID;
    } else if (m_cfg.simple_camera)
        rc = rtx_camera_simple(m_cfg.width, m_cfg.height, &m_frame);
    else
        rc = rtx_camera_look_at(m_cfg.cam_pos, m_cfg.cam_look_at, m_cfg.up, m_cfg.vfov, m_cfg.aspect,
                                m_cfg.aperture, 0.0f, m_cfg.width, m_cfg.height, &m_frame);
    m_frame.rng_mode = m_cfg.rng_mode;
    m_frame.flags = m_cfg.lambert_guard ? RTX_FRAME_LAMBERT_GUARD : 0u;
    if (rc == RTX_OK && m_cfg.lens_aperture > 0.0f) rc = rtx_camera_set_aperture(&m_frame, m_cfg.lens_aperture);
    ++m_frame_count;
    if (rc != RTX_OK || rtx_set_frame(m_ctx, &m_frame) != RTX_OK) {
        m_error = rtx_last_error();
        m_ok = false;
    }
}

void RtxCSApp::Render() {
    // Dispatch(32,32,1)  (DxCSApp.cpp:524)
    if (!m_ok) return;
    if (rtx_render(m_ctx) != RTX_OK) {
        m_error = rtx_last_error();
        m_ok = false;
    }
}

bool RtxCSApp::Download(std::vector<float> &rgba) {
    rgba.resize(4 * (size_t)m_cfg.width * m_cfg.height);
    if (rtx_download(m_ctx, rgba.data(), rgba.size() * sizeof(float)) != RTX_OK) {
        m_error = rtx_last_error();
        return false;
    }
    return true;
}

bool write_pfm(const std::string &path, const float *rgba, uint32_t w, uint32_t h) {
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    std::fprintf(f, "PF\n%u %u\n-1.0\n", w, h);  // negative scale: little endian
    std::vector<float> row(3 * (size_t)w);
    bool ok = true;
    for (uint32_t y = 0; y < h && ok; ++y) {  // PFM rows run bottom-to-top
        for (uint32_t x = 0; x < w; ++x)
            for (int c = 0; c < 3; ++c) row[3 * x + c] = rgba[4 * ((size_t)y * w + x) + c];
        ok = std::fwrite(row.data(), sizeof(float), row.size(), f) == row.size();
    }
    return std::fclose(f) == 0 && ok;
}

bool write_ppm(const std::string &path, const float *rgba, uint32_t w, uint32_t h) {
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    std::fprintf(f, "P6\n%u %u\n255\n", w, h);
    std::vector<unsigned char> row(3 * (size_t)w);
    bool ok = true;
    for (uint32_t yy = 0; yy < h && ok; ++yy) {
        const uint32_t y = h - 1 - yy;  // top row first
        for (uint32_t x = 0; x < w; ++x)
            for (int c = 0; c < 3; ++c) {
                float v = rgba[4 * ((size_t)y * w + x) + c];
                v = std::isnan(v) ? 0.0f : std::min(1.0f, std::max(0.0f, v));
                row[3 * x + c] = (unsigned char)(255.999f * v);  // Color.h:6-11 scaling
            }
        ok = std::fwrite(row.data(), 1, row.size(), f) == row.size();
    }
    return std::fclose(f) == 0 && ok;
}

}  // namespace rtx
