// rtx_cli — headless driver replacing the reference's Win32 shell
// (CSVersion/main.cpp:16-58: Initialize, one Update + Render, Terminate).
// Renders K frames, prints one JSON line of timing/counters, optionally
// writes the last frame as PFM / PPM.
//
//   rtx_cli [--width W] [--height H] [--spp S] [--depth D]
//           [--scene rtiow9|rtiow11|test|ps|random:EXT[:MAX]] [--simple-camera]
//           [--rng chain|per-sample] [--frames K] [--device N]
//           [--aperture A] [--accumulate] [--lambert-guard]
//           [--reference-frame] [--pfm out.pfm] [--ppm out.ppm]
// --accumulate renders the K frames progressively (rtx_accumulate) instead
// of K independent frames; --aperture enables the thin lens;
// --lambert-guard the near-zero diffuse guard (RTX_FRAME_LAMBERT_GUARD).
// --reference-frame: the reference's frame as shipped — 1024x576, spp 60,
// depth 50, random_world with 326 spheres, camera (13,2,3) -> 0, vfov 20,
// aspect 16/9 (DxCSApp.cpp:133,176-179,330-331) — uploaded as the reference's
// own WorldDef and PerFrame cbuffer bytes through rtx_world_from_worlddef /
// rtx_frame_from_perframe; a preset: every other option, before or after
// it, overrides its values.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rtx_app.hpp"

static void usage() {
    std::fprintf(stderr,
                 "usage: rtx_cli [--width W] [--height H] [--spp S] [--depth D]\n"
                 "               [--scene rtiow9|rtiow11|test|ps|random:EXT[:MAX]] [--simple-camera]\n"
                 "               [--rng chain|per-sample] [--frames K] [--device N]\n"
                 "               [--aperture A] [--accumulate] [--lambert-guard] [--reference-frame]\n"
                 "               [--pfm FILE] [--ppm FILE]\n");
}

int main(int argc, char **argv) {
    rtx::AppConfig cfg;
    cfg.width = 1920;
    cfg.height = 1080;
    cfg.spp = 100;
    cfg.depth = 50;
    cfg.grid_half_extent = 11;
    // --reference-frame is a preset: it sets the reference's values first,
    // wherever it stands, and every other option then overrides them
    for (int i = 1; i < argc; ++i) {
        if (std::string(argv[i]) == "--reference-frame") {
            cfg = rtx::AppConfig();  // the reference's values (include/rtx_app.hpp)
            cfg.cbuffers = true;
        }
    }
    int frames = 1, device = 0;
    bool accumulate = false;
    std::string pfm, ppm;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char * {
            if (i + 1 >= argc) {
                usage();
                std::exit(2);
            }
            return argv[++i];
        };
        if (a == "--width") cfg.width = (uint32_t)std::atoi(next());
        else if (a == "--height") cfg.height = (uint32_t)std::atoi(next());
        else if (a == "--spp") cfg.spp = (uint32_t)std::atoi(next());
        else if (a == "--depth") cfg.depth = (uint32_t)std::atoi(next());
        else if (a == "--frames") frames = std::atoi(next());
        else if (a == "--device") device = std::atoi(next());
        else if (a == "--pfm") pfm = next();
        else if (a == "--ppm") ppm = next();
        else if (a == "--simple-camera") cfg.simple_camera = true;
        else if (a == "--aperture") cfg.lens_aperture = (float)std::atof(next());
        else if (a == "--accumulate") accumulate = true;
        else if (a == "--lambert-guard") cfg.lambert_guard = true;
        else if (a == "--reference-frame") {
            // a preset, applied before the loop (below): here it only keeps its place
        }
        else if (a == "--rng") {
            const std::string m = next();
            cfg.rng_mode = (m == "per-sample") ? RTX_RNG_PER_SAMPLE : RTX_RNG_CHAIN;
        } else if (a == "--scene") {
            const std::string s = next();
            if (s == "rtiow9") cfg.grid_half_extent = 9;
            else if (s == "rtiow11") cfg.grid_half_extent = 11;
            else if (s == "test") cfg.scene = rtx::SceneKind::TestWorld;
            else if (s == "ps") cfg.scene = rtx::SceneKind::PsWorld;
            else if (s.rfind("random:", 0) == 0) {
                unsigned ext = 0, mx = 0;
                if (std::sscanf(s.c_str() + 7, "%u:%u", &ext, &mx) < 1) {
                    usage();
                    return 2;
                }
                cfg.grid_half_extent = (int32_t)ext;
                cfg.max_spheres = mx;
            } else {
                usage();
                return 2;
            }
        } else {
            usage();
            return 2;
        }
    }
    if (cfg.width == 0 || cfg.height == 0 || frames < 1) {
        usage();
        return 2;
    }
    cfg.aspect = (float)cfg.width / (float)cfg.height;
    rtx::RtxCSApp app(cfg);
    if (!app.Initialize(device)) {
        std::fprintf(stderr, "rtx_cli: initialize failed: %s\n", app.last_error().c_str());
        return 1;
    }
    app.Update();
    app.Render();  // warm-up frame (also the reference's single frame, main.cpp:38-39)
    rtx_sync(app.context());
    rtx_stats_reset(app.context());
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < frames; ++k) {
        app.Update();
        if (accumulate) {
            if (rtx_accumulate(app.context(), k == 0) != RTX_OK) {
                std::fprintf(stderr, "rtx_cli: accumulate failed: %s\n", rtx_last_error());
                return 1;
            }
        } else {
            app.Render();
        }
    }
    rtx_sync(app.context());
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (!app.ok()) {
        std::fprintf(stderr, "rtx_cli: render failed: %s\n", app.last_error().c_str());
        return 1;
    }
    rtx_stats st{};
    rtx_get_stats(app.context(), &st);
    std::printf("{\"width\": %u, \"height\": %u, \"spp\": %u, \"depth\": %u, \"spheres\": %u, "
                "\"cbuffers\": %s, \"frames\": %d, \"wall_s\": %.6f, \"kernel_ms\": %.4f, \"msamples_per_s\": %.3f, "
                "\"segments\": %llu, \"sphere_tests\": %llu}\n",
                cfg.width, cfg.height, cfg.spp, cfg.depth, app.sphere_count(), cfg.cbuffers ? "true" : "false",
                frames, wall,
                st.kernel_ms, (double)st.samples / wall / 1e6, (unsigned long long)st.segments,
                (unsigned long long)st.sphere_tests);
    if (!pfm.empty() || !ppm.empty()) {
        std::vector<float> img;
        if (!app.Download(img)) {
            std::fprintf(stderr, "rtx_cli: download failed: %s\n", app.last_error().c_str());
            return 1;
        }
        if (!pfm.empty() && !rtx::write_pfm(pfm, img.data(), cfg.width, cfg.height)) return 1;
        if (!ppm.empty() && !rtx::write_ppm(ppm, img.data(), cfg.width, cfg.height)) return 1;
    }
    app.Terminate();
    return 0;
}
