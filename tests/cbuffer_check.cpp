// cbuffer_check.cpp — the reference's cbuffer byte path of rtx_app.cpp
// (fill_worlddef / fill_perframe, then the library's adapters
// rtx_world_from_worlddef / rtx_frame_from_perframe) on the CPU, no GPU:
//   cbuffer_check out_dir
// writes worlddef.bin (18,448 B), perframe.bin (112 B), and what the adapters
// parse them into: world.f32 (count x [sphere 4, type 1, value 4]) with
// world.txt "count depth spp", and frame.bin (the rtx_frame struct).
#include <cstdio>
#include <string>
#include <vector>

#include "../include/rtx_app.hpp"

static bool dump(const std::string &path, const void *p, size_t n) {
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = std::fwrite(p, 1, n, f) == n;
    return std::fclose(f) == 0 && ok;
}

int main(int argc, char **argv) {
    if (argc != 2) return 2;
    const std::string dir = argv[1];
    rtx::AppConfig cfg;  // the reference's defaults: 1024x576, spp 60, depth 50, grid 9
    cfg.cbuffers = true;
    rtx::WorldDefBytes wd;
    rtx::PerFrameBytes pf;
    if (!rtx::fill_worlddef(cfg, wd) || !rtx::fill_perframe(cfg, 1.0f, pf)) return 3;
    std::vector<float> sph(4 * 512), mt(512), mv(4 * 512);
    rtx_world w{};
    if (rtx_world_from_worlddef(&wd, sizeof(wd), sph.data(), mt.data(), mv.data(), &w) != RTX_OK) return 4;
    rtx_frame f{};
    if (rtx_frame_from_perframe(&pf, sizeof(pf), cfg.width, cfg.height, &f) != RTX_OK) return 5;
    std::vector<float> rows;
    for (uint32_t i = 0; i < w.count; ++i) {
        for (int k = 0; k < 4; ++k) rows.push_back(sph[4 * i + k]);
        rows.push_back(mt[i]);
        for (int k = 0; k < 4; ++k) rows.push_back(mv[4 * i + k]);
    }
    char txt[64];
    const int n = std::snprintf(txt, sizeof(txt), "%u %u %u\n", w.count, w.depth, w.spp);
    if (!dump(dir + "/worlddef.bin", &wd, sizeof(wd)) || !dump(dir + "/perframe.bin", &pf, sizeof(pf)) ||
        !dump(dir + "/world.f32", rows.data(), rows.size() * sizeof(float)) || !dump(dir + "/world.txt", txt, (size_t)n) ||
        !dump(dir + "/frame.bin", &f, sizeof(f)))
        return 6;
    return 0;
}
