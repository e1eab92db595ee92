// image_writer_check.cpp — drives the image writers of rtx_cli (rtx_app.cpp
// write_pfm / write_ppm) on a synthetic framebuffer, no GPU:
//   image_writer_check W H in.f32 out.pfm out.ppm
// in.f32: W*H float4 (row 0 = image bottom, as rtx_download returns it).
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/rtx_app.hpp"

int main(int argc, char **argv) {
    if (argc != 6) return 2;
    const unsigned w = (unsigned)std::atoi(argv[1]), h = (unsigned)std::atoi(argv[2]);
    std::vector<float> img(4 * (size_t)w * h);
    FILE *f = std::fopen(argv[3], "rb");
    if (!f || std::fread(img.data(), sizeof(float), img.size(), f) != img.size()) return 3;
    std::fclose(f);
    if (!rtx::write_pfm(argv[4], img.data(), w, h)) return 4;
    if (!rtx::write_ppm(argv[5], img.data(), w, h)) return 5;
    return 0;
}
