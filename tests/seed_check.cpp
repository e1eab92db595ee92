// seed_check.cpp — CPU check of rtx::seed_advance (raytrace-we-gpu_amd/csrc/
// rtx_seed.h) against the reference's literal seed steps (`seed += 0.1` in
// fp32, ShaderCompute.hlsl:30-48): for many start seeds (uniform in [0, 1] as
// the kernel's h / 2^32, values at and around every binade boundary up to
// 2^24, the tie binade [1/8, 1/4), 0 and tiny values), every step count up to
// N and sampled step counts up to 2^22, the jump must equal the literal
// additions bit for bit. Prints one JSON line; exit 1 on any mismatch.
// Build: g++ -O2 -std=c++17 -ffp-contract=off seed_check.cpp
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../raytrace-we-gpu_amd/csrc/rtx_seed.h"

static unsigned long long g_s = 0x2545f4914f6cdd1dull;
static uint32_t rnd() {
    g_s ^= g_s << 13;
    g_s ^= g_s >> 7;
    g_s ^= g_s << 17;
    return (uint32_t)(g_s >> 32);
}
static uint32_t bits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
static float fbits(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

int main(int argc, char **argv) {
    const uint32_t N = argc > 1 ? (uint32_t)atoi(argv[1]) : 12000;
    std::vector<float> starts = {0.0f, 1e-30f, 1e-7f, 0.05f, 0.1f, 0.125f, 0.2f, 0.25f, 0.3f, 1.0f};
    for (int k = 0; k < 1500; ++k) starts.push_back((float)rnd() / 4294967296.0f);  // pixel_seed range
    for (int e = -4; e <= 24; ++e)  // each binade boundary and its neighbours
        for (int d = -3; d <= 3; ++d) starts.push_back(fbits(bits(__builtin_ldexpf(1.0f, e)) + (uint32_t)(d + 8) - 8u));
    for (int k = 0; k < 200; ++k) starts.push_back(fbits(bits(0.125f) + (rnd() & 0x7fffffu)));  // tie binade
    uint64_t checked = 0, bad = 0;
    for (float s0 : starts) {
        float lit = s0;
        for (uint32_t n = 0; n <= N; ++n) {
            const float j = rtx::seed_advance(s0, n);
            ++checked;
            if (bits(j) != bits(lit)) {
                if (bad < 5) fprintf(stderr, "mismatch s0=%a n=%u jump=%a literal=%a\n", s0, n, j, lit);
                ++bad;
            }
            lit = lit + 0.1f;
        }
    }
    // long chains: sampled step counts up to ~4M from random seeds
    for (int k = 0; k < 24; ++k) {
        const float s0 = (float)rnd() / 4294967296.0f;
        float lit = s0;
        uint32_t n = 0;
        while (n < (1u << 22)) {
            const uint32_t step = 1u + (rnd() % 50000u);
            for (uint32_t i = 0; i < step; ++i) lit = lit + 0.1f;
            n += step;
            const float j = rtx::seed_advance(s0, n);
            ++checked;
            if (bits(j) != bits(lit)) {
                if (bad < 5) fprintf(stderr, "mismatch s0=%a n=%u jump=%a literal=%a\n", s0, n, j, lit);
                ++bad;
            }
        }
    }
    printf("{\"checked\": %llu, \"mismatches\": %llu}\n", (unsigned long long)checked, (unsigned long long)bad);
    return bad ? 1 : 0;
}
