// grid_check.cpp — CPU check of the exactness claim of the layer grid
// (raytrace-we-gpu_amd/csrc/rtx_grid.h): for layers of spheres at one
// height — the RTIOW layer (unit cells, jitter 0.9, r 0.2) and random ones
// (heights -5..5, radii 1e-2..2, extents 1..100, 8..512 spheres, so cell
// sides from 1/8 to 16) — and adversarial rays — near-tangent to a sphere
// of the layer (relative distance 1e-9..1e-1 from the silhouette) at every
// slope down to grazing the layer (|dy| 1e-7 of |d|), aimed at cell corners
// and edges, along the x or z axis or level (dx, dz or dy exactly 0),
// leaving a sphere's surface, origins out to |o| = 64 — every sphere the
// reference accepts (a root >= t_min, t_min 0 and 1e-3; the op order of
// oracle/rtx_oracle.c hit_world32) must have its block's bit in the walk's
// mask, whenever the kernel applies the grid (the prefilter's line test in
// its safe range). The grid is built and walked by the header's own code.
// Prints one JSON line; exit status 1 if any accepted sphere is missed.
// Build: g++ -O2 -std=c++17 -ffp-contract=off -mfma grid_check.cpp
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../raytrace-we-gpu_amd/csrc/rtx_grid.h"
#include "../raytrace-we-gpu_amd/csrc/rtx_prefilter.h"

static unsigned long long g_s = 0x2545f4914f6cdd1dull;
static double uni() {
    g_s ^= g_s << 13;
    g_s ^= g_s >> 7;
    g_s ^= g_s << 17;
    return (double)(g_s >> 11) * (1.0 / 9007199254740992.0);
}
static double sym() { return 2.0 * uni() - 1.0; }
static void unit(double v[3]) {
    do {
        v[0] = sym(), v[1] = sym(), v[2] = sym();
    } while (v[0] * v[0] + v[1] * v[1] + v[2] * v[2] < 1e-6);
    const double n = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    v[0] /= n, v[1] /= n, v[2] /= n;
}

// hit_world32's acceptance of one sphere (best = +inf): a root >= t_min;
// *root receives it.
static bool ref_accepts(const float o[3], const float d[3], const float *c, float a, float t_min,
                        float *root = nullptr) {
    const float negr2 = -(c[3] * c[3]);
    const float ocx = o[0] - c[0], ocy = o[1] - c[1], ocz = o[2] - c[2];
    const float hb = fmaf(ocz, d[2], fmaf(ocy, d[1], ocx * d[0]));
    const float cc = fmaf(ocz, ocz, fmaf(ocy, ocy, fmaf(ocx, ocx, negr2)));
    const float disc = fmaf(hb, hb, -(a * cc));
    if (disc < 0.0f) return false;
    const float inv_a = 1.0f / a, sq = std::sqrt(disc);
    const float rn = (-hb - sq) * inv_a;
    if (!(rn < t_min || INFINITY < rn)) {
        if (root) *root = rn;
        return true;
    }
    const float rf = (-hb + sq) * inv_a;
    if (root) *root = rf;
    return !(rf < t_min || INFINITY < rf);
}

struct Layer {
    std::vector<float> s;  // (cx, cy, cz, r)
    rtx::LayerGrid G;
    std::vector<unsigned long long> cell;
};

static bool make_layer(Layer &L, bool rtiow) {
    L.s.clear();
    if (rtiow) {
        for (int a = -11; a < 11; ++a)
            for (int b = -11; b < 11; ++b) {
                if (uni() < 0.03) continue;  // a few holes, as the 0.9 cutoff leaves
                L.s.insert(L.s.end(), {(float)(a + 0.9 * uni()), 0.2f, (float)(b + 0.9 * uni()), 0.2f});
                if (L.s.size() / 4 == 480) break;
            }
    } else {
        const int n = 8 + (int)(uni() * 505);
        const float y0 = (float)(5.0 * sym());
        const double ext = std::pow(10.0, 4.0 * uni() - 2.0) * std::sqrt((double)n);  // 1e-2..1e2 per sphere
        const double rmax = std::pow(10.0, -2.0 + 2.3 * uni());
        for (int i = 0; i < n; ++i)
            L.s.insert(L.s.end(), {(float)(ext * sym()), y0, (float)(ext * sym()), (float)(rmax * (0.05 + 0.95 * uni()))});
    }
    return rtx::build_layer_grid(L.s.data(), 0u, (uint32_t)(L.s.size() / 4), L.G, L.cell);
}

int main(int argc, char **argv) {
    const long nlayers = argc > 1 ? atol(argv[1]) : 300;
    const long nrays = argc > 2 ? atol(argv[2]) : 4000;
    long rays = 0, applied = 0, all = 0, accepted = 0, missed = 0, layers = 0, nogrid = 0;
    long far_checked = 0, far_missed = 0;
    double far_bits = 0.0;
    double bits = 0.0;
    for (long li = 0; li < nlayers; ++li) {
        Layer L;
        if (!make_layer(L, li % 3 == 0)) {
            ++nogrid;
            continue;
        }
        ++layers;
        const uint32_t n = (uint32_t)(L.s.size() / 4);
        const float y0 = L.s[1];
        auto cellf = [&L](uint32_t k) { return (uint64_t)L.cell[k]; };
        for (long k = 0; k < nrays; ++k) {
            const float *c = &L.s[4 * (size_t)(uni() * n)];
            const double r = c[3];
            double dir[3], o[3];
            const int kind = (int)(uni() * 5.0);
            unit(dir);
            // slope: uniform, or grazing the layer
            if (uni() < 0.4) dir[1] = std::pow(10.0, -7.0 + 6.0 * uni()) * sym();
            if (kind == 3) {  // along an axis or level
                const int z = (int)(uni() * 3.0);
                dir[z == 0 ? 0 : z == 1 ? 2 : 1] = 0.0;
            }
            if (kind == 1) {  // aimed at a cell corner / edge, from anywhere
                const double cxg = L.G.x0 + L.G.h * std::floor(uni() * L.G.nx), czg = L.G.z0 + L.G.h * std::floor(uni() * L.G.nz);
                const double tgt[3] = {cxg + (uni() < 0.5 ? 0.0 : L.G.h * uni()), y0 + r * sym(), czg + (uni() < 0.5 ? 0.0 : L.G.h * uni())};
                const double back = std::pow(10.0, -1.0 + 2.5 * uni());
                for (int i = 0; i < 3; ++i) o[i] = tgt[i] - back * dir[i];
            } else if (kind == 4) {  // leaving a sphere's surface (radially, or at random)
                double nrm[3];
                unit(nrm);
                const double dl = uni() < 0.3 ? 0.0 : std::pow(10.0, -7.0 + 5.0 * uni()) * sym();
                for (int i = 0; i < 3; ++i) o[i] = c[i] + r * (1.0 + dl) * nrm[i];
                if (uni() < 0.5)
                    for (int i = 0; i < 3; ++i) dir[i] = nrm[i];
            } else {  // near-tangent to sphere c (kinds 0, 2, 3)
                double t[3], e[3];
                unit(t);
                const double td = t[0] * dir[0] + t[1] * dir[1] + t[2] * dir[2];
                for (int i = 0; i < 3; ++i) e[i] = t[i] - td * dir[i];
                const double en = std::sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
                if (en < 1e-9) continue;
                const double delta = std::pow(10.0, -9.0 + 8.0 * uni()) * (uni() < 0.5 ? -1.0 : 1.0);
                const double dist = uni() < 0.8 ? r * (1.0 + delta) : 2.0 * r * uni();
                const double along = sym() * std::pow(10.0, -1.0 + 2.8 * uni());
                for (int i = 0; i < 3; ++i) o[i] = c[i] + dist * e[i] / en - along * dir[i];
            }
            const double on = std::sqrt(o[0] * o[0] + o[1] * o[1] + o[2] * o[2]);
            if (on > 63.9) continue;
            const double dlen = std::pow(10.0, -2.0 + 4.0 * uni());
            float of[3], df[3];
            for (int i = 0; i < 3; ++i) of[i] = (float)o[i], df[i] = (float)(dir[i] * dlen);
            ++rays;
            const float a = fmaf(df[2], df[2], fmaf(df[1], df[1], df[0] * df[0]));
            // the kernel applies the grid only where the line test is safe
            const rtx::LineTest T = rtx::line_test_setup(of[0], of[1], of[2], df[0], df[1], df[2], a, 200.0f);
            if (T.thr == -INFINITY) continue;
            ++applied;
            const uint64_t m = rtx::grid_mask(L.G, cellf, of[0], of[1], of[2], df[0], df[1], df[2]);
            if (m == ~0ull) {
                ++all;
                continue;
            }
            bits += (double)__builtin_popcountll(m);
            std::vector<float> roots(n, INFINITY);
            float win = INFINITY;
            for (uint32_t i = 0; i < n; ++i) {
                const float *ci = &L.s[4 * (size_t)i];
                const bool a0 = ref_accepts(of, df, ci, a, 0.0f);
                const bool a1 = ref_accepts(of, df, ci, a, 1e-3f, &roots[i]);
                if (!a1) roots[i] = INFINITY;
                win = fminf(win, roots[i]);
                if (!a0 && !a1) continue;
                ++accepted;
                if (!((m >> (i / 8)) & 1ull)) {
                    if (missed < 5)
                        fprintf(stderr, "miss: sphere %u (%g %g %g r %g) o (%.9g %.9g %.9g) d (%.9g %.9g %.9g)\n", i,
                                ci[0], ci[1], ci[2], ci[3], of[0], of[1], of[2], df[0], df[1], df[2]);
                    ++missed;
                }
            }
            // the far cut (t_min 1e-3, the render's): B at the winner's own root
            // (a tie goes to the later sphere: every root <= B must be scanned),
            // and at a random fraction of it, t_stop = B + far_m / |d| in fp32
            if (win < INFINITY) {
                const float inv_len = 1.0f / std::sqrt(a);
                for (int rep = 0; rep < 2; ++rep) {
                    const float B = rep == 0 ? win : win * (float)(0.5 + uni());
                    const float ts = fmaf(L.G.far_m, inv_len, B);
                    const uint64_t mf = rtx::grid_mask(L.G, cellf, of[0], of[1], of[2], df[0], df[1], df[2], ts);
                    far_bits += (double)__builtin_popcountll(mf);
                    for (uint32_t i = 0; i < n; ++i) {
                        if (!(roots[i] <= B)) continue;
                        ++far_checked;
                        if (!((mf >> (i / 8)) & 1ull)) {
                            if (far_missed < 5)
                                fprintf(stderr, "far miss: sphere %u root %.9g B %.9g o (%.9g %.9g %.9g) d (%.9g %.9g %.9g)\n",
                                        i, roots[i], B, of[0], of[1], of[2], df[0], df[1], df[2]);
                            ++far_missed;
                        }
                    }
                }
            }
        }
    }
    const long masked = applied - all;
    printf("{\"layers\": %ld, \"layers_without_grid\": %ld, \"rays\": %ld, \"grid_applied\": %ld, "
           "\"every_block\": %ld, \"accepted_spheres\": %ld, \"missed\": %ld, \"mean_blocks_marked\": %.3f, "
           "\"far_checked\": %ld, \"far_missed\": %ld}\n",
           layers, nogrid, rays, applied, all, accepted, missed, masked ? bits / (double)masked : 0.0, far_checked,
           far_missed);
    return missed == 0 && far_missed == 0 ? 0 : 1;
}
