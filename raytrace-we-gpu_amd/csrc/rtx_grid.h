// rtx_grid.h — the layer grid of the lane-mode scan, shared
// by the HIP kernel, the upload (rtx_api.hip) and the CPU checker
// (tests/grid_check.cpp).
//
// The RTIOW scenes keep almost every sphere in one thin layer: the scan's
// flat run, blocks [flat_lo, flat_hi) of `pre`, whose centres all sit at one
// fp32 height y0 (rtx_internal.h KScene). The reference tests every sphere
// of the list for every ray segment (Hittable_list.cpp:3-20,
// ShaderCompute.hlsl:194), and so does the scan — with the prefilter, 5 fp32
// ops a sphere. A ray's line, though, comes near the layer only where it
// crosses the slab |y - y0| <= rho around it, a short stretch for all but
// grazing rays. The grid says which blocks of the flat run can hold a
// sphere the reference accepts; the wave then scans only the blocks some
// lane needs, in index order, with the scan's own tests, and resolves with
// the reference's ops: the answer is unchanged (rtx_kernels.hip
// hit_world_pre_ld). No other part of the scene uses it.
//
// Exactness. rtx_prefilter.h (HalfTest) shows: if the reference accepts
// sphere i (a root >= t_min >= 0), some point p = o + t d with t >= 0 lies
// within sqrt(A_i + B) (1 + u) of c_i, A_i = r_i^2 (1 + 8u) + 27u |c_i|^2,
// B = 26u |o|^2. The grid is built for |o| <= kGridOMax (a ray with a farther
// origin scans every block), so that point is within
//   rho_i = sqrt(A_i + 26u kGridOMax^2) (1 + 4u)
// of c_i, and c_i.y = y0: it lies in the slab |y - y0| <= rho_max and its
// (x, z) within rho_i of the centre's. The layer's (x, z) plane is cut into
// square cells of side h (a power of two); a cell lists (as a 64-bit mask
// over the flat run's blocks) every sphere whose disc of radius
// rho_i + kGridFat meets it. The walk visits, for the ray's stretch of the
// slab with t >= 0 inside the grid's box, the cells its (x, z) projection
// crosses (a DDA whose every crossing time is computed afresh from the
// cell boundary, no accumulation), and ORs their masks. Its computed path
// leaves the true one by at most ~4u |p - o| (crossing order decided on
// rounded times: a skipped cell is touched by the true line only within
// that distance of a corner; the start cell from a rounded point; the slab
// and box ends from rounded times, and the slab carries kGridSlabPad more
// than rho_max, ~100x the rounding of its ends at |o| <= 64): at |p|,
// |o| <= 64 that is < 1e-4, far inside kGridFat = 2^-8 h. So the accepted
// point's cell, or a visited cell within 1e-4 of it, lists sphere i, and
// its block is scanned. A lane whose walk would pass kGridMaxSteps cells,
// or whose ray the prefilter's line test finds outside its safe range,
// or whose origin is farther than kGridOMax, marks every block.
// tests/grid_check.cpp checks the claim on adversarial rays (near-tangent,
// through cell corners, along the axes, grazing the layer, leaving a
// sphere's surface, at t_min 0 and 1e-3).
#pragma once

#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <utility>
#include <vector>

#if defined(__HIPCC__)
#define RTX_GD __host__ __device__ __forceinline__
#else
#define RTX_GD static inline
#endif

namespace rtx {

constexpr float kGridOMax = 64.0f;      // rays with |o| above this scan every block
constexpr double kGridFatCells = 1.0 / 256.0;  // cell-list fattening, in cells
constexpr double kGridSlabPad = 1e-3;          // slab half-width past rho_max (y units)
#ifndef RTX_GRID_STEPS  // A/B: the walk's step limit
#define RTX_GRID_STEPS 48
#endif
#ifndef RTX_GRID_HLOG  // A/B: cell side 2^k times the one-sphere-per-cell size
#define RTX_GRID_HLOG 0
#endif
constexpr uint32_t kGridMaxSteps = RTX_GRID_STEPS;  // a longer walk scans every block
constexpr uint32_t kGridMaxCells = 4096;  // cells of a grid at most

struct LayerGrid {
    float x0, z0;      // the grid's corner (multiples of h)
    float h, inv_h;    // cell side (a power of two) and its inverse (exact)
    float ylo, yhi;    // the slab: y0 -+ (rho_max + kGridSlabPad), rounded outwards
    uint32_t nx, nz;   // cells along x and z; cell (ix, iz) covers [x0 + ix h, x0 + (ix + 1) h] x ...
    float far_m;       // far cut: the walk may stop kGridFar(...) past the best root so far (distance units)
    uint32_t nblk;     // blocks the cells' masks name (<= 64)
};

// The far cut (the render's walks run before its scan and do
// not use it, t_stop = inf). A walk that knows the ray's best root B so far
// (the non-flat part of the scene resolved first) need only reach t = B + far_m / |d|: a sphere the reference accepts at a
// root c <= B has a point of its rho-ball chord at t <= c + e, e the fp32
// root's error, <= 2 sqrt(8u) |o - c_i| / |d| (the discriminant's rounding,
// 8u (hb^2 + a|cc|), through the square root) — far_m = 4e-3 (|o|max +
// |c|max) + 1e-3 covers it with a factor >= 2.8; tests/grid_check.cpp checks
// the cut with B at the winner's own root (ties go to the later sphere).
// The walk: visits the cells (k = ix * nz + iz) the (x, z) projection of the
// ray's stretch inside the slab and the grid's box, t in [0, t_stop], crosses;
// returns false when it gives up (far or non-finite ray, or more than
// max_steps cells): the caller then scans every block.
template <typename Visit>
RTX_GD bool grid_walk(const LayerGrid &G, uint32_t max_steps, float ox, float oy, float oz, float dx, float dy,
                      float dz, float t_stop, Visit visit) {
    const float o2 = fmaf(ox, ox, fmaf(oy, oy, oz * oz));
    const float d2 = fmaf(dx, dx, fmaf(dy, dy, dz * dz));
    if (!(o2 <= kGridOMax * kGridOMax) || !(d2 <= 3.0e38f)) return false;  // far or non-finite
    const float inf = INFINITY;
    float t0 = 0.0f, t1 = t_stop >= 0.0f ? t_stop : inf;  // (NaN t_stop: no cut)
    // the slab and the grid's box, one axis at a time: [lo, hi] along o + t d
    auto clip = [&](float o, float d, float lo, float hi) {
        if (d == 0.0f) {
            if (!(o >= lo && o <= hi)) t1 = -inf;  // parallel and outside: nothing
            return;
        }
        const float inv = 1.0f / d;
        const float ta = (lo - o) * inv, tb = (hi - o) * inv;
        t0 = fmaxf(t0, fminf(ta, tb));
        t1 = fminf(t1, fmaxf(ta, tb));
    };
    clip(oy, dy, G.ylo, G.yhi);
    clip(ox, dx, G.x0, G.x0 + (float)G.nx * G.h);
    clip(oz, dz, G.z0, G.z0 + (float)G.nz * G.h);
    if (!(t0 <= t1)) return true;  // the ray's t >= 0 part never enters the slab inside the grid
    // start cell: the rounded point at t0 (clamped: it is within rounding of the box)
    const float sx = (fmaf(t0, dx, ox) - G.x0) * G.inv_h, sz = (fmaf(t0, dz, oz) - G.z0) * G.inv_h;
    int ix = (int)fminf(fmaxf(floorf(sx), 0.0f), (float)(G.nx - 1));
    int iz = (int)fminf(fmaxf(floorf(sz), 0.0f), (float)(G.nz - 1));
    const int stx = dx > 0.0f ? 1 : -1, stz = dz > 0.0f ? 1 : -1;
    const float ivx = dx == 0.0f ? 0.0f : 1.0f / dx, ivz = dz == 0.0f ? 0.0f : 1.0f / dz;
    for (uint32_t k = 0; k < max_steps; ++k) {
        if (!visit((uint32_t)ix * G.nz + (uint32_t)iz)) return false;
        // the next boundary crossings, each from its boundary (exact: a multiple of h)
        const float bx = fmaf((float)(ix + (dx > 0.0f ? 1 : 0)), G.h, G.x0);
        const float bz = fmaf((float)(iz + (dz > 0.0f ? 1 : 0)), G.h, G.z0);
        const float tx = dx == 0.0f ? inf : (bx - ox) * ivx;
        const float tz = dz == 0.0f ? inf : (bz - oz) * ivz;
        if (!(fminf(tx, tz) <= t1)) return true;
        if (tx <= tz) {
            ix += stx;
            if (ix < 0 || ix >= (int)G.nx) return true;
        } else {
            iz += stz;
            if (iz < 0 || iz >= (int)G.nz) return true;
        }
    }
    return false;
}

// The block-mask grid (small scenes): the mask of the flat run's blocks the
// ray (o, d) may need (bit j: block flat_lo + j); ~0 when the lane must scan
// every block. `cell(k)` returns cell k's mask.
template <typename Cell>
RTX_GD uint64_t grid_mask(const LayerGrid &G, Cell cell, float ox, float oy, float oz, float dx, float dy, float dz,
                          float t_stop = INFINITY) {
    uint64_t m = 0ull;
    const bool done = grid_walk(G, kGridMaxSteps, ox, oy, oz, dx, dy, dz, t_stop, [&](uint32_t k) {
        m |= cell(k);
        return true;
    });
    return done ? m : ~0ull;
}

// Host: the geometry of a layer grid over `m` spheres sph[4 j] = (cx, cy,
// cz, r) (every cy equal: y0) and, for each, every cell its disc of radius
// rho_j + kGridFat meets: add(cell, j). Returns false (no grid) past
// max_cells cells.
template <typename Add>
inline bool build_layer_grid_cells(const float *sph, uint32_t m, uint32_t max_cells, LayerGrid &G, Add add) {
    if (m == 0) return false;
    const double u = 5.9604644775390625e-08;
    const double y0 = sph[1];
    const double B = 26.0 * u * (double)kGridOMax * (double)kGridOMax;
    auto rho_of = [&](uint32_t j) {
        const double cx = sph[4 * (size_t)j], cz = sph[4 * (size_t)j + 2], r = sph[4 * (size_t)j + 3];
        const double c2 = cx * cx + y0 * y0 + cz * cz;
        return std::sqrt(r * r * (1.0 + 8.0 * u) + 27.0 * u * c2 + B) * (1.0 + 4.0 * u) * (1.0 + 1e-12);
    };
    double rho_max = 0.0, cmax = 0.0, xlo = INFINITY, xhi = -INFINITY, zlo = INFINITY, zhi = -INFINITY;
    for (uint32_t j = 0; j < m; ++j) {
        const double cx = sph[4 * (size_t)j], cz = sph[4 * (size_t)j + 2];
        const double rho = rho_of(j);
        rho_max = std::fmax(rho_max, rho);
        cmax = std::fmax(cmax, std::sqrt(cx * cx + y0 * y0 + cz * cz));
        xlo = std::fmin(xlo, cx - rho), xhi = std::fmax(xhi, cx + rho);
        zlo = std::fmin(zlo, cz - rho), zhi = std::fmax(zhi, cz + rho);
    }
    // cell side: the power of two nearest one sphere per cell, at least rho_max
    const double area = std::fmax((xhi - xlo) * (zhi - zlo), 1e-30);
    double h = std::exp2(std::round(std::log2(std::sqrt(area / m))) + RTX_GRID_HLOG);
    while (h < rho_max) h *= 2.0;
    const double fat = kGridFatCells * h;
    // the box: a spare cell on every side (no disc reaches it)
    const double x0 = (std::floor((xlo - fat) / h) - 1.0) * h, z0 = (std::floor((zlo - fat) / h) - 1.0) * h;
    const double nxd = std::ceil((xhi + fat - x0) / h) + 1.0, nzd = std::ceil((zhi + fat - z0) / h) + 1.0;
    if (nxd * nzd > max_cells || !(std::fabs(x0) < 1e6 && std::fabs(z0) < 1e6)) return false;
    G.nx = (uint32_t)nxd, G.nz = (uint32_t)nzd;
    G.h = (float)h, G.inv_h = (float)(1.0 / h);
    G.x0 = (float)x0, G.z0 = (float)z0;
    const double slab = rho_max + kGridSlabPad;
    G.ylo = nextafterf((float)(y0 - slab), -INFINITY);
    G.yhi = nextafterf((float)(y0 + slab), INFINITY);
    G.far_m = nextafterf((float)(4e-3 * ((double)kGridOMax + cmax) + 1e-3), INFINITY);
    for (uint32_t j = 0; j < m; ++j) {
        const double cx = sph[4 * (size_t)j], cz = sph[4 * (size_t)j + 2];
        const double rho = rho_of(j) + fat;
        const int ax = (int)std::floor((cx - rho - x0) / h), bxi = (int)std::floor((cx + rho - x0) / h);
        const int az = (int)std::floor((cz - rho - z0) / h), bzi = (int)std::floor((cz + rho - z0) / h);
        for (int ix = std::max(ax, 0); ix <= std::min(bxi, (int)G.nx - 1); ++ix)
            for (int iz = std::max(az, 0); iz <= std::min(bzi, (int)G.nz - 1); ++iz) {
                // the closed square's nearest point to the centre
                const double qx = std::fmin(std::fmax(cx, x0 + ix * h), x0 + (ix + 1) * h);
                const double qz = std::fmin(std::fmax(cz, z0 + iz * h), z0 + (iz + 1) * h);
                if ((qx - cx) * (qx - cx) + (qz - cz) * (qz - cz) <= rho * rho) add((uint32_t)ix * G.nz + iz, j);
            }
    }
    return true;
}

// Host: the block-mask grid of the spheres [i_lo, i_hi) of `sph` (bit
// (i - i_lo) / 8 of a cell's mask). Returns false (no grid) if the run spans
// more than 64 blocks or the grid would exceed kGridMaxCells cells. `cell`
// receives nx * nz masks.
template <typename Vec>
inline bool build_layer_grid(const float *sph, uint32_t i_lo, uint32_t i_hi, LayerGrid &G, Vec &cell) {
    const uint32_t m = i_hi - i_lo;
    if (m == 0 || (m + 7) / 8 > 64) return false;
    std::vector<std::pair<uint32_t, uint32_t>> hits;
    if (!build_layer_grid_cells(sph + 4 * (size_t)i_lo, m, kGridMaxCells, G,
                                [&](uint32_t k, uint32_t j) { hits.emplace_back(k, j); }))
        return false;
    G.nblk = (m + 7) / 8;
    cell.assign((size_t)G.nx * G.nz, 0ull);
    for (const auto &h : hits) cell[h.first] |= 1ull << (h.second / 8);
    return true;
}

}  // namespace rtx
