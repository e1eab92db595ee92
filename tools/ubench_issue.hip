// ubench_issue.hip — VALU issue cost on this MI355X, in the chip's own cycles
// (reconcile the round-5 ubench's 3.3 "cycles" per
// v_fma_f32, which were wall time at a nominal 2.4 GHz, with the guide's 2).
// Each kernel issues one instruction class from independent chains (no
// dependency stalls, no memory in the loop) at a chosen occupancy; run under
// `rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE ...`
// (tools/issue_probe.py), SIMD-cycles / SQ_INSTS_VALU is the class's cost per
// wave64 instruction at that occupancy, GRBM_GUI_ACTIVE being the chip's real
// clock (DVFS included). `mix` replays the render's instruction mix (its
// class shares from the render's own PMC pass, bench.py) without memory:
// the rate the render could issue at if nothing but issue held it back.
//
//   ubench_issue [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

#define CHAINS 8

// one instruction class, CHAINS independent chains per lane
template <int W>
__global__ void __launch_bounds__(256, W) k_fma(float *out, int iters, float a, float b) {
    float acc[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = threadIdx.x * 1e-3f + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(acc[c]) : "v"(a), "v"(b));
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += acc[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int W>
__global__ void __launch_bounds__(256, W) k_pkfma(float *out, int iters, float a, float b) {
    f2 acc[CHAINS];
    const f2 av = {a, a}, bv = {b, b};
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = (f2){threadIdx.x * 1e-3f + c, c * 0.5f};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(acc[c]) : "v"(av), "v"(bv));
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += acc[c].x + acc[c].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int W>
__global__ void __launch_bounds__(256, W) k_int(float *out, int iters, float a, float b) {
    unsigned acc[CHAINS];
    const unsigned k = __float_as_uint(a);
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = threadIdx.x + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(acc[c]) : "v"(k));
    }
    unsigned s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += acc[c];
    out[blockIdx.x * 256 + threadIdx.x] = (float)s + b;
}

template <int W>
__global__ void __launch_bounds__(256, W) k_trans(float *out, int iters, float a, float b) {
    float acc[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) asm volatile("v_sqrt_f32 %0, %0" : "+v"(acc[c]));
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += acc[c];
    out[blockIdx.x * 256 + threadIdx.x] = s + a * b;
}

// VALU with one SALU instruction per VALU instruction beside it (the render
// issues ~0.34 SALU per VALU): does scalar issue take VALU slots?
template <int W>
__global__ void __launch_bounds__(256, W) k_fma_salu(float *out, int iters, float a, float b) {
    float acc[CHAINS];
    unsigned s0 = 1u;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = threadIdx.x * 1e-3f + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(acc[c]) : "v"(a), "v"(b));
            asm volatile("s_add_u32 %0, %0, 0x9e3779b9" : "+s"(s0) : : "scc");
        }
    }
    float s = (float)s0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += acc[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

// The render's mix (per 32 VALU instructions: `pk` v_pk_fma_f32, `fm` v_fma_f32,
// `in` integer/logic, `tr` transcendental, the rest v_cndmask_b32 selects) with
// `sa` SALU instructions, all independent; counts are kernel arguments so the
// runner can set them from the render's own counters.
template <int W>
__global__ void __launch_bounds__(256, W) k_mix(float *out, int iters, float a, float b, int pk, int fm, int in,
                                                int tr, int sa) {
    f2 p0 = {threadIdx.x * 1e-3f, 0.5f}, p1 = {0.25f, threadIdx.x * 2e-3f};
    float f0 = threadIdx.x * 1e-3f, f1 = 0.5f, f2v_ = 1.5f, c0 = 0.f, t0 = 2.0f;
    unsigned u0 = threadIdx.x, u1 = 7u, s0 = 1u;
    const f2 av = {a, a}, bv = {b, b};
    const unsigned k = __float_as_uint(a);
    const int sel = 32 - pk - fm - in - tr;
    for (int i = 0; i < iters; ++i) {
        // wave-uniform counts: scalar loops around straight-line bodies (their
        // SALU is part of the measured mix, and is counted by SQ_INSTS_SALU)
        for (int j = 0; j < pk; j += 2) {
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p0) : "v"(av), "v"(bv));
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p1) : "v"(av), "v"(bv));
        }
        for (int j = 0; j < fm; j += 2) {
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f0) : "v"(a), "v"(b));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f1) : "v"(a), "v"(b));
        }
        for (int j = 0; j < in; j += 2) {
            asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(u0) : "v"(k));
            asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(u1) : "v"(k));
        }
        for (int j = 0; j < tr; ++j) asm volatile("v_sqrt_f32 %0, %0" : "+v"(t0));
        for (int j = 0; j < sel; ++j) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(c0) : "v"(f2v_), "v"(a));
        for (int j = 0; j < sa; ++j) asm volatile("s_add_u32 %0, %0, 0x9e3779b9" : "+s"(s0) : : "scc");
    }
    out[blockIdx.x * 256 + threadIdx.x] = p0.x + p0.y + p1.x + p1.y + f0 + f1 + (float)(u0 ^ u1) + t0 + c0 + (float)s0;
}

template <typename K, typename... A>
static void run(const char *name, int w, K kern, int blocks, A... args) {
    float *out;
    (void)hipMalloc(&out, (size_t)blocks * 256 * sizeof(float));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float ms = 0.f;
    for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, args...);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
    }
    std::printf("{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f}\n", name, w, ms);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(out);
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 4000;
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const float a = 0.999f, b = 0.001f;
    // occupancy w: w blocks of 4 waves per CU = w waves per SIMD
    run("fma", 1, k_fma<1>, cus * 1, iters, a, b);
    run("fma", 2, k_fma<2>, cus * 2, iters, a, b);
    run("fma", 5, k_fma<5>, cus * 5, iters, a, b);
    run("fma", 8, k_fma<8>, cus * 8, iters, a, b);
    run("pk_fma", 1, k_pkfma<1>, cus * 1, iters, a, b);
    run("pk_fma", 2, k_pkfma<2>, cus * 2, iters, a, b);
    run("pk_fma", 5, k_pkfma<5>, cus * 5, iters, a, b);
    run("int", 5, k_int<5>, cus * 5, iters, a, b);
    run("trans", 5, k_trans<5>, cus * 5, iters / 4, a, b);
    run("fma_salu", 5, k_fma_salu<5>, cus * 5, iters, a, b);
    // the render's mix (C2 chain render, R9k counters: 42 % of VALU packed fma;
    // fma / int / trans / select shares set by tools/issue_probe.py --mix)
    const int pk = argc > 2 ? std::atoi(argv[2]) : 14, fm = argc > 3 ? std::atoi(argv[3]) : 6,
              in = argc > 4 ? std::atoi(argv[4]) : 6, tr = argc > 5 ? std::atoi(argv[5]) : 0,
              sa = argc > 6 ? std::atoi(argv[6]) : 11;
    run("mix", 5, k_mix<5>, cus * 5, iters / 4, a, b, pk, fm, in, tr, sa);
    return 0;
}
