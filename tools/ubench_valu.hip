// ubench_valu.hip — measured FP32 VALU ceiling on this MI355X, to price the
// roofline's compute peak: independent FMA chains, scalar v_fma_f32 vs
// packed v_pk_fma_f32, 256-thread blocks, 8 blocks per CU.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float float2v __attribute__((ext_vector_type(2)));

template <int CHAINS>
__global__ void __launch_bounds__(256) k_fma(float *out, int iters, float a, float b) {
    float acc[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = threadIdx.x * 1e-3f + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c)
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(acc[c]) : "v"(a), "v"(b));
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += acc[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int CHAINS>
__global__ void __launch_bounds__(256) k_pkfma(float *out, int iters, float a, float b) {
    float2v acc[CHAINS];
    const float2v av = {a, a}, bv = {b, b};
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = (float2v){threadIdx.x * 1e-3f + c, c * 0.5f};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_elementwise_fma(acc[c], av, bv);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += acc[c].x + acc[c].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

typedef _Float16 half2v __attribute__((ext_vector_type(2)));
template <int CHAINS>
__global__ void __launch_bounds__(256) k_pkfma16(float *out, int iters, float a, float b) {
    half2v acc[CHAINS];
    const half2v av = {(_Float16)a, (_Float16)a}, bv = {(_Float16)b, (_Float16)b};
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = (half2v){(_Float16)(threadIdx.x * 1e-3f + c), (_Float16)(c * 0.5f)};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_elementwise_fma(acc[c], av, bv);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += (float)acc[c].x + (float)acc[c].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

// The render scan's own step on synthetic data (the issue
// ceiling of the kernel's mix): per 8-sphere block, 4 sphere pairs of the
// flat-run test (pu = fma(cx, ux, fma(cz, uz, ku)); pv = fma(cz, vz, kv);
// q = fma(-pv, pv, fma(-pu, pu, R)): 5 v_pk_fma_f32 per pair) with the block
// operands wave-uniform, then the max chain (v_max3) and a compare; no memory.
// 5 waves per SIMD like the render (256-thread blocks, 5 per CU).
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(256, 5) k_scanmix(float *out, int iters, const float *blk) {
    const float t = threadIdx.x * 1e-3f;
    const f2 ux = {0.3f + t, 0.3f + t}, uz = {0.5f - t, 0.5f - t}, vz = {0.7f, 0.7f};
    const f2 ku = {t, t}, kv = {-t, -t};
    float acc = 0.f;
    for (int i = 0; i < iters; ++i) {
        const float *b = blk + 32 * (i & 7);  // wave-uniform: scalar loads, cache-resident
        f2 q[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const f2 cx = {b[2 * p], b[2 * p + 1]}, cz = {b[16 + 2 * p], b[17 + 2 * p]}, R = {b[24 + 2 * p], b[25 + 2 * p]};
            const f2 pu = __builtin_elementwise_fma(cx, ux, __builtin_elementwise_fma(cz, uz, ku));
            const f2 pv = __builtin_elementwise_fma(cz, vz, kv);
            q[p] = __builtin_elementwise_fma(-pv, pv, __builtin_elementwise_fma(-pu, pu, R));
        }
        const float mx = fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(q[0].x, q[0].y), q[1].x), q[1].y), q[2].x), q[2].y),
                                     q[3].x), q[3].y);
        acc += mx > 0.0f ? 1.0f : 0.0f;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// The same step over two blocks per wait (both blocks' scalar loads issued
// together, one s_waitcnt per two blocks): does the per-block wait set the
// scan's rate?
__global__ void __launch_bounds__(256, 5) k_scanmix2(float *out, int iters, const float *blk) {
    const float t = threadIdx.x * 1e-3f;
    const f2 ux = {0.3f + t, 0.3f + t}, uz = {0.5f - t, 0.5f - t}, vz = {0.7f, 0.7f};
    const f2 ku = {t, t}, kv = {-t, -t};
    float acc = 0.f;
    for (int i = 0; i < iters; i += 2) {
        float m2[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float *b = blk + 32 * ((i + h) & 7);
            f2 q[4];
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const f2 cx = {b[2 * p], b[2 * p + 1]}, cz = {b[16 + 2 * p], b[17 + 2 * p]},
                         R = {b[24 + 2 * p], b[25 + 2 * p]};
                const f2 pu = __builtin_elementwise_fma(cx, ux, __builtin_elementwise_fma(cz, uz, ku));
                const f2 pv = __builtin_elementwise_fma(cz, vz, kv);
                q[p] = __builtin_elementwise_fma(-pv, pv, __builtin_elementwise_fma(-pu, pu, R));
            }
            m2[h] = fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(q[0].x, q[0].y), q[1].x), q[1].y), q[2].x), q[2].y),
                                q[3].x), q[3].y);
        }
        acc += (m2[0] > 0.0f ? 1.0f : 0.0f) + (m2[1] > 0.0f ? 1.0f : 0.0f);
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int blocks = p.multiProcessorCount * 8, iters = 20000;
    float *out;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
        float ms;
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_fma<8>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f, 0.001f);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double fl = 2.0 * 8 * iters * (double)blocks * 256;
        std::printf("{\"kernel\": \"v_fma_f32 x8 chains\", \"cus\": %d, \"ms\": %.3f, \"tflops\": %.2f}\n",
                    p.multiProcessorCount, ms, fl / ms / 1e9);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_pkfma<8>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f, 0.001f);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double fl2 = 2.0 * 16 * iters * (double)blocks * 256;
        std::printf("{\"kernel\": \"v_pk_fma_f32 x8 chains\", \"cus\": %d, \"ms\": %.3f, \"tflops\": %.2f}\n",
                    p.multiProcessorCount, ms, fl2 / ms / 1e9);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_pkfma16<8>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f, 0.001f);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        std::printf("{\"kernel\": \"v_pk_fma_f16 x8 chains\", \"cus\": %d, \"ms\": %.3f, \"tflops\": %.2f}\n",
                    p.multiProcessorCount, ms, fl2 / ms / 1e9);
    }
    {  // the scan step's mix at the render's occupancy
        float *blk;
        (void)hipMalloc(&blk, 8 * 32 * sizeof(float));
        float h[8 * 32];
        for (int i = 0; i < 8 * 32; ++i) h[i] = 0.01f * (float)(i % 29) - 0.1f;
        (void)hipMemcpy(blk, h, sizeof(h), hipMemcpyHostToDevice);
        const int sblocks = p.multiProcessorCount * 5, sit = 4000;
        for (int rep = 0; rep < 3; ++rep) {
            float ms;
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k_scanmix, dim3(sblocks), dim3(256), 0, 0, out, sit, blk);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            // per wave-iteration: 20 v_pk_fma_f32 + 4 max + 1 cmp/cndmask (+ the loop's scalar work)
            const double wave_iters = (double)sblocks * 4 * sit;
            const double simd_cycles = ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4;
            std::printf("{\"kernel\": \"scan step mix (20 pk_fma + ~6 VALU per block), 5 waves/SIMD\", \"ms\": %.3f, "
                        "\"simd_cycles_per_wave_block_at_2.4GHz\": %.1f}\n",
                        ms, simd_cycles / wave_iters);
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k_scanmix2, dim3(sblocks), dim3(256), 0, 0, out, sit, blk);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            std::printf("{\"kernel\": \"scan step mix, two blocks per scalar wait\", \"ms\": %.3f, "
                        "\"simd_cycles_per_wave_block_at_2.4GHz\": %.1f}\n",
                        ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / wave_iters);
        }
        (void)hipFree(blk);
    }
    (void)hipFree(out);
    return 0;
}
