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
    (void)hipFree(out);
    return 0;
}
