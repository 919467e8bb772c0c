// Microbenchmark: VALU issue rate of v_fma_f32 vs v_pk_fma_f32 (wave64, gfx950).
// Each thread runs N iterations of 8 independent FMA chains; time per kernel
// gives wave-instructions per cycle per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>

typedef float float2v __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_fma(float* out, int n, float a, float b) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_pkfma(float* out, int n, float a, float b) {
    float2v x[8];
    for (int i = 0; i < 8; ++i) x[i] = float2v{threadIdx.x * 0.001f + i, 1.f + i};
    float2v av = {a, a}, bv = {b, b};
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(av), "v"(bv));
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_mix(float* out, int n, float a, float b) {
    float x[8];
    _Float16 h = (_Float16)a;
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_fma_mix_f32 %0, %1, %0, %2 op_sel_hi:[1,0,0]" : "+v"(x[i]) : "v"(h), "v"(b));
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    int dev = 0;
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, dev);
    const int cus = p.multiProcessorCount;
    float* out;
    (void)hipMalloc(&out, sizeof(float) * 256 * cus * 64);
    const int n = 4096;
    for (int waves_per_simd = 1; waves_per_simd <= 8; waves_per_simd *= 2) {
        const int blocks = cus * waves_per_simd;  // 256 threads = 4 waves = 1 per SIMD
        for (int k = 0; k < 3; ++k) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            for (int rep = 0; rep < 2; ++rep) {
                (void)hipEventRecord(e0);
                if (k == 0) hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, out, n, 1.0001f, 0.5f);
                if (k == 1) hipLaunchKernelGGL(k_pkfma, dim3(blocks), dim3(256), 0, 0, out, n, 1.0001f, 0.5f);
                if (k == 2) hipLaunchKernelGGL(k_mix, dim3(blocks), dim3(256), 0, 0, out, n, 1.0001f, 0.5f);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
            }
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double instr_per_simd = (double)n * 8 * waves_per_simd;  // wave-instructions per SIMD
            const double ghz = 2.4;
            printf("%-8s waves/SIMD %d: %.3f ms, %.2f cycles per wave-instruction per SIMD (at %.1f GHz)\n",
                   k == 0 ? "fma" : k == 1 ? "pk_fma" : "fma_mix", waves_per_simd, ms,
                   ms * 1e-3 * ghz * 1e9 / instr_per_simd, ghz);
        }
    }
    return 0;
}
