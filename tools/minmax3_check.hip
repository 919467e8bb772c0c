// Exhaustive-ish check that v_min3_f32 / v_max3_f32 equal the nested
// v_min_f32 / v_max_f32 chains bit for bit (incl. signed zeros, infinities,
// quiet NaNs, denormals) on gfx950 -- the property K2's TAA relies on.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

__device__ float f_min(float a, float b) { float r; asm volatile("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
__device__ float f_max(float a, float b) { float r; asm volatile("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
__device__ float f_min3(float a, float b, float c) { float r; asm volatile("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c)); return r; }
__device__ float f_max3(float a, float b, float c) { float r; asm volatile("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c)); return r; }

__global__ void k(const float* v, int n, unsigned long long* bad) {
    const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    const long total = (long)n * n * n;
    if (i >= total) return;
    const float a = v[i % n], b = v[(i / n) % n], c = v[i / ((long)n * n)];
    const float m1 = f_min(f_min(a, b), c), m3 = f_min3(a, b, c);
    const float x1 = f_max(f_max(a, b), c), x3 = f_max3(a, b, c);
    if (__float_as_uint(m1) != __float_as_uint(m3)) atomicAdd(bad, 1ull);
    if (__float_as_uint(x1) != __float_as_uint(x3)) atomicAdd(bad + 1, 1ull);
}

int main() {
    std::vector<float> v;
    const uint32_t specials[] = {0x00000000u, 0x80000000u, 0x7f800000u, 0xff800000u, 0x7fc00000u, 0xffc00000u,
                                 0x00000001u, 0x80000001u, 0x007fffffu, 0x3f800000u, 0xbf800000u, 0x7f7fffffu};
    for (uint32_t s : specials) { float f; std::memcpy(&f, &s, 4); v.push_back(f); }
    uint32_t x = 12345;
    while (v.size() < 400) { x = x * 1664525u + 1013904223u; float f; std::memcpy(&f, &x, 4); if (f == f) v.push_back(f); }
    const int n = (int)v.size();
    float* dv; unsigned long long* bad;
    (void)hipMalloc(&dv, n * 4); (void)hipMalloc(&bad, 16);
    (void)hipMemcpy(dv, v.data(), n * 4, hipMemcpyHostToDevice); (void)hipMemset(bad, 0, 16);
    const long total = (long)n * n * n;
    hipLaunchKernelGGL(k, dim3((total + 255) / 256), dim3(256), 0, 0, dv, n, bad);
    unsigned long long h[2];
    (void)hipMemcpy(h, bad, 16, hipMemcpyDeviceToHost);
    printf("%ld triples (incl. +-0, +-inf, qNaN, denormals): min3 mismatches %llu, max3 mismatches %llu\n", total, h[0], h[1]);
    return (h[0] || h[1]) ? 1 : 0;
}
