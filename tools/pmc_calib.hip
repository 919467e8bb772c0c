// pmc_calib.hip -- known-byte-count read/write kernels for calibrating
// rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 in the access widths K1 and
// K2 use (MI355X_MICROARCH.md: "other access widths are uncalibrated").
// Built by tools/pmc_calibrate.py; each kernel touches exactly `bytes` bytes.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "../bmfr_amd/csrc/bmfr_device.h"

namespace {
__global__ void k_read4(const float4* __restrict__ src, long n, float* __restrict__ sink) {
    long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    float acc = 0.f;
    for (; i < n; i += (long)gridDim.x * blockDim.x) {
        const float4 v = src[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 123.456f) sink[0] = acc;
}
__global__ void k_read3(const float* __restrict__ src, long n, float* __restrict__ sink) {
    long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    float acc = 0.f;
    for (; i < n; i += (long)gridDim.x * blockDim.x) {
        const bmfr::f3 v = bmfr::ld3(src, i);
        acc += v.x + v.y + v.z;
    }
    if (acc == 123.456f) sink[0] = acc;
}
__global__ void k_read1(const uint8_t* __restrict__ src, long n, float* __restrict__ sink) {
    long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (; i < n; i += (long)gridDim.x * blockDim.x) acc += src[i];
    if (acc == 0xdeadbeefu) sink[0] = (float)acc;
}
__global__ void k_write3(float* __restrict__ dst, long n) {
    long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    for (; i < n; i += (long)gridDim.x * blockDim.x) bmfr::st3(dst, i, bmfr::f3{1.f, 2.f, 3.f});
}
__global__ void k_write1(uint8_t* __restrict__ dst, long n) {
    long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    for (; i < n; i += (long)gridDim.x * blockDim.x) dst[i] = (uint8_t)i;
}
}  // namespace

extern "C" int calib_run(int kind, void* buf, long bytes, float* sink) {
    const dim3 grid(8192), block(256);
    switch (kind) {
        case 0: hipLaunchKernelGGL(k_read4, grid, block, 0, 0, (const float4*)buf, bytes / 16, sink); break;
        case 1: hipLaunchKernelGGL(k_read3, grid, block, 0, 0, (const float*)buf, bytes / 12, sink); break;
        case 2: hipLaunchKernelGGL(k_read1, grid, block, 0, 0, (const uint8_t*)buf, bytes, sink); break;
        case 3: hipLaunchKernelGGL(k_write3, grid, block, 0, 0, (float*)buf, bytes / 12); break;
        case 4: hipLaunchKernelGGL(k_write1, grid, block, 0, 0, (uint8_t*)buf, bytes); break;
        default: return -1;
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}
