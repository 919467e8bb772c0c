// Exhaustive check of gamma_clamped (bmfr_amd/csrc/bmfr_powr.h) against the
// CPU oracle's (float)pow((double)x, (double)0.454545f) over every
// non-negative float below 1.5, plus the device library's powr for
// comparison.  Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off
//   -I bmfr_amd/csrc tools/powr_check.hip -o tools/powr_check -lpthread
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "bmfr_powr.h"

extern "C" __device__ float __ocml_powr_f32(float, float);

__global__ void k_eval(uint32_t first, uint32_t n, float* fast, float* lib) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = __uint_as_float(first + i);
    fast[i] = gamma_clamped(x);
    lib[i] = fminf(fmaxf(__ocml_powr_f32(fmaxf(0.f, x), 0.454545f), 0.f), 1.f);
}

static float oracle(float x) {
    return fminf(fmaxf((float)pow((double)fmaxf(0.f, x), (double)0.454545f), 0.f), 1.f);
}

int main() {
    const uint32_t end = 0x3FC00000u;  // 1.5f
    const uint32_t chunk = 1u << 26;
    float *dfast, *dlib;
    if (hipMalloc(&dfast, chunk * 4) || hipMalloc(&dlib, chunk * 4)) return 2;
    std::vector<float> fast(chunk), lib(chunk);
    unsigned nthr = 16;
    long long bad_fast = 0, bad_lib = 0;
    int shown = 0;
    for (uint32_t first = 0; first < end; first += chunk) {
        const uint32_t n = end - first < chunk ? end - first : chunk;
        k_eval<<<(n + 255) / 256, 256>>>(first, n, dfast, dlib);
        if (hipMemcpy(fast.data(), dfast, n * 4, hipMemcpyDeviceToHost) ||
            hipMemcpy(lib.data(), dlib, n * 4, hipMemcpyDeviceToHost)) return 3;
        std::vector<long long> bf(nthr), bl(nthr);
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nthr; ++t)
            th.emplace_back([&, t] {
                for (uint32_t i = t; i < n; i += nthr) {
                    float x;
                    const uint32_t bits = first + i;
                    std::memcpy(&x, &bits, 4);
                    const float o = oracle(x);
                    if (std::memcmp(&o, &fast[i], 4)) ++bf[t];
                    if (std::memcmp(&o, &lib[i], 4)) ++bl[t];
                }
            });
        for (auto& t : th) t.join();
        for (unsigned t = 0; t < nthr; ++t) bad_fast += bf[t], bad_lib += bl[t];
        for (uint32_t i = 0; i < n && shown < 10; ++i) {
            float x;
            const uint32_t bits = first + i;
            std::memcpy(&x, &bits, 4);
            const float o = oracle(x);
            if (std::memcmp(&o, &fast[i], 4)) {
                std::printf("mismatch x=%a fast=%a oracle=%a\n", x, fast[i], o);
                ++shown;
            }
        }
        std::printf("[0x%08x..0x%08x) fast mismatches so far %lld, device powr mismatches %lld\n", first,
                    first + n, bad_fast, bad_lib);
        std::fflush(stdout);
    }
    std::printf("inputs %u  gamma_clamped != oracle: %lld  __ocml_powr_f32 != oracle: %lld\n", end, bad_fast,
                bad_lib);
    return bad_fast ? 1 : 0;
}
