// bmfr_generic.h -- kernels templated on the feature counts (NS =
// FEATURES_NOT_SCALED, FS = FEATURES_SCALED) with runtime feature codes: the
// stage-2 fitter (bmfr.cl:490-700) and the generic-feature fused K1.  The
// canonical lists run the specialised K1 (bmfr_fused*.hip) instead.
// Instantiated per NS in bmfr_generic_ns*.hip (parallel compilation).
#pragma once

#include "bmfr_kernels.h"
#include "bmfr_launch.h"

namespace bmfr {

// Features recomputed in f32 from normals/positions, scaled with the block's
// min/max, dotted with the block's weights (bmfr.cl:703-758).
__device__ __forceinline__ f3 weighted_color(const Params& P, const float* __restrict__ w,
                                             const float* __restrict__ mm, f3 n, f3 p) {
    f3 c{0.f, 0.f, 0.f};
    for (int f = 0; f < P.buffers - 3; ++f) {
        float v = feature_value(P.codes[f], n, p);
        if (f >= P.not_scaled) v = scale(v, mm[2 * (f - P.not_scaled)], mm[2 * (f - P.not_scaled) + 1]);
        c.x = c.x + w[3 * f] * v;
        c.y = c.y + w[3 * f + 1] * v;
        c.z = c.z + w[3 * f + 2] * v;
    }
    c.x = c.x < 0.f ? 0.f : c.x;
    c.y = c.y < 0.f ? 0.f : c.y;
    c.z = c.z < 0.f ? 0.f : c.z;
    return c;
}

// ---------------------------------------------------------------- stage 2 --
template <int NS, int FS, bool HALF>
__global__ __launch_bounds__(256) void k_fitter(Params P, float* __restrict__ weights,
                                                float* __restrict__ mins_maxs, void* tmp, int frame) {
    constexpr int B = NS + FS + 3;
    __shared__ FitLds<B> L;
    const int t = threadIdx.x, g = blockIdx.x;
    const size_t base = (size_t)g * B * kBlockPixels;
    float a[B][kSubs];
#pragma unroll
    for (int f = 0; f < B; ++f)
#pragma unroll
        for (int s = 0; s < kSubs; ++s) {
            const size_t i = base + (size_t)f * kBlockPixels + t + s * kLocal;
            a[f][s] = HALF ? (float)((const _Float16*)tmp)[i] : ((const float*)tmp)[i];
        }
    fit_block<NS, FS, HALF, true, false>(a, L, t, frame, P.noise2);
#pragma unroll
    for (int f = 0; f < B; ++f)
#pragma unroll
        for (int s = 0; s < kSubs; ++s) {
            const size_t i = base + (size_t)f * kBlockPixels + t + s * kLocal;
            if (HALF) ((_Float16*)tmp)[i] = (_Float16)a[f][s];
            else ((float*)tmp)[i] = a[f][s];
        }
    if (t < (B - 3) * 3) weights[(size_t)g * (B - 3) * 3 + t] = L.weights[t];
    if (t < FS * 2) mins_maxs[(size_t)g * FS * 2 + t] = L.minmax[t];
}

// ------------------------------------------- generic-feature fused K1 ----
// Fallback K1 for feature lists other than the canonical ones (runtime
// feature codes); the canonical lists use k_fused (bmfr_fused.hip).
template <int NS, int FS, bool HALF>
__global__ __launch_bounds__(256) void k_fused_block(Params P, NoisyInputs in, Camera cam, int frame,
                                                     const float* __restrict__ albedo,
                                                     const float* __restrict__ acc_prev,
                                                     float* __restrict__ noisy_out,
                                                     uint8_t* __restrict__ spp_out,
                                                     float2* __restrict__ prev_pixel_out,
                                                     float* __restrict__ acc_out,
                                                     float* __restrict__ tone_out) {
    constexpr int B = NS + FS + 3;
    __shared__ FitLds<B> L;
    const int t = threadIdx.x, g = blockIdx.x;
    const int bx = g % P.blocks_x, by = g / P.blocks_x;

    float a[B][kSubs];
    f3 n_keep[kSubs], p_keep[kSubs];
    float pfx[kSubs], pfy[kSubs];
    uint32_t lin[kSubs];
    uint32_t flags = 0;  // per s: bit 8s owner, bits 8s+1.. accept(4)
    uint32_t spps = 0;
#pragma unroll
    for (int s = 0; s < kSubs; ++s) {
        const int r = t + s * kLocal;
        const int gx = bx * kEdge + (r & (kEdge - 1)), gy = by * kEdge + (r >> 5);
        const NoisyItem it = noisy_item(P, in, cam, gx, gy, frame);
#pragma unroll
        for (int f = 0; f < B; ++f) {
            const float v = design_value(P, f, it);
            a[f][s] = HALF ? round_half(v) : v;
        }
        n_keep[s] = it.n;
        p_keep[s] = it.p;
        pfx[s] = it.pfx;
        pfy[s] = it.pfy;
        lin[s] = it.lin;
        flags |= ((uint32_t)it.owner | ((uint32_t)it.accept << 1)) << (8 * s);
        spps |= (uint32_t)it.spp << (8 * s);
        if (it.owner) {
            st3(noisy_out, it.lin, it.color);
            spp_out[it.lin] = it.spp;
            prev_pixel_out[it.lin] = make_float2(it.pfx, it.pfy);
        }
    }

    fit_block<NS, FS, HALF, false, true>(a, L, t, frame, P.noise2);

#pragma unroll
    for (int s = 0; s < kSubs; ++s) {
        const uint32_t fl = flags >> (8 * s);
        if (fl & 1u) {
            const f3 filtered = weighted_color(P, L.weights, L.minmax, n_keep[s], p_keep[s]);
            const f3 acc = blend_filtered(P, filtered, pfx[s], pfy[s], (uint8_t)((fl >> 1) & 15u),
                                          (uint8_t)(spps >> (8 * s)), acc_prev, frame);
            st3(acc_out, lin[s], acc);
            st3(tone_out, lin[s], tone_map(P, ld3(albedo, lin[s]), acc));
        }
    }
}

template <int NS, int FS>
static hipError_t launch_fitter_t(const Params& P, hipStream_t st, float* w, float* mm, void* tmp,
                                  int frame) {
    const int G = P.blocks_x * P.blocks_y;
    if (P.half_tmp) hipLaunchKernelGGL((k_fitter<NS, FS, true>), dim3(G), dim3(256), 0, st, P, w, mm, tmp, frame);
    else hipLaunchKernelGGL((k_fitter<NS, FS, false>), dim3(G), dim3(256), 0, st, P, w, mm, tmp, frame);
    return hipGetLastError();
}

template <int NS, int FS>
static hipError_t launch_fused_t(const Params& P, hipStream_t st, const FusedArgs& A) {
    const int G = P.blocks_x * P.blocks_y;
    if (P.half_tmp)
        hipLaunchKernelGGL((k_fused_block<NS, FS, true>), dim3(G), dim3(256), 0, st, P, A.in, A.cam,
                           A.frame, A.albedo, A.acc_prev, A.noisy_out, A.spp_out, A.prev_pixel_out,
                           A.acc_out, A.tone_out);
    else
        hipLaunchKernelGGL((k_fused_block<NS, FS, false>), dim3(G), dim3(256), 0, st, P, A.in, A.cam,
                           A.frame, A.albedo, A.acc_prev, A.noisy_out, A.spp_out, A.prev_pixel_out,
                           A.acc_out, A.tone_out);
    return hipGetLastError();
}

// Entry points per FEATURES_NOT_SCALED: FEATURES_SCALED 0..9 dispatched at
// run time (defined in bmfr_generic_ns<NS>.hip).
template <int NS>
hipError_t launch_fitter_ns(const Params& P, hipStream_t st, float* w, float* mm, void* tmp, int frame);
template <int NS>
hipError_t launch_fused_block_ns(const Params& P, hipStream_t st, const FusedArgs& A);
#define BMFR_DECLARE_NS(N)                                                                                  \
    template <>                                                                                             \
    hipError_t launch_fitter_ns<N>(const Params& P, hipStream_t st, float* w, float* mm, void* tmp, int frame); \
    template <>                                                                                             \
    hipError_t launch_fused_block_ns<N>(const Params& P, hipStream_t st, const FusedArgs& A);
BMFR_DECLARE_NS(1)
BMFR_DECLARE_NS(2)
BMFR_DECLARE_NS(3)
BMFR_DECLARE_NS(4)
#undef BMFR_DECLARE_NS

#ifdef BMFR_GENERIC_NS
template <>
hipError_t launch_fitter_ns<BMFR_GENERIC_NS>(const Params& P, hipStream_t st, float* w, float* mm, void* tmp,
                                             int frame) {
    constexpr int NS = BMFR_GENERIC_NS;
    switch (P.scaled) {
        case 0: return launch_fitter_t<NS, 0>(P, st, w, mm, tmp, frame);
        case 1: return launch_fitter_t<NS, 1>(P, st, w, mm, tmp, frame);
        case 2: return launch_fitter_t<NS, 2>(P, st, w, mm, tmp, frame);
        case 3: return launch_fitter_t<NS, 3>(P, st, w, mm, tmp, frame);
        case 4: return launch_fitter_t<NS, 4>(P, st, w, mm, tmp, frame);
        case 5: return launch_fitter_t<NS, 5>(P, st, w, mm, tmp, frame);
        case 6: return launch_fitter_t<NS, 6>(P, st, w, mm, tmp, frame);
        case 7: return launch_fitter_t<NS, 7>(P, st, w, mm, tmp, frame);
        case 8: return launch_fitter_t<NS, 8>(P, st, w, mm, tmp, frame);
        case 9: return launch_fitter_t<NS, 9>(P, st, w, mm, tmp, frame);
        default: return hipErrorInvalidValue;
    }
}

template <>
hipError_t launch_fused_block_ns<BMFR_GENERIC_NS>(const Params& P, hipStream_t st, const FusedArgs& A) {
    constexpr int NS = BMFR_GENERIC_NS;
    switch (P.scaled) {
        case 0: return launch_fused_t<NS, 0>(P, st, A);
        case 1: return launch_fused_t<NS, 1>(P, st, A);
        case 2: return launch_fused_t<NS, 2>(P, st, A);
        case 3: return launch_fused_t<NS, 3>(P, st, A);
        case 4: return launch_fused_t<NS, 4>(P, st, A);
        case 5: return launch_fused_t<NS, 5>(P, st, A);
        case 6: return launch_fused_t<NS, 6>(P, st, A);
        case 7: return launch_fused_t<NS, 7>(P, st, A);
        case 8: return launch_fused_t<NS, 8>(P, st, A);
        case 9: return launch_fused_t<NS, 9>(P, st, A);
        default: return hipErrorInvalidValue;
    }
}
#endif

}  // namespace bmfr
