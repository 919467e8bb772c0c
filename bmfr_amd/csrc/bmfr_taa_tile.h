// K2's tile body (fused TAA, bmfr.cl:860-974, with the tone map of
// bmfr.cl:851-856 when TONE): one 64 x TH output tile per 256-thread
// work-group.  The tile's tone-mapped colours and a 1-pixel halo go to LDS
// (Y) once as YCoCg, and the 3x3 neighbourhoods (bmfr.cl:897-920) are read
// from there; each thread keeps the RGB of its own TH / 4 output pixels in
// registers.  Shared by k_fused_taa (bmfr_kernels.hip) and the sequence
// kernel k_fused_cols_taa (bmfr_fused_cols.hip).
#pragma once

#include "bmfr_kernels.h"

namespace bmfr {

struct TaaArgs {
    const float* src;         // accumulated filtered colour (TONE) or K1's tone-mapped frame
    const float* albedo;      // float3 or half3 (IN)
    const float2* prev_pixel;
    float* result;
    const float* prev_frame;  // previous TAA output
    int frame;
};

#ifndef BMFR_K2_EARLY_TAPS  // previous-frame taps loaded before the tone map
#define BMFR_K2_EARLY_TAPS 1
#endif
#ifndef BMFR_K2_SHARE_TAPS  // right-hand taps taken from the next lane's left-hand taps when they coincide
#define BMFR_K2_SHARE_TAPS 0  // measured slower: K2 0.131 vs 0.109 ms (the lane moves and the serialised fallback)
#endif

// taa_load_taps for a wave whose lane l + 1 holds the pixel right of lane
// l's: the previous-frame taps (ix + 1, iy) and (ix + 1, iy + 1) of lane l
// are lane l + 1's (ix, iy) and (ix, iy + 1) whenever the clamped addresses
// coincide (the same whole-pixel motion), and are then moved across lanes
// instead of loaded again; the other lanes (always lane 63) load them.  The
// values are the same loads' values: bit-identical to taa_load_taps.
__device__ __forceinline__ void taa_load_taps_shared(const Params& P, float2 pf, const float* __restrict__ prev_frame,
                                                     f3 (&pc)[4]) {
    const int ix = (int)fminf(fmaxf(floorf(pf.x), -2.f), (float)P.width + 1.f);
    const int iy = (int)fminf(fmaxf(floorf(pf.y), -2.f), (float)P.height + 1.f);
    const int xa = clamp_rx(P, ix), xb = clamp_rx(P, ix + 1), ya = clamp_ry(P, iy), yb = clamp_ry(P, iy + 1);
    const int lane = __lane_id();
    const int nxa = __shfl_down(xa, 1, 64), nya = __shfl_down(ya, 1, 64), nyb = __shfl_down(yb, 1, 64);
    const bool own = lane == 63 || nxa != xb || nya != ya || nyb != yb;  // this lane loads its right-hand taps
    pc[0] = ld3(prev_frame, pix(P, xa, ya));
    pc[2] = ld3(prev_frame, pix(P, xa, yb));
    if (own) {
        pc[1] = ld3(prev_frame, pix(P, xb, ya));
        pc[3] = ld3(prev_frame, pix(P, xb, yb));
    }
    const f3 r0{__shfl_down(pc[0].x, 1, 64), __shfl_down(pc[0].y, 1, 64), __shfl_down(pc[0].z, 1, 64)};
    const f3 r2{__shfl_down(pc[2].x, 1, 64), __shfl_down(pc[2].y, 1, 64), __shfl_down(pc[2].z, 1, 64)};
    if (!own) {
        pc[1] = r0;
        pc[3] = r2;
    }
}

// Y: (64 + 2) * (TH + 2) float4; sE / sRP: the powr tables' LDS copies (TONE).
template <bool TONE, class IN, int TH>
__device__ __forceinline__ void taa_tile(const Params& P, const TaaArgs& T, int x0, int y0, float4* __restrict__ Y,
                                         double* __restrict__ sE, double2* __restrict__ sRP) {
    static_assert(TH % 4 == 0 && TH >= 4, "tile height");
    constexpr int HW = 64 + 2, HH = TH + 2, N = HW * HH;
    constexpr int RING = N - 64 * TH;  // halo pixels
    constexpr int KN = TH / 4;         // output pixels per thread
    static_assert(RING <= 256, "one ring pixel per thread");
    const int t = threadIdx.x;
    if constexpr (TONE) bmfr_powr_tables_to_lds<256>(sE, sRP, t);
    const int tx = t & (64 - 1), ty = t >> 6;
    // Reprojected positions first, then the tile and its ring behind them.
    float2 pf[KN];
#pragma unroll
    for (int k = 0; k < KN; ++k)
        pf[k] = T.prev_pixel[pix(P, min(x0 + tx, P.tx1 - 1), min(y0 + ty + 4 * k, P.ty1 - 1))];
    f3 v[KN + 1], al[KN + 1];
    int hx = 0, hy = 0;  // this thread's ring pixel (t < RING), in tile + halo coordinates
    if (t < 2 * HW) {
        hx = t % HW;
        hy = t < HW ? 0 : HH - 1;
    } else {
        hx = t < 2 * HW + TH ? 0 : HW - 1;
        hy = 1 + (t - 2 * HW) % TH;
    }
#pragma unroll
    for (int k = 0; k <= KN; ++k) {
        const int lx = k < KN ? tx + 1 : hx, ly = k < KN ? ty + 4 * k + 1 : hy;
        if (k == KN && t >= RING) break;
        const long lin = pix(P, min(max(x0 - 1 + lx, 0), P.width - 1), min(max(y0 - 1 + ly, 0), P.height - 1));
        v[k] = ld3(T.src, lin);
        if (TONE) al[k] = ld3in<IN>(T.albedo, lin);
    }
    f3 taps[KN][4];
    if constexpr (BMFR_K2_EARLY_TAPS) {
#pragma unroll
        for (int k = 0; k < KN; ++k) {
            if constexpr (BMFR_K2_SHARE_TAPS) taa_load_taps_shared(P, pf[k], T.prev_frame, taps[k]);
            else taa_load_taps(P, pf[k], T.prev_frame, taps[k]);
        }
    }
    if constexpr (TONE) __syncthreads();  // the powr tables are in LDS
#pragma unroll
    for (int k = 0; k <= KN; ++k) {
        if (k == KN && t >= RING) break;
        const int lx = k < KN ? tx + 1 : hx, ly = k < KN ? ty + 4 * k + 1 : hy;
        v[k] = TONE ? tone_map(P, al[k], v[k], sE, sRP) : v[k];
        const f3 yc = rgb_to_ycocg(v[k]);
        Y[ly * HW + lx] = make_float4(yc.x, yc.y, yc.z, 0.f);
    }
    __syncthreads();
    if constexpr (!BMFR_K2_EARLY_TAPS) {
#pragma unroll
        for (int k = 0; k < KN; ++k) {
            if constexpr (BMFR_K2_SHARE_TAPS) taa_load_taps_shared(P, pf[k], T.prev_frame, taps[k]);
            else taa_load_taps(P, pf[k], T.prev_frame, taps[k]);
        }
    }
    // Tiles that reach the image border check every neighbour (bmfr.cl:901);
    // the others have all nine in the image.
    const bool edge = x0 == 0 || y0 == 0 || x0 + 64 >= P.width || y0 + TH >= P.height;
#pragma unroll
    for (int k = 0; k < KN; ++k) {
        const int x = x0 + tx, y = y0 + ty + 4 * k;
        if (x < P.tx1 && y < P.ty1) {
            const int c = (ty + 4 * k + 1) * HW + tx + 1;
            f3 nb[9];
#pragma unroll
            for (int j = 0; j < 9; ++j) {
                const float4 q = Y[c + (j / 3 - 1) * HW + (j % 3 - 1)];
                nb[j] = f3{q.x, q.y, q.z};
            }
            const f3 r = edge ? taa_resolve<true>(P, x, y, v[k], pf[k], nb, taps[k], T.frame)
                              : taa_resolve<false>(P, x, y, v[k], pf[k], nb, taps[k], T.frame);
            st3(T.result, pix(P, x, y), r);
        }
    }
}

}  // namespace bmfr
