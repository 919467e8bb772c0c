// bmfr_kernels.h -- device building blocks shared by the stage kernels and
// the fused frame kernels (bmfr_kernels.hip).
//
// Fitter work decomposition: one 256-thread work-group per 32x32 block, as
// upstream (bmfr.cl:487-501), but the block's whole design matrix lives in
// VGPRs: thread t owns rows t + 256*s (s = 0..3) of every column, i.e. the
// rows upstream work-item t touches, so the per-thread partial sums and the
// 256->64->8->1 reduction tree can be reproduced in the reference's exact
// association while tmp_data is read from HBM once instead of once per
// Householder column (bmfr.cl:555-656 re-reads it every pass).
#pragma once

#include "bmfr_device.h"
#include "bmfr_powr.h"

namespace bmfr {

// --------------------------------------------------------------------------
// Batched block reductions with the association of bmfr.cl:25-87.
// `v[k]` is work-item t's partial of reduction k (k < n, n <= K).  The result
// of reduction k lands in res[k]; all threads may read it on return.
// --------------------------------------------------------------------------
enum class RedOp { Sum, Max, Min };

template <RedOp OP>
__device__ __forceinline__ float red(float a, float b) {
    if constexpr (OP == RedOp::Sum) return a + b;
    else if constexpr (OP == RedOp::Max) return fmaxf(a, b);
    else return fminf(a, b);
}

template <RedOp OP>
__device__ __forceinline__ float bcast_lane(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

template <RedOp OP, int K>
__device__ __forceinline__ void block_reduce(const float (&v)[K], int n, float* __restrict__ part,
                                             float* __restrict__ res, int t) {
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (k < n) part[k * kLocal + t] = v[k];
    __syncthreads();
    const int w = t >> 6, l = t & 63;
#pragma unroll
    for (int i = 0; i < (K + 3) / 4; ++i) {
        const int k = w + 4 * i;
        if (k < n) {  // wave-uniform
            const float* p = part + k * kLocal;
            // 256 -> 64 (bmfr.cl:32-33 / 51-53 / 73-75)
            float s;
            if constexpr (OP == RedOp::Sum) s = p[l] + ((p[l + 64] + p[l + 128]) + p[l + 192]);
            else s = red<OP>(red<OP>(red<OP>(p[l], p[l + 64]), p[l + 128]), p[l + 192]);
            // 64 -> 8 (bmfr.cl:35-37 / 55-58 / 77-80), computed on lanes 0..7
            float e;
            if constexpr (OP == RedOp::Sum) {
                float acc = __shfl(s, (l + 8) & 63);
#pragma unroll
                for (int j = 2; j < 8; ++j) acc = acc + __shfl(s, (l + 8 * j) & 63);
                e = s + acc;
            } else {
                e = s;
#pragma unroll
                for (int j = 1; j < 8; ++j) e = red<OP>(e, __shfl(s, (l + 8 * j) & 63));
            }
            // 8 -> 1 (bmfr.cl:39-42), left to right
            float r = bcast_lane<OP>(e, 0);
#pragma unroll
            for (int j = 1; j < 8; ++j) r = red<OP>(r, bcast_lane<OP>(e, j));
            if (l == 0) res[k] = r;
        }
    }
    __syncthreads();
}

// --------------------------------------------------------------------------
// accumulate_noisy_data for one work-item of the margin grid (bmfr.cl:310-476).
// --------------------------------------------------------------------------
struct NoisyItem {
    f3 n, p;          // current normal / world position of the (mirrored) pixel
    f3 color;         // blended colour (features B-3..B-1)
    float pfx, pfy;   // prev_frame_pixel_f
    uint32_t lin;     // linear (mirrored) pixel
    uint8_t accept;
    uint8_t spp;
    bool owner;       // pixel_without_mirror inside the image
    // noisy_item_spec<true> only: the previous accumulated filtered colour
    // at the same taps, as accumulate_filtered_data sums it (bmfr.cl:786-842)
    // -- prev_f, divided by the tap weight sum when that is > 0; the blend
    // acc = alpha_f * filtered + (1 - alpha_f) * prev_f with alpha_f from the
    // new spp happens where the filtered colour is known (phase 3).
    f3 prev_f;
    bool prev_f_divided;  // the tap weights summed to > 0 (alpha_f from spp)
    int over;             // noisy_item_spec, P.check_reach: px by which an in-image tap leaves [vx0, vx1) x [vy0, vy1)
                          // ([wx0, wx1) x [wy0, wy1) for a pixel of the output tile)
};

struct NoisyInputs {
    const float* __restrict__ n_cur;
    const float* __restrict__ n_prev;
    const float* __restrict__ p_cur;
    const float* __restrict__ p_prev;
    const float* noisy_cur;  // may alias the stage kernel's output (in-place, bmfr.cl:297)
    const float* __restrict__ noisy_prev;
    const uint8_t* __restrict__ spp_prev;
};

struct Camera {
    float m[16];   // previous frame's VP, column-major
    float jx, jy;  // this frame's pixel offset
};

// XCD-aware work-group order.  Work-groups are dealt round-robin to the 8
// XCDs (g % 8), each with its own L2; renumbering so that XCD x gets the
// contiguous range [x*G/8, (x+1)*G/8) keeps neighbouring blocks -- which
// share cache lines of every plane and of the reprojection taps -- on one
// L2.  A bijection on [0, G) for any G; placement only affects speed.
__device__ __forceinline__ int xcd_swizzle(int g, int G) {
    constexpr int kXcds = 8;
    const int xcd = g % kXcds, k = g / kXcds;
    const int per = G / kXcds, rem = G % kXcds;
    return xcd < rem ? xcd * (per + 1) + k : rem * (per + 1) + (xcd - rem) * per + k;
}

// Block (bx, by) of K1 work-group g: row-major over the launch rectangle, or
// (ring launches) over its part outside the inner rectangle -- full rows
// above it, the left and right pieces of the rows beside it, full rows below.
__device__ __forceinline__ void k1_block(const Params& P, int g, int& bx, int& by) {
    if (P.ring == 0) {
        bx = P.bx0 + g % P.nbx;
        by = P.by0 + g / P.nbx;
        return;
    }
    const int W = P.nbx;
    const int top = (P.ry0 - P.by0) * W;
    if (g < top) {
        bx = P.bx0 + g % W;
        by = P.by0 + g / W;
        return;
    }
    g -= top;
    const int lw = P.rx0 - P.bx0, rw = P.bx0 + W - P.rx1, per_row = lw + rw, mid = (P.ry1 - P.ry0) * per_row;
    if (g < mid) {
        const int k = g % per_row;
        by = P.ry0 + g / per_row;
        bx = k < lw ? P.bx0 + k : P.rx1 + (k - lw);
        return;
    }
    g -= mid;
    bx = P.bx0 + g % W;
    by = P.ry1 + g / W;
}

// Linear index of image pixel (x, y) in a plane of the buffer region, and
// clamps into the region (= the image when untiled).
// (y - oy) and the stride are below 2^24 for every valid context (a plane is
// at most 4 GiB and at least 32 pixels high, validate() in bmfr_capi.hip), so
// the row offset is one 24-bit multiply-add (v_mad_u32_u24, full rate).
__device__ __forceinline__ uint32_t pix(const Params& P, int x, int y) {
    return __umul24((uint32_t)(y - P.oy), (uint32_t)P.stride) + (uint32_t)(x - P.ox);
}
__device__ __forceinline__ int clamp_rx(const Params& P, int x) { return min(max(x, P.ox), P.ox + P.stride - 1); }
__device__ __forceinline__ int clamp_ry(const Params& P, int y) { return min(max(y, P.oy), P.oy + P.rows - 1); }

__device__ __forceinline__ NoisyItem noisy_item(const Params& P, const NoisyInputs& in,
                                                const Camera& cam, int gx, int gy, int frame) {
    NoisyItem o;
    const int2 off = kBlockOffsets[frame & 15];
    const int ux = gx - kEdge / 2 + off.x, uy = gy - kEdge / 2 + off.y;
    const int px = mirror(ux, P.width), py = mirror(uy, P.height);
    o.owner = ux >= 0 && ux < P.width && uy >= 0 && uy < P.height;
    o.lin = (uint32_t)(py * P.width + px);

    const f3 wp = ld3(in.p_cur, o.lin);
    const f3 nrm = ld3(in.n_cur, o.lin);
    const f3 cur = ld3(in.noisy_cur, o.lin);
    o.n = nrm;
    o.p = wp;

    float pfx = (float)px, pfy = (float)py;
    uint8_t accept = 0;
    float alpha = 1.f;
    f3 prev{0.f, 0.f, 0.f};
    float sample_spp = 0.f;
    if (frame > 0) {
        const float* M = cam.m;
        // .s048c / .s159d / .s37bf rows of the column-major matrix (bmfr.cl:343-347)
        float u = dot4(M[0], M[4], M[8], M[12], wp.x, wp.y, wp.z, 1.f);
        float v = dot4(M[1], M[5], M[9], M[13], wp.x, wp.y, wp.z, 1.f);
        const float w = dot4(M[3], M[7], M[11], M[15], wp.x, wp.y, wp.z, 1.f);
        const float rw = 1.f / w;  // u / w and v / w share the divisor
        u = div_shared(u, w, rw);
        v = div_shared(v, w, rw);
        u = u + 1.f;
        v = v + 1.f;
        u = u / 2.f;
        v = v / 2.f;
        pfx = u * (float)P.width - cam.jx;
        pfy = v * (float)P.height - (1 - cam.jy);
        const float flx = floorf(pfx), fly = floorf(pfy);
        const int ix = (int)flx, iy = (int)fly;
        const float fx = pfx - flx, fy = pfy - fly;
        const float omx = 1.f - fx, omy = 1.f - fy;
        const float wts[4] = {omx * omy, fx * omy, omx * fy, fx * fy};
        float total = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // bmfr.cl:374-419
            const int sx = ix + (i & 1), sy = iy + (i >> 1);
            if (sx >= 0 && sy >= 0 && sx < P.width && sy < P.height) {
                const uint32_t s = (uint32_t)(sy * P.width + sx);
                const f3 pp = ld3(in.p_prev, s);
                const f3 d{pp.x - wp.x, pp.y - wp.y, pp.z - wp.z};
                if (dot3(d, d) < P.position_limit_sq) {
                    const f3 pn = ld3(in.n_prev, s);
                    const f3 dn{pn.x - nrm.x, pn.y - nrm.y, pn.z - nrm.z};
                    if (dot3(dn, dn) < P.normal_limit_sq) {
                        accept |= (uint8_t)(1 << i);
                        sample_spp = sample_spp + wts[i] * (float)ld_px(in.spp_prev, s);
                        const f3 pc = ld3(in.noisy_prev, s);
                        prev.x = prev.x + wts[i] * pc.x;
                        prev.y = prev.y + wts[i] * pc.y;
                        prev.z = prev.z + wts[i] * pc.z;
                        total = total + wts[i];
                    }
                }
            }
        }
        if (total > 0.f) {  // bmfr.cl:421-429
            const float rt = 1.f / total;
            prev.x = div_shared(prev.x, total, rt);
            prev.y = div_shared(prev.y, total, rt);
            prev.z = div_shared(prev.z, total, rt);
            sample_spp = div_shared(sample_spp, total, rt);
            alpha = 1.f / (sample_spp + 1.f);
            alpha = fmaxf(alpha, P.blend_alpha);
        }
    }
    uint8_t new_spp = 1;  // bmfr.cl:433-442
    if (alpha < 1.f) new_spp = sample_spp > 254.f ? 255 : (uint8_t)((int)rintf(sample_spp) + 1);
    const float beta = 1.f - alpha;
    o.color = f3{alpha * cur.x + beta * prev.x, alpha * cur.y + beta * prev.y,
                 alpha * cur.z + beta * prev.z};
    o.pfx = pfx;
    o.pfy = pfy;
    o.accept = accept;
    o.spp = new_spp;
    return o;
}

// The same work-item with every load issued up front: the previous-frame
// position, normal, colour and spp of all four bilinear taps are fetched
// unconditionally (out-of-image taps at a clamped in-image address, then
// ignored), so a pixel costs two dependent memory round trips instead of up
// to four.  The arithmetic, its order and the results are noisy_item's.
// The current-frame planes of one item, as loaded (widened where used).
template <class IN = float>
struct NoisyCur {
    In3<IN> wp, nrm, cur;
    int px, py;
    bool owner;
};
// COLOUR = false: position and normal only (c.cur left for the caller).
// Margin-grid item (gx, gy): its (mirrored) image pixel and whether it owns
// it (bmfr.cl:310-317).
__device__ __forceinline__ void item_pixel(const Params& P, int gx, int gy, int frame, int& px, int& py, bool& owner) {
    const int2 off = kBlockOffsets[frame & 15];
    const int ux = gx - kEdge / 2 + off.x, uy = gy - kEdge / 2 + off.y;
    px = mirror(ux, P.width);
    py = mirror(uy, P.height);
    owner = ux >= 0 && ux < P.width && uy >= 0 && uy < P.height;
}

template <class IN = float, bool COLOUR = true>
__device__ __forceinline__ NoisyCur<IN> noisy_load_current(const Params& P, const NoisyInputs& in, int gx, int gy,
                                                           int frame) {
    NoisyCur<IN> c;
    item_pixel(P, gx, gy, frame, c.px, c.py, c.owner);
    const uint32_t lin = pix(P, c.px, c.py);
#ifdef BMFR_PROBE_K1_NOCUR  // timing probe (wrong results): current planes from one pixel (cache hits)
    const uint32_t l0 = lin & 63u;
    c.wp = ld3raw<IN>(in.p_cur, l0);
    c.nrm = ld3raw<IN>(in.n_cur, l0);
    if constexpr (COLOUR) c.cur = ld3raw<IN>(in.noisy_cur, l0);
#else
    c.wp = ld3raw<IN>(in.p_cur, lin);
    c.nrm = ld3raw<IN>(in.n_cur, lin);
    if constexpr (COLOUR) c.cur = ld3raw<IN>(in.noisy_cur, lin);
#endif
    return c;
}

// noisy_item_spec in two halves, so a caller can issue the next item's
// current-frame loads while this item's taps are in flight: _issue does the
// reprojection (bmfr.cl:343-372) and issues the tap loads, _finish tests,
// weighs and blends them (bmfr.cl:374-445).
// Half input planes: previous position / normal taps loaded a row pair at a
// time (noisy_taps_issue); -DBMFR_PAIR_TAPS=0 loads them pixel by pixel.
#ifndef BMFR_PAIR_TAPS
#define BMFR_PAIR_TAPS 1
#endif
template <class IN>
constexpr bool kPairTaps = BMFR_PAIR_TAPS && sizeof(IN) == 2;

template <class IN = float>
struct NoisyTaps {
    In3<IN> pp[4], pn[4];  // previous position / normal (input planes), as loaded
    // half input planes (kPairTaps): the previous position / normal of tap row
    // r's two pixels as one 12-byte load each, split into pp / pn in _finish;
    // fix bit 2 r: the row's pair was read one pixel to the right (it would
    // start before the plane), bit 2 r + 1: one to the left (it would end past it)
    h3pair pq[2], nq[2];
    uint32_t fix;
    bool any_fix;  // wave-uniform: some lane has a fix bit
    f3 pc[4], pa[4];
    // spp taps as loaded (u8 zero-extended): converted in _finish, so no
    // conversion -- and no wait for the loads -- sits in the issue half
    uint32_t spu[4];
    float wts[4];
    uint32_t inb;  // bit i: tap i inside the image
    float pfx, pfy, flx, fly;
    int over;
};


// The reprojection of one item (bmfr.cl:343-372): the previous-frame pixel
// position pf, the top-left bilinear tap (ix, iy) -- clamped in float first,
// so a far-off reprojection cannot overflow int --, the four tap weights,
// which taps lie inside the image (bit i: tap (ix + (i & 1), iy + (i >> 1)))
// and, tiled contexts, how far the in-image taps reach past the valid state.
// The bilinear tap weights at pf (bmfr.cl:359-372).
__device__ __forceinline__ void bilinear_weights(float pfx, float pfy, float (&wts)[4]) {
    const float fx = pfx - floorf(pfx), fy = pfy - floorf(pfy);
    const float omx = 1.f - fx, omy = 1.f - fy;
    wts[0] = omx * omy;
    wts[1] = fx * omy;
    wts[2] = omx * fy;
    wts[3] = fx * fy;
}

struct Reproj {
    float pfx, pfy;
    int ix, iy;
    float wts[4];
    uint32_t inb;
    int over;
};
__device__ __forceinline__ Reproj reproject(const Params& P, const Camera& cam, const f3& wp, int px, int py) {
    Reproj r;
    const float* M = cam.m;
    float u = dot4(M[0], M[4], M[8], M[12], wp.x, wp.y, wp.z, 1.f);
    float v = dot4(M[1], M[5], M[9], M[13], wp.x, wp.y, wp.z, 1.f);
    const float w = dot4(M[3], M[7], M[11], M[15], wp.x, wp.y, wp.z, 1.f);
    const float rw = 1.f / w;
    u = div_shared(u, w, rw);
    v = div_shared(v, w, rw);
    u = u + 1.f;
    v = v + 1.f;
    u = u / 2.f;
    v = v / 2.f;
    const float pfx = u * (float)P.width - cam.jx;
    const float pfy = v * (float)P.height - (1 - cam.jy);
    r.pfx = pfx;
    r.pfy = pfy;
    const float flx = floorf(pfx), fly = floorf(pfy);
    const int ix = (int)fminf(fmaxf(flx, -2.f), (float)P.width + 1.f);
    const int iy = (int)fminf(fmaxf(fly, -2.f), (float)P.height + 1.f);
    r.ix = ix;
    r.iy = iy;
    bilinear_weights(pfx, pfy, r.wts);
    r.over = 0;
    if (P.check_reach) {  // the in-image taps span [x0, x1] x [y0, y1]
        const int x0 = max(ix, 0), x1 = min(ix + 1, P.width - 1);
        const int y0 = max(iy, 0), y1 = min(iy + 1, P.height - 1);
        // a tile pixel's taps also read the previous TAA output (in K2)
        const bool tpx = px >= P.tx0 && px < P.tx1 && py >= P.ty0 && py < P.ty1;
        const int vx0 = tpx ? P.wx0 : P.vx0, vx1 = tpx ? P.wx1 : P.vx1;
        const int vy0 = tpx ? P.wy0 : P.vy0, vy1 = tpx ? P.wy1 : P.vy1;
        if (x0 <= x1 && y0 <= y1)
            r.over = max(max(max(vx0 - x0, x1 - (vx1 - 1)), max(vy0 - y0, y1 - (vy1 - 1))), 0);
    }
    r.inb = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int sx = ix + (i & 1), sy = iy + (i >> 1);
        r.inb |= (uint32_t)(sx >= 0 && sy >= 0 && sx < P.width && sy < P.height) << i;
    }
    return r;
}

template <bool FILT = false, class IN = float>
__device__ __forceinline__ NoisyTaps<IN> noisy_taps_issue(const Params& P, const NoisyInputs& in, const Camera& cam,
                                                         const NoisyCur<IN>& c, int frame,
                                                         const float* __restrict__ acc_prev = nullptr) {
    NoisyTaps<IN> tp;
    tp.pfx = (float)c.px;
    tp.pfy = (float)c.py;
    tp.over = 0;
    tp.inb = 0;
    if (frame > 0) {
        const Reproj r = reproject(P, cam, widen(c.wp), c.px, c.py);
        tp.pfx = r.pfx;
        tp.pfy = r.pfy;
        tp.over = r.over;
        tp.inb = r.inb;
        // The tap loads plane by plane (the four taps of a plane back to
        // back hit the same cache lines while they are in flight): K1 -2 %
        // against tap by tap (profiles/r04_ab_tap_order.txt).
        uint32_t sidx[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            tp.wts[i] = r.wts[i];
            const uint32_t s = pix(P, clamp_rx(P, r.ix + (i & 1)), clamp_ry(P, r.iy + (i >> 1)));
#ifdef BMFR_PROBE_K1_NOTAPS  // timing probe (wrong results): no previous-frame tap loads
            (void)s;
            tp.pp[i] = c.wp;
            tp.pn[i] = c.nrm;
            tp.pc[i] = f3{r.pfx, r.pfy, 0.f};
            tp.spu[i] = i;
            if (FILT) tp.pa[i] = f3{r.pfy, r.pfx, 0.f};
#else
            sidx[i] = s;
#endif
        }
#ifndef BMFR_PROBE_K1_NOTAPS
        if constexpr (kPairTaps<IN>) {
            // Half input planes: a tap row's two pixels (ix, y), (ix + 1, y) in
            // one 12-byte load per plane instead of two loads per pixel (a
            // dword and a short).  The pair starts at ix clamped to
            // [ox - 1, ox + stride - 1]: in-region taps are read where they lie,
            // an out-of-region one (ignored, or a reach overshoot the context
            // reports) from a neighbouring row.  Only a pair starting at linear
            // index -1 or n - 1 would leave the plane: it is read one pixel
            // over, and _finish takes its in-region tap from the other half.
            const int n = P.stride * P.rows;
            const int xc = min(max(r.ix, P.ox - 1), P.ox + P.stride - 1) - P.ox;
            uint32_t spair[2];
            tp.fix = 0;
#pragma unroll
            for (int row = 0; row < 2; ++row) {
                const int sr = (int)__umul24((uint32_t)(clamp_ry(P, r.iy + row) - P.oy), (uint32_t)P.stride) + xc;
                spair[row] = (uint32_t)min(max(sr, 0), n - 2);
                tp.fix |= ((uint32_t)(sr < 0) << (2 * row)) | ((uint32_t)(sr > n - 2) << (2 * row + 1));
            }
            tp.any_fix = __builtin_amdgcn_ballot_w64(tp.fix != 0) != 0;
#ifdef BMFR_PROBE_NO_PAIR_FIX  // test probe (wrong results at the plane's ends): tests/test_gpu_pair_taps.py
            tp.any_fix = false;
#endif
#pragma unroll
            for (int row = 0; row < 2; ++row) tp.pq[row] = ld3pair_h(in.p_prev, spair[row]);
#pragma unroll
            for (int row = 0; row < 2; ++row) tp.nq[row] = ld3pair_h(in.n_prev, spair[row]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) tp.pp[i] = ld3raw<IN>(in.p_prev, sidx[i]);
#pragma unroll
            for (int i = 0; i < 4; ++i) tp.pn[i] = ld3raw<IN>(in.n_prev, sidx[i]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) tp.pc[i] = ld3(in.noisy_prev, sidx[i]);
#pragma unroll
        for (int i = 0; i < 4; ++i) tp.spu[i] = ld_px(in.spp_prev, sidx[i]);
        if (FILT) {  // same taps (bmfr.cl:801-832)
#pragma unroll
            for (int i = 0; i < 4; ++i) tp.pa[i] = ld3(acc_prev, sidx[i]);
        }
#endif
    }
    return tp;
}

// The acceptance half of noisy_taps_finish (bmfr.cl:380-404): bit i set when
// tap i is inside the image and its previous position and normal are close
// enough to the pixel's current ones.
template <class IN = float>
__device__ __forceinline__ uint32_t taps_accept(const Params& P, const f3& wp, const f3& nrm, const In3<IN> (&pp)[4],
                                                const In3<IN> (&pn)[4], uint32_t inb) {
    uint32_t accept = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const f3 q = widen(pp[i]), m = widen(pn[i]);
        const f3 d{q.x - wp.x, q.y - wp.y, q.z - wp.z};
        const f3 dn{m.x - nrm.x, m.y - nrm.y, m.z - nrm.z};
        if ((inb & (1u << i)) && dot3(d, d) < P.position_limit_sq && dot3(dn, dn) < P.normal_limit_sq)
            accept |= 1u << i;
    }
    return accept;
}

// The accumulation half (bmfr.cl:405-445, and with FILT accumulate_filtered_
// data's sums at the same taps, bmfr.cl:786-842): the accepted taps' colours,
// spp and filtered colours weighed and blended.  o.n / o.p are left to the
// caller.
template <bool FILT = false>
__device__ __forceinline__ NoisyItem taps_blend(const Params& P, const f3& cur, uint32_t accept, const float (&wts)[4],
                                                const f3 (&pc)[4], const uint32_t (&spu)[4], const f3 (&pa)[4],
                                                float pfx, float pfy, int over, uint32_t lin, bool owner, int frame) {
    NoisyItem o;
    o.owner = owner;
    o.lin = lin;
    float alpha = 1.f;
    f3 prev{0.f, 0.f, 0.f};
    float sample_spp = 0.f;
    o.prev_f = f3{0.f, 0.f, 0.f};
    o.prev_f_divided = false;
    o.over = over;
    if (frame > 0) {
        float total = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // bmfr.cl:374-419
            if (accept & (1u << i)) {
                sample_spp = sample_spp + wts[i] * (float)spu[i];
                prev.x = prev.x + wts[i] * pc[i].x;
                prev.y = prev.y + wts[i] * pc[i].y;
                prev.z = prev.z + wts[i] * pc[i].z;
                total = total + wts[i];
                if (FILT) {  // accumulate_filtered_data's sums: same weights, same order
                    o.prev_f.x = o.prev_f.x + wts[i] * pa[i].x;
                    o.prev_f.y = o.prev_f.y + wts[i] * pa[i].y;
                    o.prev_f.z = o.prev_f.z + wts[i] * pa[i].z;
                }
            }
        }
        if (total > 0.f) {  // bmfr.cl:421-429
            const float rt = 1.f / total;
            prev.x = div_shared(prev.x, total, rt);
            prev.y = div_shared(prev.y, total, rt);
            prev.z = div_shared(prev.z, total, rt);
            sample_spp = div_shared(sample_spp, total, rt);
            // 1 / (sample_spp + 1): sample_spp is a weighted mean of spp
            // values in [0, 255], so the divisor lies in [1, 257) (rcp_nr)
            alpha = rcp_nr(sample_spp + 1.f);
            alpha = fmaxf(alpha, P.blend_alpha);
            if (FILT) {  // bmfr.cl:834-842: the same sum of accepted tap weights, one reciprocal
                o.prev_f_divided = true;
                o.prev_f.x = div_shared(o.prev_f.x, total, rt);
                o.prev_f.y = div_shared(o.prev_f.y, total, rt);
                o.prev_f.z = div_shared(o.prev_f.z, total, rt);
            }
        }
    }
    uint8_t new_spp = 1;  // bmfr.cl:433-442
    if (alpha < 1.f) new_spp = sample_spp > 254.f ? 255 : (uint8_t)((int)rintf(sample_spp) + 1);
    const float beta = 1.f - alpha;
    o.color = f3{alpha * cur.x + beta * prev.x, alpha * cur.y + beta * prev.y, alpha * cur.z + beta * prev.z};
    o.pfx = pfx;
    o.pfy = pfy;
    o.accept = (uint8_t)accept;
    o.spp = new_spp;
    return o;
}

// The four taps of a plane from its two row pairs (noisy_taps_issue, half
// input planes): tap 2 r + k is pixel k of row r's pair, except where the
// pair was read one pixel over (fix bits, see NoisyTaps): then the in-region
// tap is the pair's other pixel.
__device__ __forceinline__ void split_pairs(const h3pair (&q)[2], uint32_t fix, bool any_fix, In3<_Float16> (&t)[4]) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        t[2 * r].v.xy = q[r].a;
        t[2 * r].v.z = (uint16_t)(q[r].b & 0xffffu);
        t[2 * r + 1].v.xy = __builtin_amdgcn_alignbit(q[r].c, q[r].b, 16);
        t[2 * r + 1].v.z = (uint16_t)(q[r].c >> 16);
    }
    if (any_fix) {  // wave-uniform, and only at the plane's first / last pixel
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            if (fix & (1u << (2 * r))) t[2 * r + 1] = t[2 * r];    // read from pixel 0: tap 1 is its first pixel
            if (fix & (2u << (2 * r))) t[2 * r] = t[2 * r + 1];    // read from pixel n - 2: tap 0 is its second
        }
    }
}

template <bool FILT = false, class IN = float>
__device__ __forceinline__ NoisyItem noisy_taps_finish(const Params& P, const NoisyCur<IN>& c,
                                                      const NoisyTaps<IN>& tp, int frame) {
    const f3 wp = widen(c.wp), nrm = widen(c.nrm), cur = widen(c.cur);
    uint32_t accept = 0u;
    if constexpr (kPairTaps<IN>) {
        if (frame > 0) {
            In3<IN> pp[4], pn[4];
            split_pairs(tp.pq, tp.fix, tp.any_fix, pp);
            split_pairs(tp.nq, tp.fix, tp.any_fix, pn);
            accept = taps_accept<IN>(P, wp, nrm, pp, pn, tp.inb);
        }
    } else {
        accept = frame > 0 ? taps_accept<IN>(P, wp, nrm, tp.pp, tp.pn, tp.inb) : 0u;
    }
    NoisyItem o = taps_blend<FILT>(P, cur, accept, tp.wts, tp.pc, tp.spu, tp.pa, tp.pfx, tp.pfy, tp.over,
                                   pix(P, c.px, c.py), c.owner, frame);
    o.n = nrm;
    o.p = wp;
    return o;
}

template <bool FILT = false, class IN = float>
__device__ __forceinline__ NoisyItem noisy_item_spec(const Params& P, const NoisyInputs& in, const Camera& cam,
                                                     const NoisyCur<IN>& c, int frame,
                                                     const float* __restrict__ acc_prev = nullptr) {
    return noisy_taps_finish<FILT, IN>(P, c, noisy_taps_issue<FILT, IN>(P, in, cam, c, frame, acc_prev), frame);
}

// One work-group's reprojection-reach report (tiled contexts): the lanes
// whose taps left the valid state rectangle raise the context's maximum.
__device__ __forceinline__ void report_reach(const Params& P, unsigned* reach, int over) {
    if (P.check_reach && __builtin_amdgcn_ballot_w64(over > 0) != 0 && over > 0)
        atomicMax(reach, (unsigned)over);
}

// tmp_data value of feature f for an item (bmfr.cl:448-473): NaN -> 0, and
// the +-65504 clamp when the matrix is kept in half.
__device__ __forceinline__ float design_value(const Params& P, int f, const NoisyItem& it) {
    const int B = P.buffers;
    float v;
    if (f < B - 3) v = feature_value(P.codes[f], it.n, it.p);
    else v = f == B - 3 ? it.color.x : (f == B - 2 ? it.color.y : it.color.z);
    if (__builtin_isnan(v)) v = 0.0f;
    if (P.half_tmp) v = fmaxf(fminf(v, 65504.f), -65504.f);
    return v;
}

// --------------------------------------------------------------------------
// The fitter (bmfr.cl:503-699) on a register-resident block.
//   a[f][s]  : row t + 256*s of feature column f (rounded to half if HALF)
//   FULL     : also run the colour columns' own Householder steps, which only
//              touch rows >= B-3 and the never-read slot R(R_EDGE-1,R_EDGE-1)
//              (bmfr.cl:550,606); needed only to leave tmp_data exactly as
//              upstream does.  The fused kernel skips them.
//   FAST_DIV : trailing update divides through div_by_recip (bit-identical
//              to the correctly rounded quotient; see bmfr_device.h).
// On return lds.weights[(B-3)*3] holds the block's weights and
// lds.minmax[FS*2] its min/max (mins_maxs layout).
// --------------------------------------------------------------------------
template <int B>
struct FitLds {
    float part[(B - 1) * kLocal];
    float res[B];
    float bc[2];
    float R[(B - 2) * (B - 2) * 3];  // R[x][y][ch], x = column, y = row
    float weights[(B - 3) * 3];
    float minmax[2 * (B - 3)];
};

template <int NS, int FS, bool HALF, bool FULL, bool FAST_DIV>
__device__ __forceinline__ void fit_block(float (&a)[NS + FS + 3][kSubs], FitLds<NS + FS + 3>& L,
                                          int t, int frame, double noise2) {
    constexpr int B = NS + FS + 3;
    constexpr int RE = B - 2;  // R_EDGE

    // Scale the position features to the block's [min, max] (bmfr.cl:510-542).
    if constexpr (FS > 0) {
        float mx[FS], mn[FS];
#pragma unroll
        for (int f = 0; f < FS; ++f) {
            float hi = -INFINITY, lo = INFINITY;
#pragma unroll
            for (int s = 0; s < kSubs; ++s) {
                hi = fmaxf(a[NS + f][s], hi);
                lo = fminf(a[NS + f][s], lo);
            }
            mx[f] = hi;
            mn[f] = lo;
        }
        block_reduce<RedOp::Max, FS>(mx, FS, L.part, L.res, t);
        float bmax[FS];
#pragma unroll
        for (int f = 0; f < FS; ++f) bmax[f] = L.res[f];
        block_reduce<RedOp::Min, FS>(mn, FS, L.part, L.res, t);
#pragma unroll
        for (int f = 0; f < FS; ++f) {
            const float bmin = L.res[f];
            if (t == 0) {
                L.minmax[2 * f] = bmin;
                L.minmax[2 * f + 1] = bmax[f];
            }
#pragma unroll
            for (int s = 0; s < kSubs; ++s) {
                const float v = scale(a[NS + f][s], bmin, bmax[f]);
                a[NS + f][s] = HALF ? round_half(v) : v;
            }
        }
    }

    // Householder QR (bmfr.cl:544-656).
    constexpr int COLS = FULL ? B : B - 3;
#pragma unroll
    for (int col = 0; col < COLS; ++col) {
        constexpr int dummy = 0;
        (void)dummy;
        const int cl = col < B - 3 ? col : B - 3;  // col_limited
        float sq = 0.f;
#pragma unroll
        for (int s = 0; s < kSubs; ++s) {
            const int i = t + s * kLocal;
            if (i >= cl + 1) sq = sq + a[col][s] * a[col][s];
        }
        if (t == cl) L.bc[0] = a[col][0];  // u_vec[col_limited], row cl is row t=cl, s=0
        {
            float one[1] = {sq};
            block_reduce<RedOp::Sum, 1>(one, 1, L.part, L.res, t);
        }
        const float sumsq = L.res[0];
        const float ucl = L.bc[0];
        const float vlen = sqrtf(sumsq + ucl * ucl);  // bmfr.cl:582-585
        const float ucl2 = ucl - vlen;
        const float ulen2 = sumsq + ucl2 * ucl2;

        // R column (bmfr.cl:574-601).  Rows y < col belong to thread y, s = 0.
        if (col < B - 3) {
            if (t < col) {
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) L.R[(col * RE + t) * 3 + ch] = a[col][0];
            }
            if (t == col) {
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) L.R[(col * RE + col) * 3 + ch] = vlen;
            }
        } else {
            if (t < B - 3) L.R[((RE - 1) * RE + t) * 3 + (col - (B - 3))] = a[col][0];
        }

        float u[kSubs];
#pragma unroll
        for (int s = 0; s < kSubs; ++s) u[s] = a[col][s];
        if (t == cl) u[0] = ucl2;

        // Trailing columns fb = cl+1 .. B-1 (bmfr.cl:606-655): all dots first
        // (one batched reduction), then all updates.  Each column's update only
        // depends on its own dot, so the per-element arithmetic is upstream's.
        float dp[B - 1];
#pragma unroll
        for (int fb = 1; fb < B; ++fb) {
            float d = 0.f;
            if (fb > cl) {
#pragma unroll
                for (int s = 0; s < kSubs; ++s) {
                    const int i = t + s * kLocal;
                    if (i >= cl) {
                        float v = a[fb][s];
                        if (col == 0 && fb < B - 3)  // noise once, on first load (bmfr.cl:625-627)
                            v = add_random(v, noise2, t + s * kLocal + fb * kBlockPixels +
                                                          frame * B * kBlockPixels);
                        a[fb][s] = v;
                        d = d + v * u[s];
                    }
                }
            }
            dp[fb - 1] = d;
        }
        // Reduction k covers column fb = cl + 1 + k.
        float dk[B - 1];
#pragma unroll
        for (int k = 0; k < B - 1; ++k) dk[k] = 0.f;
#pragma unroll
        for (int fb = 1; fb < B; ++fb)
            if (fb > cl) dk[fb - cl - 1] = dp[fb - 1];
        block_reduce<RedOp::Sum, B - 1>(dk, B - 1 - cl, L.part, L.res, t);

        const float recip = 1.f / ulen2;
#pragma unroll
        for (int fb = 1; fb < B; ++fb) {
            if (fb > cl) {
                const float c2 = 2.f * L.res[fb - cl - 1];  // 2*u*dot == u*(2*dot), both exact doublings
#pragma unroll
                for (int s = 0; s < kSubs; ++s) {
                    const int i = t + s * kLocal;
                    if (i >= cl) {
                        const float num = u[s] * c2;
                        const float q = FAST_DIV ? div_by_recip(num, ulen2, recip) : num / ulen2;
                        const float v = a[fb][s] - q;
                        a[fb][s] = HALF ? round_half(v) : v;
                    }
                }
            }
        }
    }
    if constexpr (!FULL) {
        // Right-hand side = rows 0..B-4 of the colour columns, untouched by the
        // colour columns' own steps (they only write rows >= B-3).
        if (t < B - 3) {
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) L.R[((RE - 1) * RE + t) * 3 + ch] = a[B - 3 + ch][0];
        }
    }
    __syncthreads();

    // Back substitution (bmfr.cl:658-699), one lane per colour channel.  Each
    // element sees upstream's operations in upstream's order.
    if (t < 3) {
        const int ch = t;
        float R[RE][RE];
#pragma unroll
        for (int x = 0; x < RE; ++x)
#pragma unroll
            for (int y = 0; y <= (x < RE - 1 ? x : RE - 2); ++y) R[x][y] = L.R[(x * RE + y) * 3 + ch];
#pragma unroll
        for (int i = RE - 2; i >= 0; --i) {
            const float div = R[i][i];
#pragma unroll
            for (int x = i; x < RE; ++x) R[x][i] = R[x][i] / div;
#pragma unroll
            for (int j = i + 1; j < RE - 1; ++j) R[RE - 1][i] = R[RE - 1][i] - R[j][i];
#pragma unroll
            for (int y = 0; y <= i; ++y) R[i][y] = R[i][y] * R[RE - 1][i];
        }
#pragma unroll
        for (int id = 0; id < B - 3; ++id) L.weights[id * 3 + ch] = R[RE - 1][id];
    }
    __syncthreads();
}

// --------------------------------------------------------------------------
// Temporal blend of the filtered colour (bmfr.cl:778-849): the accumulated
// colour of a pixel, given its filtered colour, reprojection, accept bits and
// spp and the previous accumulated frame.
__device__ __forceinline__ f3 blend_filtered(const Params& P, f3 filtered, float pfx, float pfy,
                                             uint8_t acc_bits, uint8_t spp,
                                             const float* __restrict__ acc_prev, int frame) {
    f3 prev{0.f, 0.f, 0.f};
    float alpha = 1.f;
    if (frame > 0 && acc_bits > 0) {
        const float flx = floorf(pfx), fly = floorf(pfy);
        const int ix = (int)flx, iy = (int)fly;
        const float fx = pfx - flx, fy = pfy - fly;
        const float omx = 1.f - fx, omy = 1.f - fy;
        const float wts[4] = {omx * omy, fx * omy, omx * fy, fx * fy};
        float total = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (acc_bits & (1 << i)) {
                total = total + wts[i];
                const f3 pc = ld3(acc_prev, pix(P, ix + (i & 1), iy + (i >> 1)));
                prev.x = prev.x + wts[i] * pc.x;
                prev.y = prev.y + wts[i] * pc.y;
                prev.z = prev.z + wts[i] * pc.z;
            }
        }
        if (total > 0.f) {
            alpha = 1.f / (float)spp;
            alpha = fmaxf(alpha, P.second_blend_alpha);
            const float rt = 1.f / total;
            prev.x = div_shared(prev.x, total, rt);
            prev.y = div_shared(prev.y, total, rt);
            prev.z = div_shared(prev.z, total, rt);
        }
    }
    const float beta = 1.f - alpha;
    return f3{alpha * filtered.x + beta * prev.x, alpha * filtered.y + beta * prev.y,
              alpha * filtered.z + beta * prev.z};
}

// Albedo remodulation + 1/2.2 gamma + clamp (bmfr.cl:851-856), with powr
// correctly rounded (bmfr_powr.h: equal to the oracle's for every input) or,
// with library_powr, the device library's as the reference kernel calls it.
__device__ __forceinline__ f3 tone_map(const Params& P, f3 albedo, f3 a, const double* tE = kPowrE,
                                       const double2* tRP = kPowrRP) {
    const f3 p{albedo.x * a.x, albedo.y * a.y, albedo.z * a.z};
    if (P.library_powr) {
        const float g = 0.454545f;
        return f3{fminf(fmaxf(__ocml_powr_f32(fmaxf(0.f, p.x), g), 0.f), 1.f),
                  fminf(fmaxf(__ocml_powr_f32(fmaxf(0.f, p.y), g), 0.f), 1.f),
                  fminf(fmaxf(__ocml_powr_f32(fmaxf(0.f, p.z), g), 0.f), 1.f)};
    }
    return f3{gamma_clamped(p.x, tE, tRP), gamma_clamped(p.y, tE, tRP), gamma_clamped(p.z, tE, tRP)};
}

// The four bilinear taps of the previous TAA output at reprojected position
// pf (bmfr.cl:929-960), loaded unconditionally: the address is clamped in
// float first, so an off-screen or non-finite pf still reads a valid pixel
// (taa_resolve then ignores it).  On every path taa_resolve takes, the clamp
// is the identity and the taps are upstream's.
__device__ __forceinline__ void taa_load_taps(const Params& P, float2 pf, const float* __restrict__ prev_frame,
                                              f3 (&pc)[4]) {
    const int ix = (int)fminf(fmaxf(floorf(pf.x), -2.f), (float)P.width + 1.f);
    const int iy = (int)fminf(fmaxf(floorf(pf.y), -2.f), (float)P.height + 1.f);
#pragma unroll
    for (int i = 0; i < 4; ++i)
        pc[i] = ld3(prev_frame, pix(P, clamp_rx(P, ix + (i & 1)), clamp_ry(P, iy + (i >> 1))));
}

// TAA for one pixel (bmfr.cl:873-973) in two halves.  taa_history: the
// bilinear blend of the previous TAA output's taps (from taa_load_taps) at
// reprojected position pf, in YCoCg (bmfr.cl:925-966); any value when the
// reprojection is off-screen (taa_clamp then returns the pixel's own colour).
// It needs no neighbour, so a tile forms it as soon as the taps arrive and
// keeps three values instead of twelve.
__device__ __forceinline__ f3 taa_history(const Params& P, float2 pf, const f3 (&pc)[4]) {
    const int W = P.width, H = P.height;
    const float flx = floorf(pf.x), fly = floorf(pf.y);
    // as taa_load_taps: in the int range whatever pf is (the result is only
    // used when pf is on screen, where this is the identity)
    const int ix = (int)fminf(fmaxf(flx, -2.f), (float)W + 1.f);
    const int iy = (int)fminf(fmaxf(fly, -2.f), (float)H + 1.f);
    f3 prev{0.f, 0.f, 0.f};
    float total = 0.f;
    const float fx = pf.x - flx, fy = pf.y - fly;
    const float omx = 1.f - fx, omy = 1.f - fy;
    const float tw[4] = {omx * omy, fx * omy, omx * fy, fx * fy};
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // bmfr.cl:929-960
        const bool okx = (i & 1) ? (ix < W - 1) : (ix >= 0);
        const bool oky = (i >> 1) ? (iy < H - 1) : (iy >= 0);
        if (okx && oky) {
            prev.x = prev.x + tw[i] * pc[i].x;
            prev.y = prev.y + tw[i] * pc[i].y;
            prev.z = prev.z + tw[i] * pc[i].z;
            total = total + tw[i];
        }
    }
    const float rt = 1.f / total;  // total can be 0 only in a degenerate case (bmfr.cl:962)
    prev = f3{div_shared(prev.x, total, rt), div_shared(prev.y, total, rt), div_shared(prev.z, total, rt)};
    return rgb_to_ycocg(prev);
}

// taa_clamp: the history py (taa_history) clamped to the YCoCg box / cross
// of the pixel's 3x3 neighbourhood in the current tone-mapped frame,
// nb[3 * (dy + 1) + (dx + 1)] (nb[4] is the centre's), and blended with the
// pixel's own colour me.
// CHECK: skip out-of-image neighbours as upstream does (any value may stand
// in nb[] for them); without it every neighbour must be in the image.  A
// skipped neighbour enters the min / max as +inf / -inf, which leaves them
// unchanged bit for bit, so both forms are upstream's sequence.
__device__ __forceinline__ f3 taa_clamp_tail(const Params& P, f3 me, f3 mnb, f3 mxb, f3 mnc, f3 mxc, f3 py);
// The off-screen test of bmfr.cl:884-890: the pixel keeps its own colour.
__device__ __forceinline__ bool taa_offscreen(const Params& P, float2 pf, int frame) {
    const float flx = floorf(pf.x), fly = floorf(pf.y);
    return frame == 0 || flx < -1.f || fly < -1.f || flx >= (float)P.width || fly >= (float)P.height;
}
template <bool CHECK>
__device__ __forceinline__ f3 taa_clamp(const Params& P, int x, int y, f3 me, float2 pf, const f3 (&nb)[9], f3 py,
                                        int frame) {
    const int W = P.width, H = P.height;
    const float flx = floorf(pf.x), fly = floorf(pf.y);
    if (frame == 0 || flx < -1.f || fly < -1.f || flx >= (float)W || fly >= (float)H)
        return me;  // bmfr.cl:884-890 (compared as floats: no int overflow)
    // bmfr.cl:897-920: min / max over the 3x3 box and the cross, visited dy
    // outer, dx inner.  A skipped neighbour enters as +inf / -inf; the
    // three-operand min / max keep upstream's left-to-right order exactly.
    f3 nlo[9], nhi[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        nlo[k] = nb[k];
        nhi[k] = nb[k];
        if (CHECK) {
            const int sx = x + k % 3 - 1, sy = y + k / 3 - 1;
            const bool in = sx >= 0 && sy >= 0 && sx < W && sy < H;
            nlo[k] = in ? nlo[k] : f3{INFINITY, INFINITY, INFINITY};
            nhi[k] = in ? nhi[k] : f3{-INFINITY, -INFINITY, -INFINITY};
        }
    }
    auto box_cross = [&](auto get, float& mnb_, float& mxb_, float& mnc_, float& mxc_) {
        const float inf = INFINITY;
        float m = vmin3s(inf, get(nlo[0]), get(nlo[1]));
        m = vmin3(m, get(nlo[2]), get(nlo[3]));
        m = vmin3(m, get(nlo[4]), get(nlo[5]));
        m = vmin3(m, get(nlo[6]), get(nlo[7]));
        mnb_ = vmin(m, get(nlo[8]));
        float M = vmax3s(-inf, get(nhi[0]), get(nhi[1]));
        M = vmax3(M, get(nhi[2]), get(nhi[3]));
        M = vmax3(M, get(nhi[4]), get(nhi[5]));
        M = vmax3(M, get(nhi[6]), get(nhi[7]));
        mxb_ = vmax(M, get(nhi[8]));
        mnc_ = vmin(vmin3(vmin3s(inf, get(nlo[1]), get(nlo[3])), get(nlo[4]), get(nlo[5])), get(nlo[7]));
        mxc_ = vmax(vmax3(vmax3s(-inf, get(nhi[1]), get(nhi[3])), get(nhi[4]), get(nhi[5])), get(nhi[7]));
    };
    f3 mnb, mxb, mnc, mxc;
    box_cross([](const f3& v) { return v.x; }, mnb.x, mxb.x, mnc.x, mxc.x);
    box_cross([](const f3& v) { return v.y; }, mnb.y, mxb.y, mnc.y, mxc.y);
    box_cross([](const f3& v) { return v.z; }, mnb.z, mxb.z, mnc.z, mxc.z);
    return taa_clamp_tail(P, me, mnb, mxb, mnc, mxc, py);
}

// taa_clamp's part after the neighbourhood: the history py clamped to the
// average of the box and cross bounds (bmfr.cl:922-973), blended with me.
// The min / max of a set are exact and order-independent on v_min / v_max
// (minNum: a NaN operand is ignored, -0 < +0), so a caller may form the box
// and cross bounds in any grouping -- e.g. from per-row partial bounds shared
// by vertically neighbouring pixels -- as long as each set starts from +inf /
// -inf as upstream's does (an all-NaN set then yields +inf / -inf).
__device__ __forceinline__ f3 taa_clamp_tail(const Params& P, f3 me, f3 mnb, f3 mxb, f3 mnc, f3 mxc, f3 py) {
    const f3 lo{(mnb.x + mnc.x) / 2.f, (mnb.y + mnc.y) / 2.f, (mnb.z + mnc.z) / 2.f};
    const f3 hi{(mxb.x + mxc.x) / 2.f, (mxb.y + mxc.y) / 2.f, (mxb.z + mxc.z) / 2.f};
    const f3 cl{fminf(fmaxf(py.x, lo.x), hi.x), fminf(fmaxf(py.y, lo.y), hi.y), fminf(fmaxf(py.z, lo.z), hi.z)};
    const f3 pr = ycocg_to_rgb(cl);
    const float a = P.taa_blend_alpha, b = 1.f - a;
    return f3{a * me.x + b * pr.x, a * me.y + b * pr.y, a * me.z + b * pr.z};
}

// Both halves for one pixel.
template <bool CHECK>
__device__ __forceinline__ f3 taa_resolve(const Params& P, int x, int y, f3 me, float2 pf, const f3 (&nb)[9],
                                          const f3 (&pc)[4], int frame) {
    return taa_clamp<CHECK>(P, x, y, me, pf, nb, taa_history(P, pf, pc), frame);
}

}  // namespace bmfr
