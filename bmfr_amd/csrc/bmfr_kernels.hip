// bmfr_kernels.hip -- BMFR kernels for MI355X (gfx950).
//
// Two families:
//  * Stage kernels: one per reference kernel, same buffer layouts and
//    argument roles (bmfr.cl:290-974).  They back the stage C-ABI entry
//    points and the per-stage parity tests.
//  * Fused frame kernels: K1 = accumulate_noisy -> scale -> QR -> solve ->
//    weighted_sum -> accumulate_filtered -> tone map for one 32x32 block per
//    256-thread work-group, with the design matrix never leaving VGPRs
//    (upstream round-trips it through HBM ~30 times per block, bmfr.cl:555-656);
//    K2 = TAA (needs the 3x3 neighbourhood across block borders).
#include "bmfr_kernels.h"
#include "bmfr_generic.h"
#include "bmfr_launch.h"

namespace bmfr {

// ---------------------------------------------------------------- stage 1 --
// pass 0: margin work-items only, pass 1: owners only.  Launched in that
// order, every read of current_noisy sees the input colour.
__global__ __launch_bounds__(256) void k_accumulate_noisy(Params P, NoisyInputs in, Camera cam,
                                                          int frame, int pass, float2* prev_pixel,
                                                          uint8_t* accept, float* noisy_out,
                                                          uint8_t* spp_cur, void* tmp) {
    const int gx = blockIdx.x * blockDim.x + threadIdx.x;
    const int gy = blockIdx.y * blockDim.y + threadIdx.y;
    if (gx >= P.margins_w || gy >= P.margins_h) return;
    const int2 off = kBlockOffsets[frame & 15];
    const int ux = gx - kEdge / 2 + off.x, uy = gy - kEdge / 2 + off.y;
    const bool owner = ux >= 0 && ux < P.width && uy >= 0 && uy < P.height;
    if ((int)owner != pass) return;

    const NoisyItem it = noisy_item(P, in, cam, gx, gy, frame);
    spp_cur[it.lin] = it.spp;
    const int bx = gx / kEdge, by = gy / kEdge;
    const size_t base = ((size_t)by * P.blocks_x + bx) * (size_t)P.buffers * kBlockPixels +
                        (size_t)(gy % kEdge) * kEdge + (gx % kEdge);
    for (int f = 0; f < P.buffers; ++f) {
        const float v = design_value(P, f, it);
        if (P.half_tmp) ((_Float16*)tmp)[base + (size_t)f * kBlockPixels] = (_Float16)v;
        else ((float*)tmp)[base + (size_t)f * kBlockPixels] = v;
    }
    if (it.owner) {
        st3(noisy_out, it.lin, it.color);
        prev_pixel[it.lin] = make_float2(it.pfx, it.pfy);
        accept[it.lin] = it.accept;
    }
}

// ---------------------------------------------------------------- stage 3 --
__device__ __forceinline__ int block_of_pixel(const Params& P, int x, int y, int frame) {
    const int2 off = kBlockOffsets[frame & 15];
    return (x + kEdge / 2 - off.x) / kEdge + ((y + kEdge / 2 - off.y) / kEdge) * P.blocks_x;
}

__global__ __launch_bounds__(256) void k_weighted_sum(Params P, const float* __restrict__ weights,
                                                      const float* __restrict__ mins_maxs,
                                                      float* __restrict__ out,
                                                      const float* __restrict__ normals,
                                                      const float* __restrict__ positions, int frame) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y * blockDim.y + threadIdx.y;
    if (x >= P.width || y >= P.height) return;
    const uint32_t lin = (uint32_t)(y * P.width + x);
    const int g = block_of_pixel(P, x, y, frame);
    const f3 c = weighted_color(P, weights + (size_t)g * (P.buffers - 3) * 3,
                                mins_maxs + (size_t)g * P.scaled * 2, ld3(normals, lin),
                                ld3(positions, lin));
    st3(out, lin, c);
}

// ---------------------------------------------------------------- stage 4 --
__global__ __launch_bounds__(256) void k_accumulate_filtered(
    Params P, const float* __restrict__ filtered, const float2* __restrict__ prev_pixel,
    const uint8_t* __restrict__ accept, const float* __restrict__ albedo,
    float* __restrict__ tone_mapped, const uint8_t* __restrict__ spp,
    const float* __restrict__ acc_prev, float* __restrict__ acc, int frame) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y * blockDim.y + threadIdx.y;
    if (x >= P.width || y >= P.height) return;
    const uint32_t lin = (uint32_t)(y * P.width + x);
    const float2 pp = prev_pixel[lin];
    const f3 a = blend_filtered(P, ld3(filtered, lin), pp.x, pp.y, frame > 0 ? accept[lin] : 0, spp[lin],
                                acc_prev, frame);
    st3(acc, lin, a);
    st3(tone_mapped, lin, tone_map(P, ld3(albedo, lin), a));
}

// ---------------------------------------------------------------- stage 5 --
__global__ __launch_bounds__(256) void k_taa(Params P, const float2* __restrict__ prev_pixel,
                                             const float* __restrict__ new_frame,
                                             float* __restrict__ result,
                                             const float* __restrict__ prev_frame, int frame) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y * blockDim.y + threadIdx.y;
    if (x >= P.width || y >= P.height) return;
    const uint32_t lin = (uint32_t)(y * P.width + x);
    const f3 me = ld3(new_frame, lin);
    const float2 pf = prev_pixel[lin];
    f3 pc[4], nb[9];
    taa_load_taps(P, pf, prev_frame, pc);
#pragma unroll
    for (int k = 0; k < 9; ++k)  // out-of-image neighbours: a clamped in-image pixel, skipped by taa_resolve
        nb[k] = rgb_to_ycocg(ld3(new_frame, pix(P, clamp_rx(P, x + k % 3 - 1), clamp_ry(P, y + k / 3 - 1))));
    st3(result, lin, taa_resolve<true>(P, x, y, me, pf, nb, pc, frame));
}

// --------------------------------------------------------- fused K2: TAA --
// Tone map + TAA, one 64 x kTaaH tile per 256-thread work-group (taa_tile,
// bmfr_taa_tile.h).
// Tile height measured at 4K (K2 ms): 8: 0.114, 12: 0.105, 16: 0.112,
// 24: 0.130, 32: 0.135; forcing 4 waves/SIMD (128 VGPRs) at 16: 0.159.
// Round 4 (taps after the tone map, -DBMFR_K2_H / -DBMFR_K2_NT): 12: 0.1028,
// 8 (80 VGPRs, six waves): 0.1028, 16: 0.1062, 512 threads x 16: 0.1074,
// 512 x 24: 0.1190 (profiles/r04_ab_k2_shapes.txt).
#ifndef BMFR_K2_H
#define BMFR_K2_H 12
#endif
constexpr int kTaaW = 64, kTaaH = BMFR_K2_H;
// Threads per tile (experiment: -DBMFR_K2_NT=384 / 768 -- 2 / 1 output
// pixels per thread instead of 3, fewer registers, more waves per SIMD).
#ifndef BMFR_K2_NT
#define BMFR_K2_NT 256
#endif
constexpr int kTaaNT = BMFR_K2_NT;
// Minimum waves per SIMD for the register allocator: six (80 VGPRs, no
// spills since the strip resolve; K2 0.0989 -> 0.0980 ms against five,
// profiles/r05_ab_k2.txt).
#ifndef BMFR_K2_MINW
#define BMFR_K2_MINW 6
#endif
template <class IN>
__global__ __launch_bounds__(kTaaNT, BMFR_K2_MINW) void k_fused_taa(Params P, TaaArgs T) {
    __shared__ float4 Y[(kTaaW + 2) * (kTaaH + 2)];  // YCoCg (+ pad): one 16-byte read per neighbour
    __shared__ double sE[kPowrENum];
    __shared__ double2 sRP[kPowrRPNum];
    // Output tile of this launch (the whole image, or a multi-GPU tile whose
    // one-pixel halo lies inside the buffer region).
    const int gi = xcd_swizzle(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
    const int bxi = gi % gridDim.x, byi = gi / gridDim.x;
    forward_reach(T, blockIdx.x == 0 && blockIdx.y == 0);
    taa_tile<IN, kTaaH, false, kTaaNT, kStrip>(P, T, P.tx0 + bxi * kTaaW, P.ty0 + byi * kTaaH, Y, sE, sRP);
}

// ------------------------------------------------------------ halo copy --
// Rectangles of state planes <-> one packed buffer (multi-GPU halo exchange),
// all segments in one launch: blockIdx.y = segment.  Segments whose rows are
// 4-byte multiples copy by dword, the rest (spp rows) by byte.
__global__ __launch_bounds__(256) void k_halo_copy(HaloArgs a, uint8_t* __restrict__ buf, int unpack) {
    const HaloSeg& s = a.seg[blockIdx.y];
    uint8_t* plane = reinterpret_cast<uint8_t*>(s.plane);
    uint8_t* packed = buf + s.buf_off;
    const long total = (long)s.row_bytes * s.rows;
    const bool words = (s.row_bytes & 3) == 0 && (s.pitch & 3) == 0 && (s.plane & 3) == 0;
    const long stride = (long)gridDim.x * blockDim.x;
    if (words) {
        const int rw = s.row_bytes >> 2;
        for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total / 4; i += stride) {
            const long row = i / rw, col = i % rw;
            uint32_t* p = reinterpret_cast<uint32_t*>(plane + row * s.pitch) + col;
            uint32_t* q = reinterpret_cast<uint32_t*>(packed) + i;
            if (unpack) *p = *q;
            else *q = *p;
        }
    } else {
        for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += stride) {
            const long row = i / s.row_bytes, col = i % s.row_bytes;
            uint8_t* p = plane + row * s.pitch + col;
            if (unpack) *p = packed[i];
            else packed[i] = *p;
        }
    }
}

hipError_t launch_halo_copy(const HaloArgs& a, hipStream_t st, void* buf, int unpack) {
    if (a.nseg <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_halo_copy, dim3(64, a.nseg), dim3(256), 0, st, a, static_cast<uint8_t*>(buf), unpack);
    return hipGetLastError();
}

// ------------------------------------------------------------ noise table --
// add_random()'s noise term (bmfr.cl:173-182) depends only on the row, the
// feature and the frame, never on the block; K1 reads it from this table
// instead of re-hashing per element: table[(fb-1)*1024 + row] = random() - 0.5f
// for fb = 1..B-4; the kernel forms NOISE_AMOUNT*2.f*that in double as upstream.
// Tables of `frames` consecutive frames from `first` are made in one launch
// (one per kNoiseFrames frames), frame first + k at table + k * per_frame.
__global__ __launch_bounds__(256) void k_noise_table(int first, int frames, int buffers, float* __restrict__ table) {
    const int per_frame = (buffers - 4) * kBlockPixels;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= frames * per_frame) return;
    const int frame = first + i / per_frame, j = i % per_frame;
    const int fb = 1 + j / kBlockPixels, r = j % kBlockPixels;
    // add_random's addend (bmfr.cl:173-182) for row r of feature fb is
    // NOISE_AMOUNT * 2 (double) times this float: the same for every block, so
    // computed once per frame; the fitters form the double product (exactly
    // upstream's) where they add it -- half the bytes of storing the double.
    table[i] = hash_random((uint32_t)(r + fb * kBlockPixels + frame * buffers * kBlockPixels)) - 0.5f;
}

// ---------------------------------------------------------------- launch --
namespace {
dim3 grid2d(int w, int h, dim3 blk) { return dim3((w + blk.x - 1) / blk.x, (h + blk.y - 1) / blk.y); }
}  // namespace

hipError_t launch_accumulate_noisy(const Params& P, hipStream_t st, float2* prev_pixel, uint8_t* accept,
                                   const NoisyInputs& in, float* noisy_out, uint8_t* spp_cur, void* tmp,
                                   const Camera& cam, int frame) {
    const dim3 blk(16, 16);
    const dim3 grd = grid2d(P.margins_w, P.margins_h, blk);
    for (int pass = 0; pass < 2; ++pass) {
        hipLaunchKernelGGL(k_accumulate_noisy, grd, blk, 0, st, P, in, cam, frame, pass, prev_pixel,
                           accept, noisy_out, spp_cur, tmp);
    }
    return hipGetLastError();
}

// Feature counts with compiled kernels (bmfr_generic.h): FEATURES_NOT_SCALED
// 1..4 (1.f and / or the normal components) x FEATURES_SCALED 0..9
// (position monomials), any feature codes (bmfr.cpp:65-77); one translation
// unit per FEATURES_NOT_SCALED (bmfr_generic_ns*.hip).
bool fitter_supported(int ns, int fs) { return ns >= 1 && ns <= 4 && fs >= 0 && fs <= 9; }

hipError_t launch_fitter(const Params& P, hipStream_t st, float* weights, float* mins_maxs, void* tmp,
                         int frame) {
    switch (P.not_scaled) {
        case 1: return launch_fitter_ns<1>(P, st, weights, mins_maxs, tmp, frame);
        case 2: return launch_fitter_ns<2>(P, st, weights, mins_maxs, tmp, frame);
        case 3: return launch_fitter_ns<3>(P, st, weights, mins_maxs, tmp, frame);
        case 4: return launch_fitter_ns<4>(P, st, weights, mins_maxs, tmp, frame);
        default: return hipErrorInvalidValue;
    }
}

static hipError_t launch_fused_generic(const Params& P, hipStream_t st, const FusedArgs& A) {
    switch (P.not_scaled) {
        case 1: return launch_fused_block_ns<1>(P, st, A);
        case 2: return launch_fused_block_ns<2>(P, st, A);
        case 3: return launch_fused_block_ns<3>(P, st, A);
        case 4: return launch_fused_block_ns<4>(P, st, A);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_weighted_sum(const Params& P, hipStream_t st, const float* weights,
                               const float* mins_maxs, float* out, const float* normals,
                               const float* positions, int frame) {
    const dim3 blk(64, 4);
    hipLaunchKernelGGL(k_weighted_sum, grid2d(P.width, P.height, blk), blk, 0, st, P, weights,
                       mins_maxs, out, normals, positions, frame);
    return hipGetLastError();
}

hipError_t launch_accumulate_filtered(const Params& P, hipStream_t st, const float* filtered,
                                      const float2* prev_pixel, const uint8_t* accept,
                                      const float* albedo, float* tone, const uint8_t* spp,
                                      const float* acc_prev, float* acc, int frame) {
    const dim3 blk(64, 4);
    hipLaunchKernelGGL(k_accumulate_filtered, grid2d(P.width, P.height, blk), blk, 0, st, P, filtered,
                       prev_pixel, accept, albedo, tone, spp, acc_prev, acc, frame);
    return hipGetLastError();
}

hipError_t launch_taa(const Params& P, hipStream_t st, const float2* prev_pixel, const float* new_frame,
                      float* result, const float* prev_frame, int frame) {
    const dim3 blk(64, 4);
    hipLaunchKernelGGL(k_taa, grid2d(P.width, P.height, blk), blk, 0, st, P, prev_pixel, new_frame,
                       result, prev_frame, frame);
    return hipGetLastError();
}

hipError_t launch_noise_tables(const Params& P, hipStream_t st, int first, int frames, float* table) {
    const int n = frames * (P.buffers - 4) * kBlockPixels;
    hipLaunchKernelGGL(k_noise_table, dim3((n + 255) / 256), dim3(256), 0, st, first, frames, P.buffers, table);
    return hipGetLastError();
}

hipError_t launch_noise_table(const Params& P, hipStream_t st, const FusedArgs& A) {
    return launch_noise_tables(P, st, A.frame, 1, A.noise_table);
}

hipError_t launch_fused_k1_blocks(const Params& P, hipStream_t st, const FusedArgs& A) {
    if (P.nbx <= 0 || P.nby <= 0 || P.ring < 0) return hipSuccess;
    return fused_cols_supported(P) ? launch_fused_k1_cols(P, st, A) : launch_fused_k1(P, st, A);
}

hipError_t launch_fused_k2(const Params& P, hipStream_t st, const FusedArgs& A) {
    const dim3 grd((P.tx1 - P.tx0 + kTaaW - 1) / kTaaW, (P.ty1 - P.ty0 + kTaaH - 1) / kTaaH);
    if (P.input_half) hipLaunchKernelGGL((k_fused_taa<_Float16>), grd, dim3(kTaaNT), 0, st, P, taa_args(A));
    else hipLaunchKernelGGL((k_fused_taa<float>), grd, dim3(kTaaNT), 0, st, P, taa_args(A));
    return hipGetLastError();
}

hipError_t launch_fused_frame(const Params& P, hipStream_t st, const FusedArgs& A, hipEvent_t mid) {
    hipError_t e;
    // One launch for the frame, unless K1 and K2 are timed apart (mid event).
    // One launch for the frame (K1 blocks, then the TAA tiles waiting on their
    // completion flags) below kTwoLaunchBlocks K1 blocks; above, K1 and K2
    // as two launches, where K2 runs at its own occupancy (90 VGPRs, five
    // waves per SIMD; inside the frame kernel it has K1's four) and the gap
    // between the launches is small beside the frame: measured (round 4,
    // profiles/r04_bench_two_launch.txt) 4K 0.3758 -> 0.3711, 8K 1.409 ->
    // 1.365, f32 tmp_data 0.444 -> 0.425 ms/frame, but 1080p 0.111 -> 0.118.
    const bool one = P.frame_launches == 1 || (P.frame_launches == 0 && k1_blocks(P) < kTwoLaunchBlocks);
    if (!mid && A.done && frame_fused_supported(P) && one) return launch_fused_frame_one(P, st, A);
    if (fused_supported(P)) {
        if ((e = launch_fused_k1_blocks(P, st, A)) != hipSuccess) return e;
        if (mid) (void)hipEventRecord(mid, st);
        return launch_fused_k2(P, st, A);
    }
    e = launch_fused_generic(P, st, A);
    if (e != hipSuccess) return e;
    if (mid) (void)hipEventRecord(mid, st);
    return launch_taa(P, st, A.prev_pixel_out, A.tone_out, A.result_out, A.result_prev, A.frame);
}

}  // namespace bmfr
