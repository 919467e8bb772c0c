// bmfr_launch.h -- host-side launchers of bmfr_kernels.hip (used by the C ABI).
#pragma once

#include <hip/hip_runtime.h>

#include "bmfr_kernels.h"
#include "bmfr_taa_tile.h"

namespace bmfr {

// Halo exchange: rectangle segments of state planes and their place in a
// packed buffer (bmfr_halo_copy).
struct HaloSeg {
    unsigned long long plane;  // device address of the rectangle's first byte in the plane
    long long buf_off;         // byte offset of the segment in the packed buffer (16-byte aligned)
    int row_bytes, rows, pitch;
};
constexpr int kMaxHaloSegs = 64;
struct HaloArgs {
    HaloSeg seg[kMaxHaloSegs];
    int nseg;
};
hipError_t launch_halo_copy(const HaloArgs& a, hipStream_t st, void* buf, int unpack);

// Arguments of one fused frame (K1 + K2).
struct FusedArgs {
    NoisyInputs in;
    Camera cam;
    int frame;
    const float* albedo;
    const float* acc_prev;
    const float* result_prev;
    float* noisy_out;
    uint8_t* spp_out;
    float2* prev_pixel_out;
    float* acc_out;
    float* tone_out;
    float* result_out;
    float* noise_table;   // (B-4) * 1024 noise factors rnd-0.5f (the term is NOISE_AMOUNT*2 * that, in double), context-owned
    unsigned* reach;      // tiled contexts: max overshoot (px) of reprojection taps past the valid state
    unsigned* reach_host; // tiled contexts: page-locked report of it (see TaaArgs)
    unsigned long long* stamps;  // diagnostic build: 8 timestamps per block, or null
    unsigned* done;       // one-launch frame: per K1 block, the epoch of the launch that completed it
    unsigned epoch;       // this launch's epoch (context-wide launch counter, never 0)
    unsigned* sync_err;   // page-locked report of an exhausted wait (kSyncPivot / kSyncTile), or null
};

// Kernel arguments of the fused K1 (canonical feature lists).
struct K1Args {
    NoisyInputs in;
    Camera cam;
    int frame;
    const float* acc_prev;
    float* noisy_out;
    uint8_t* spp_out;
    float2* prev_pixel_out;
    float* acc_out;
    const float* noise;
    unsigned* reach;
    unsigned long long* stamps;
    unsigned* done;
    unsigned epoch;
    unsigned* sync_err;
};
inline K1Args k1_args(const FusedArgs& A) {
    return K1Args{A.in,      A.cam,         A.frame, A.acc_prev, A.noisy_out, A.spp_out, A.prev_pixel_out,
                  A.acc_out, A.noise_table, A.reach, A.stamps,   A.done,      A.epoch,   A.sync_err};
}
inline TaaArgs taa_args(const FusedArgs& A) {
    return TaaArgs{A.acc_out, A.albedo, A.prev_pixel_out, A.result_out, A.result_prev, A.frame, A.reach,
                   A.reach_host, A.done, A.epoch, A.sync_err};
}

bool fitter_supported(int not_scaled, int scaled);
// Work-groups of a K1 launch (the rectangle, or its ring).
inline int k1_blocks(const Params& P) { return P.ring > 0 ? P.ring : P.nbx * P.nby; }
// launch_fused_frame: frames of at least this many K1 blocks run as two
// launches (K1, K2) instead of one (-DBMFR_FRAME_TWO_LAUNCH_BLOCKS=N).
#ifndef BMFR_FRAME_TWO_LAUNCH_BLOCKS
#define BMFR_FRAME_TWO_LAUNCH_BLOCKS 4096
#endif
constexpr int kTwoLaunchBlocks = BMFR_FRAME_TWO_LAUNCH_BLOCKS;
bool fused_supported(const Params& P);
// The canonical path tone-maps in K2 (bmfr.cl:851-856), for each tile pixel
// and its 1-px halo.  f32 tmp_data: row-split K1 (bmfr_fused.hip).
hipError_t launch_fused_k1(const Params& P, hipStream_t st, const FusedArgs& A);
// Column-split K1 (bmfr_fused_cols.hip): half tmp_data.
bool fused_cols_supported(const Params& P);
hipError_t launch_fused_k1_cols(const Params& P, hipStream_t st, const FusedArgs& A);

hipError_t launch_accumulate_noisy(const Params& P, hipStream_t st, float2* prev_pixel, uint8_t* accept,
                                   const NoisyInputs& in, float* noisy_out, uint8_t* spp_cur, void* tmp,
                                   const Camera& cam, int frame);
hipError_t launch_fitter(const Params& P, hipStream_t st, float* weights, float* mins_maxs, void* tmp,
                         int frame);
hipError_t launch_weighted_sum(const Params& P, hipStream_t st, const float* weights,
                               const float* mins_maxs, float* out, const float* normals,
                               const float* positions, int frame);
hipError_t launch_accumulate_filtered(const Params& P, hipStream_t st, const float* filtered,
                                      const float2* prev_pixel, const uint8_t* accept,
                                      const float* albedo, float* tone, const uint8_t* spp,
                                      const float* acc_prev, float* acc, int frame);
hipError_t launch_fused_frame(const Params& P, hipStream_t st, const FusedArgs& A, hipEvent_t mid = nullptr);
// The parts of launch_fused_frame (canonical feature lists): the frame's
// noise table, K1 over the block rectangle of P (bx0, by0, nbx, nby; empty:
// nothing), K2 over P's output tile.
hipError_t launch_noise_table(const Params& P, hipStream_t st, const FusedArgs& A);
// Noise tables of frames first .. first+frames-1, back to back from `table`.
constexpr int kNoiseFrames = 64;
hipError_t launch_noise_tables(const Params& P, hipStream_t st, int first, int frames, float* table);
hipError_t launch_fused_k1_blocks(const Params& P, hipStream_t st, const FusedArgs& A);
// Sequence kernel (bmfr_process_sequence): K1 of a frame (A, or none) and K2
// of the frame before it (A2, or none) in one launch.
bool seq_fused_supported(const Params& P);
// One-launch frame (bmfr_process_frame; a tiled context's border part): K1
// blocks, then the TAA tiles of the same frame, each waiting on the
// completion flags of the K1 blocks under its footprint.
bool frame_fused_supported(const Params& P);
hipError_t launch_fused_frame_one(const Params& P, hipStream_t st, const FusedArgs& A);
// The same with the row-split K1 (f32 tmp_data, bmfr_fused.hip).
hipError_t launch_fused_rows_frame_one(const Params& P, hipStream_t st, const FusedArgs& A);
hipError_t launch_fused_k1_taa(const Params& P, hipStream_t st, const FusedArgs* A, const Params& P2,
                               const FusedArgs* A2);
hipError_t launch_fused_k2(const Params& P, hipStream_t st, const FusedArgs& A);
hipError_t launch_taa(const Params& P, hipStream_t st, const float2* prev_pixel, const float* new_frame,
                      float* result, const float* prev_frame, int frame);

}  // namespace bmfr
