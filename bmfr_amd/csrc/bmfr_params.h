// bmfr_params.h -- resolved per-context constants handed to every kernel.
//
// Host code builds one Params from a bmfr_config (bmfr_capi.hip); the values
// are exactly what the reference kernels see through their -D options
// (bmfr.cpp:205-232), e.g. the limits are float(%g text of the double).
#pragma once

#include <stdint.h>

namespace bmfr {

enum FeatureCode : int {
    kFeatOne = 0,
    kFeatNx, kFeatNy, kFeatNz,
    kFeatPx, kFeatPy, kFeatPz,
    kFeatPx2, kFeatPy2, kFeatPz2,
    kFeatPx3, kFeatPy3, kFeatPz3,
};

constexpr int kEdge = 32;                 // BLOCK_EDGE_LENGTH
constexpr int kBlockPixels = kEdge * kEdge;  // BLOCK_PIXELS
constexpr int kLocal = 256;               // LOCAL_SIZE (fitter work-items)
constexpr int kSubs = kBlockPixels / kLocal; // rows per fitter work-item
constexpr int kMaxFeatures = 16;

struct Params {
    int width, height;            // IMAGE_WIDTH / IMAGE_HEIGHT
    int workset_w, workset_h;     // WORKSET_WIDTH / HEIGHT
    int margins_w, margins_h;     // WORKSET_WITH_MARGINS_WIDTH / HEIGHT
    int blocks_x, blocks_y;       // margins / 32
    int buffers;                  // BUFFER_COUNT
    int not_scaled, scaled;       // FEATURES_NOT_SCALED / FEATURES_SCALED
    int codes[kMaxFeatures];      // FEATURE_BUFFERS
    double noise2;                // NOISE_AMOUNT * 2.f, in double (bmfr.cl:179)
    float blend_alpha, second_blend_alpha, taa_blend_alpha;
    float position_limit_sq, normal_limit_sq;
    int half_tmp;                 // USE_HALF_PRECISION_IN_TMP_DATA
    int input_half;               // bmfr_config.input_half: frame input planes are half3
    int library_powr;             // bmfr_config.library_powr: tone map with __ocml_powr_f32
    int fast_fit;                 // bmfr_config.fast_fit: fused trailing update (+ butterfly reductions, hardware sqrt / rcp) in the fused K1
    // Buffer region (multi-GPU tiles): every plane of the fused path holds the
    // image pixels [ox, ox + stride) x [oy, oy + rows), row stride `stride`.
    // Untiled: 0, 0, width, height -- the reference's layout.
    int ox, oy, stride, rows;
    // Per launch: the blocks of the shifted grid K1 covers (bx0 + g % nbx,
    // by0 + g / nbx) and the output tile [tx0, tx1) x [ty0, ty1) of K2.
    int bx0, by0, nbx, nby;
    // ring > 0: the launch covers only the blocks of that rectangle outside
    // the inner rectangle [rx0, rx1) x [ry0, ry1) (a tile's border ring,
    // bmfr_process_frame_border), ring = their count.
    int ring, rx0, ry0, rx1, ry1;
    int tx0, ty0, tx1, ty1;
    // Tiled contexts (check_reach = 1): the previous frame's state is valid
    // only in [vx0, vx1) x [vy0, vy1) for this launch -- the tile before the
    // halo exchange (interior blocks), the region after it.  K1 reports the
    // largest distance by which an in-image reprojection tap (bmfr.cl:374-419)
    // falls outside it (include/bmfr.h: BMFR_ERROR_HALO_EXCEEDED).
    // [wx0, wx1) x [wy0, wy1): where the previous TAA output is valid -- it
    // bounds the taps of the tile's own pixels, which K2 reuses for its
    // bilinear read of that output (bmfr.cl:924-944).
    int check_reach;
    int vx0, vy0, vx1, vy1;
    int wx0, wy0, wx1, wy1;
    // Bounded waits of the fused kernels (K1's LDS pivot flags, the
    // one-launch frame's K1 completion flags): a wait gives up after
    // max_polls sleeps (4 * max_polls for a TAA tile) and reports
    // BMFR_ERROR_SYNC_TIMEOUT instead of running on with incomplete data.
    // kDefaultMaxPolls unless set by bmfr_debug_sync (include/bmfr_debug.h).
    int max_polls;
    // Diagnostics (bmfr_debug_sync): in the one-launch frame, every K1 block
    // g with g % kDelayStride == kDelayPhase sleeps debug_delay * 127 * 64
    // shader cycles before it publishes its completion flag, so TAA tiles
    // really wait.  0: off.
    int debug_delay;
    // Host side only (launch_fused_frame): kernel launches of an untiled
    // frame -- 0 by the frame's size (kTwoLaunchBlocks), 1 or 2 forced
    // (include/bmfr_debug.h bmfr_debug_frame_launches).
    int frame_launches;
};
constexpr int kDefaultMaxPolls = 1 << 20;
constexpr int kDelayStride = 61, kDelayPhase = 7;

// BLOCK_OFFSETS (bmfr.cl:267-285), host copy of the device table in
// bmfr_device.h: the grid shift of frame f is kBlockOffsetTable[f % 16].
constexpr int kBlockOffsetTable[16][2] = {
    {-14, -14}, {4, -6}, {-8, 14}, {8, 0}, {-10, -8}, {2, 12}, {12, -12}, {-10, 0},
    {12, 14}, {-8, -16}, {6, 6}, {-2, -2}, {6, -14}, {-16, 12}, {14, -4}, {-6, 4}};

}  // namespace bmfr
