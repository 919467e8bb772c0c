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
    int fused_variant;            // 0 = default, 1 = generic-feature K1, 2 = tone map in K1, 3 = row-split K1 (A/B diagnostics)
};

}  // namespace bmfr
