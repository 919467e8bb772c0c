/* bmfr_oracle.h -- CPU restatement of the BMFR per-frame pipeline.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (bmfr_amd/, include/,
 * libbmfr) may include, link or call this.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg use it, and only as the checker / the timed
 * CPU baseline.
 *
 * Every function restates one OpenCL kernel of the reference
 * (/root/reference/opencl/bmfr.cl) with the arithmetic the reference has when
 * it is compiled by ROCm clang for gfx950 with IEEE-strict options
 * (-ffp-contract=off -cl-fp32-correctly-rounded-divide-sqrt): every float op
 * rounded once, no contraction in the kernel source, and the OpenCL library's
 * dot() lowered to an fma chain (ROCm device-libs opencl.bc `_Z3dotDv3_fS_`:
 * fmuladd(z, fmuladd(y, x*x'))).  Pinning: oracle/ref_run.py executes the
 * reference kernels themselves (compiled from /root/reference by
 * oracle/Makefile) on an MI355X and tests/golden/ holds their outputs; the
 * oracle is checked bit-for-bit against those vectors (powr aside, see
 * oracle_accumulate_filtered_data).
 *
 * Buffer layouts are the reference's (bmfr.cpp:315-347):
 *   float3 images   : interleaved RGB f32, row stride IMAGE_WIDTH
 *   spp / accept    : u8 per pixel, stride IMAGE_WIDTH
 *   prev_pixel      : float2 per pixel
 *   tmp_data        : [block][feature][32*32] block-major (bmfr.cl:455-464),
 *                     IEEE half bits (u16) or f32
 *   weights         : [block][B-3][3] f32      mins_maxs: [block][FS][2] f32
 */
#ifndef BMFR_ORACLE_H
#define BMFR_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_MAX_FEATURES 16

/* Feature codes: the monomials the reference's FEATURE_BUFFERS text may name
 * (bmfr.cpp:65-77).  Same numbering as include/bmfr.h. */
enum {
    ORACLE_F_ONE = 0,
    ORACLE_F_NX, ORACLE_F_NY, ORACLE_F_NZ,
    ORACLE_F_PX, ORACLE_F_PY, ORACLE_F_PZ,
    ORACLE_F_PX2, ORACLE_F_PY2, ORACLE_F_PZ2,
    ORACLE_F_PX3, ORACLE_F_PY3, ORACLE_F_PZ3
};

typedef struct oracle_cfg {
    int width, height;              /* IMAGE_WIDTH / IMAGE_HEIGHT       bmfr.cpp:39-40 */
    int n_not_scaled, n_scaled;     /* FEATURES_NOT_SCALED / _SCALED    bmfr.cpp:193-202 */
    int codes[ORACLE_MAX_FEATURES]; /* FEATURE_BUFFERS, in order        bmfr.cpp:214 */
    double noise_amount;            /* NOISE_AMOUNT (a double literal)  bmfr.cpp:58 */
    float blend_alpha;              /* BLEND_ALPHA                      bmfr.cpp:60 */
    float second_blend_alpha;       /* SECOND_BLEND_ALPHA               bmfr.cpp:61 */
    float taa_blend_alpha;          /* TAA_BLEND_ALPHA                  bmfr.cpp:62 */
    float position_limit_sq;        /* convert_float(POSITION_LIMIT_SQUARED) bmfr.cl:393 */
    float normal_limit_sq;          /* convert_float(NORMAL_LIMIT_SQUARED)   bmfr.cl:404 */
    int half_tmp;                   /* USE_HALF_PRECISION_IN_TMP_DATA   bmfr.cpp:88 */
} oracle_cfg;

int oracle_num_blocks(const oracle_cfg *c);

void oracle_accumulate_noisy_data(const oracle_cfg *c,
    float *out_prev_frame_pixel, uint8_t *accept_bools,
    const float *current_normals, const float *previous_normals,
    const float *current_positions, const float *previous_positions,
    float *current_noisy, const float *previous_noisy,
    const uint8_t *previous_spp, uint8_t *current_spp,
    void *tmp_data, const float prev_frame_camera_matrix[16],
    const float pixel_offset[2], int frame_number);

void oracle_fitter(const oracle_cfg *c, float *weights, float *mins_maxs,
    void *tmp_data, int frame_number);

void oracle_weighted_sum(const oracle_cfg *c, const float *weights,
    const float *mins_maxs, float *output, const float *current_normals,
    const float *current_positions, int frame_number);

void oracle_accumulate_filtered_data(const oracle_cfg *c,
    const float *filtered_frame, const float *in_prev_frame_pixel,
    const uint8_t *accept_bools, const float *albedo, float *tone_mapped_frame,
    const uint8_t *current_spp, const float *accumulated_prev_frame,
    float *accumulated_frame, int frame_number);

void oracle_taa(const oracle_cfg *c, const float *in_prev_frame_pixel,
    const float *new_frame, float *result_frame, const float *prev_frame,
    int frame_number);

/* IEEE binary16 helpers (round-to-nearest-even), exposed for the tests. */
uint16_t oracle_f32_to_f16(float f);
float oracle_f16_to_f32(uint16_t h);

/* Threads used by the OpenMP loops (1 when built without OpenMP). */
int oracle_threads(void);

#ifdef __cplusplus
}
#endif
#endif
