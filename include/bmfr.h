/* bmfr.h -- C ABI of libbmfr, the MI355X-native BMFR denoiser.
 *
 * This is the drop-in boundary for the reference's hot path, the per-frame
 * pipeline of /root/reference/opencl/bmfr.cl driven by tasks() in
 * /root/reference/opencl/bmfr.cpp.  The reference has no plugin API: its
 * boundary is (a) the JIT `-D` option set of bmfr.cpp:205-232, mirrored here
 * by bmfr_config, and (b) the five OpenCL kernel signatures with the argument
 * binding of bmfr.cpp:349-383,429-476, mirrored by the five stage entry
 * points below with the same argument roles and buffer layouts.  On top,
 * bmfr_process_frame runs one whole frame (the loop body of
 * bmfr.cpp:417-485) through the fused MI355X kernels.
 *
 * Conventions
 *  - Plain C: pointers, sizes and a status code.  No exceptions cross the ABI
 *    (the reference maps cl::Error to a return code, bmfr.cpp:558-578).
 *  - All buffer pointers are device pointers (hipMalloc / torch tensors).
 *  - `stream` is a hipStream_t passed as void* (NULL = the null stream).
 *  - Layouts (bmfr.cpp:315-347): float3 images are interleaved RGB f32 with
 *    row stride image_width; u8 planes (spp, accept) and float2 prev-pixel
 *    planes likewise; tmp_data is [block][feature][32*32] (bmfr.cl:455-464)
 *    in IEEE half (use_half_precision_in_tmp_data = 1) or f32; weights are
 *    [block][B-3][3] f32; mins_maxs are [block][FEATURES_SCALED][2] f32.
 *  - A context is not thread-safe; contexts are independent (one per GPU).
 */
#ifndef BMFR_H
#define BMFR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BMFR_VERSION_MAJOR 0
#define BMFR_VERSION_MINOR 2

#define BMFR_BLOCK_EDGE_LENGTH 32 /* bmfr.cpp:104; other sizes unsupported, as upstream */
#define BMFR_MAX_FEATURES 16      /* NOT_SCALED + SCALED feature buffers */

typedef enum bmfr_status {
    BMFR_OK = 0,
    BMFR_ERROR_INVALID_ARGUMENT = 1,
    BMFR_ERROR_UNSUPPORTED = 2,     /* e.g. a feature count with no compiled kernel */
    BMFR_ERROR_OUT_OF_MEMORY = 3,
    BMFR_ERROR_HIP = 4,             /* a HIP runtime call failed (see bmfr_last_hip_error) */
    BMFR_ERROR_NO_DEVICE = 5,
    BMFR_ERROR_HALO_EXCEEDED = 6,   /* tiled context: a frame reprojected past the exchanged halo
                                       (see tile_halo, bmfr_halo_status) */
    BMFR_ERROR_SYNC_TIMEOUT = 7     /* a fused kernel's bounded wait for another work-group gave up
                                       (see bmfr_frame_status): that frame's output is not valid */
} bmfr_status;

/* Feature buffer monomials.  The reference pastes C expressions into the
 * kernels (NOT_SCALED_FEATURE_BUFFERS / SCALED_FEATURE_BUFFERS, bmfr.cpp:65-77
 * -> FEATURE_BUFFERS, bmfr.cl:448-453,727-729); this ABI names them. */
typedef enum bmfr_feature {
    BMFR_FEATURE_ONE = 0, /* "1.f" */
    BMFR_FEATURE_NORMAL_X, BMFR_FEATURE_NORMAL_Y, BMFR_FEATURE_NORMAL_Z,
    BMFR_FEATURE_POSITION_X, BMFR_FEATURE_POSITION_Y, BMFR_FEATURE_POSITION_Z,
    BMFR_FEATURE_POSITION_X2, BMFR_FEATURE_POSITION_Y2, BMFR_FEATURE_POSITION_Z2,
    BMFR_FEATURE_POSITION_X3, BMFR_FEATURE_POSITION_Y3, BMFR_FEATURE_POSITION_Z3,
    BMFR_FEATURE_COUNT_
} bmfr_feature;

/* The reference's #define surface (bmfr.cpp:32-118, forwarded as -D at
 * bmfr.cpp:205-232).  Fill with bmfr_config_default() and override. */
typedef struct bmfr_config {
    int image_width;                     /* IMAGE_WIDTH  (bmfr.cpp:39) */
    int image_height;                    /* IMAGE_HEIGHT (bmfr.cpp:40) */
    int features_not_scaled;             /* FEATURES_NOT_SCALED (bmfr.cpp:195-196) */
    int features_scaled;                 /* FEATURES_SCALED     (bmfr.cpp:198-199) */
    int feature_buffers[BMFR_MAX_FEATURES]; /* FEATURE_BUFFERS: not-scaled then scaled */
    double noise_amount;                 /* NOISE_AMOUNT 1e-2 (a double, bmfr.cpp:58) */
    float blend_alpha;                   /* BLEND_ALPHA 0.2f        (bmfr.cpp:60) */
    float second_blend_alpha;            /* SECOND_BLEND_ALPHA 0.1f (bmfr.cpp:61) */
    float taa_blend_alpha;               /* TAA_BLEND_ALPHA 0.2f    (bmfr.cpp:62) */
    double position_limit_squared;       /* camera_matrices.h value; used as the
                                            kernel sees it: float(%g text), bmfr.cpp:226 */
    double normal_limit_squared;         /* idem, bmfr.cpp:227 */
    int use_half_precision_in_tmp_data;  /* USE_HALF_PRECISION_IN_TMP_DATA 1 (bmfr.cpp:88) */
    /* Spatial tile of a larger frame (multi-GPU sharding);
     * 0/0/0/0 = whole image.  image_width/height stay the WHOLE frame: block
     * grid, mirroring at the borders and reprojection are the whole frame's,
     * so a tile's output equals the same pixels of the untiled output.  The
     * context's buffers then cover the tile's REGION = the tile grown by
     * tile_halo pixels on each side, clipped to the frame (bmfr_sizes
     * region_*): every plane passed to bmfr_process_frame and every state
     * plane holds that region with row stride region_width.  Before each
     * frame > 0 the caller refreshes the region's halo ring of the state
     * planes (noisy_accumulated, spp, filtered_accumulated, result of
     * bmfr_state(previous = 0)) from the neighbouring tiles, which own those
     * pixels -- at least the parts bmfr_halo_need names for that frame.  Exact for scene motion below tile_halo - 34 pixels per frame
     * (32: blocks reaching past the tile, 2: TAA + bilinear taps); the
     * reference reprojects to any pixel (bmfr.cl:343-356), so the kernels
     * check it: a frame whose reprojection taps reach past the state that
     * is valid for them (the tile before the halo exchange, the region after
     * it) makes bmfr_halo_status -- and every later bmfr_process_frame* call
     * until frame_number 0 starts a new sequence -- return
     * BMFR_ERROR_HALO_EXCEEDED instead of diverging silently from the
     * untiled frame.  Canonical feature lists, fused path only (the stage API
     * rejects tiled contexts). */
    int tile_x, tile_y, tile_width, tile_height;
    int tile_halo;
    /* Input planes of bmfr_process_frame (noisy, normals, positions, albedo
     * and the previous normals / positions) in IEEE half, interleaved RGB
     * (6 bytes per pixel), instead of f32: the .exr files' own HALF channels
     * kept as they are (the reference converts them to FLOAT on load,
     * bmfr.cpp:157-159).  Values are widened exactly to f32 on load, so the
     * output equals the f32 path's on the widened planes bit for bit.
     * Canonical feature lists, fused path only (stage API: unsupported). */
    int input_half;
    /* powr(x, 0.454545f) of the tone map (bmfr.cl:854), whose rounding
     * OpenCL leaves to the device: 0 (default) = correctly rounded, equal to
     * the CPU oracle's (float)pow for every input, ~20 instructions;
     * 1 = the device library's __ocml_powr_f32, i.e. what the reference
     * kernel compiled for gfx950 computes (one in four results 1 ulp from
     * the correctly rounded one), ~130 instructions. */
    int library_powr;
    /* Householder trailing update of the fitter (bmfr.cl:606-655), each
     * element's t - 2 u dot / |u|^2: 0 (default) = upstream's roundings (u * c,
     * then / |u|^2, then the subtraction; the output equals the reference's
     * strict build bit for bit); 1 = one fused multiply-add on the block-wide
     * factor 2 dot / |u|^2, the wave-wide sums, minima and maxima as
     * butterflies, the noise added in f32 and the pivot's square root,
     * reciprocals and feature scaling at hardware precision (half tmp_data;
     * the f32 tmp_data K1 fuses the update only) -- no longer
     * bit-exact: TAA output within 1.2e-5 relative L2 of the reference's
     * strict build and 1.6e-5 of its default build at 3840x2160 (3.0e-5 at
     * B = 16; the two reference builds differ by ~1.2e-5), ~15 % less K1
     * time.  Applies to the fused K1 (canonical feature lists, half
     * or f32 tmp_data, every frame API); the stage fitter (bmfr_fitter) and
     * the arbitrary-feature-list K1 run the exact update. */
    int fast_fit;
} bmfr_config;

/* Sizes derived from a config (bmfr.cpp:104-118, 316-343). */
typedef struct bmfr_sizes {
    int buffer_count;       /* BUFFER_COUNT = not_scaled + scaled + 3 */
    int r_edge;             /* R_EDGE = BUFFER_COUNT - 2 */
    int workset_width, workset_height;                           /* WORKSET_* */
    int workset_with_margins_width, workset_with_margins_height; /* WORKSET_WITH_MARGINS_* */
    int blocks;             /* fitter work-groups, FITTER_GLOBAL / 256 */
    size_t tmp_data_bytes;  /* in_buffer, bmfr.cpp:322-324 */
    size_t weights_bytes;   /* bmfr.cpp:338-339 */
    size_t mins_maxs_bytes; /* sized from FEATURES_SCALED (bmfr.cpp:340 assumes 6) */
    size_t image_bytes;     /* one float3 plane, W*H*3*4 */
    /* Buffer region of the context (the whole frame unless tiled): pixels
     * [region_x, region_x + region_width) x [region_y, region_y + region_height). */
    int region_x, region_y, region_width, region_height;
    size_t region_bytes;    /* one float3 plane of the region */
    /* Kernel launches of an untiled bmfr_process_frame on the fused path
     * (canonical feature lists; profiling off): 1 (K1 blocks, then the TAA
     * tiles on completion flags) for frames below 4096 K1 blocks (`blocks`),
     * 2 (K1, then K2) from there -- measured faster at 4K / 8K, slower at
     * 1080p. */
    int frame_launches;
} bmfr_sizes;

typedef struct bmfr_ctx bmfr_ctx;

void bmfr_config_default(bmfr_config *cfg, int image_width, int image_height);
bmfr_status bmfr_config_sizes(const bmfr_config *cfg, bmfr_sizes *out);
const char *bmfr_status_string(bmfr_status s);
int bmfr_last_hip_error(void);
/* Identity of the compiled library: SHA-256 (hex) of the sources it was built
 * from, followed by "+<flags>" for a variant build.  No reference counterpart
 * (the reference JIT-compiles bmfr.cl at start-up, bmfr.cpp:234-243, so its
 * binary is always its source); here it ties a shipped binary to its tree. */
const char *bmfr_build_id(void);

/* Replaces clutils::CLEnv + the addContext/addQueue/addProgram calls
 * (bmfr.cpp:183-243): binds a HIP device and selects the kernels. */
bmfr_status bmfr_create(const bmfr_config *cfg, int hip_device, bmfr_ctx **out);
bmfr_status bmfr_destroy(bmfr_ctx *ctx);
bmfr_status bmfr_get_sizes(const bmfr_ctx *ctx, bmfr_sizes *out);

/* ---- Stage API: one entry per reference kernel, same argument roles ---- */

/* accumulate_noisy_data, bmfr.cl:290-308 (args bound at bmfr.cpp:351-352,429-447).
 * current_noisy is in/out like the reference.  Margin work-items read the
 * colours current_noisy held before the call (race-free form of
 * bmfr.cl:316-322 vs 478-481). */
bmfr_status bmfr_accumulate_noisy_data(bmfr_ctx *ctx, void *stream,
    float *out_prev_frame_pixel, uint8_t *accept_bools,
    const float *current_normals, const float *previous_normals,
    const float *current_positions, const float *previous_positions,
    float *current_noisy, const float *previous_noisy,
    const uint8_t *previous_spp, uint8_t *current_spp, void *tmp_data,
    const float prev_frame_camera_matrix[16], const float pixel_offset[2],
    int frame_number);

/* fitter, bmfr.cl:490-501 (args bound at bmfr.cpp:363-367,449-453).  The LDS
 * scratch arguments of the OpenCL kernel are internal here. */
bmfr_status bmfr_fitter(bmfr_ctx *ctx, void *stream, float *weights, float *mins_maxs,
    void *tmp_data, int frame_number);

/* weighted_sum, bmfr.cl:703-710 (bmfr.cpp:370-372,455-461).  current_noisy is
 * accepted for signature parity; the reference uses it only for debugging. */
bmfr_status bmfr_weighted_sum(bmfr_ctx *ctx, void *stream, const float *weights,
    const float *mins_maxs, float *output, const float *current_normals,
    const float *current_positions, const float *current_noisy, int frame_number);

/* accumulate_filtered_data, bmfr.cl:761-770 (bmfr.cpp:375-379,463-469). */
bmfr_status bmfr_accumulate_filtered_data(bmfr_ctx *ctx, void *stream,
    const float *filtered_frame, const float *in_prev_frame_pixel,
    const uint8_t *accept_bools, const float *albedo, float *tone_mapped_frame,
    const uint8_t *current_spp, const float *accumulated_prev_frame,
    float *accumulated_frame, int frame_number);

/* taa, bmfr.cl:860-865 (bmfr.cpp:382-383,471-476). */
bmfr_status bmfr_taa(bmfr_ctx *ctx, void *stream, const float *in_prev_frame_pixel,
    const float *new_frame, float *result_frame, const float *prev_frame,
    int frame_number);

/* ---- Frame API: the loop body of bmfr.cpp:417-485 on fused kernels ---- */

/* One frame's inputs (the four planes uploaded at bmfr.cpp:420-427) plus the
 * previous frame's normals/positions (the Double_buffer halves the reference
 * keeps, bmfr.cpp:316-319).  Temporal state (accumulated noisy colour, spp,
 * accumulated filtered colour, TAA output) lives in the context and is
 * double-buffered and swapped per frame like bmfr.cpp:482-484. */
typedef struct bmfr_frame_inputs {  /* float3 planes, or half3 with input_half */
    const void *noisy;           /* 1-spp colour (demodulated) */
    const void *normals;         /* shading normals */
    const void *positions;       /* world positions */
    const void *albedo;
    const void *prev_normals;    /* previous frame's normals (ignored at frame 0) */
    const void *prev_positions;  /* previous frame's positions (ignored at frame 0) */
} bmfr_frame_inputs;

/* prev_frame_camera_matrix: column-major view-projection of frame-1
 * (camera_matrices[max(frame-1,0)], bmfr.cpp:440-442); pixel_offset: the
 * frame's jitter (pixel_offsets[frame], bmfr.cpp:443-444).  frame_number 0
 * starts a new sequence. */
bmfr_status bmfr_process_frame(bmfr_ctx *ctx, void *stream, const bmfr_frame_inputs *in,
    const float prev_frame_camera_matrix[16], const float pixel_offset[2], int frame_number);

/* bmfr_process_frame in two calls, to overlap a tiled context's halo
 * exchange with compute.  _interior (noise table + the K1
 * blocks whose reads of the previous frame's state stay inside the tile, so
 * they need no halo) may be issued BEFORE the caller refreshes the halo ring
 * of bmfr_state(previous = 0) -- which still names the previous frame's
 * state until _border returns -- and runs while the exchange is in flight;
 * _border (same arguments, after the refresh is ordered before it on
 * `stream`) launches the remaining blocks and K2 and completes the frame.
 * The pair equals bmfr_process_frame bit for bit.  Untiled contexts: every
 * block is interior. */
bmfr_status bmfr_process_frame_interior(bmfr_ctx *ctx, void *stream, const bmfr_frame_inputs *in,
    const float prev_frame_camera_matrix[16], const float pixel_offset[2], int frame_number);
bmfr_status bmfr_process_frame_border(bmfr_ctx *ctx, void *stream, const bmfr_frame_inputs *in,
    const float prev_frame_camera_matrix[16], const float pixel_offset[2], int frame_number);

/* `count` consecutive frames first_frame .. first_frame+count-1 in one call
 * (the whole loop of bmfr.cpp:417-485 over frames already in device memory,
 * as tasks() holds the sequence in memory): in[i], the column-major
 * prev_frame_camera_matrices[16*i..] and pixel_offsets[2*i..] are frame
 * first_frame+i's arguments of bmfr_process_frame.  The frames are
 * pipelined: one launch per frame on `stream` runs K1 of frame f and, in its
 * tail, TAA of frame f-1 (half tmp_data, canonical feature lists), else TAA
 * of frame f (K2) runs on a context-owned stream beside K1 of frame f+1
 * (also with the environment variable BMFR_SEQUENCE=streams); all work is
 * joined back onto `stream`, so everything the call enqueues is complete
 * when `stream` reaches the point after it.  All
 * inputs must stay valid until then.  outputs (nullable; entries nullable):
 * outputs[i] receives frame i's output (W*H float3, device or page-locked
 * host memory).  Results equal bmfr_process_frame per frame bit for bit.
 * Untiled contexts only (tiles exchange a halo between frames). */
bmfr_status bmfr_process_sequence(bmfr_ctx *ctx, void *stream, int count, const bmfr_frame_inputs *in,
    const float *prev_frame_camera_matrices, const float *pixel_offsets, int first_frame,
    float *const *outputs);

/* Halo exchange support for tiled contexts: copy the rectangles rects[n][5]
 * = {x, y, width, height, planes} (image coordinates inside the context's
 * region; planes = a non-empty mask of BMFR_HALO_*) of the exchanged state
 * planes of bmfr_state(previous = 0) -- noisy_accumulated (12 B/px), spp
 * (1), filtered_accumulated (12), result (12) -- into (unpack = 0) or out of
 * (unpack = 1) `buffer` (device memory), rectangle after rectangle, plane
 * after plane in that order, rows packed, each segment padded to 16 bytes;
 * one kernel launch on `stream`.  *bytes (nullable) receives the packed
 * size; buffer = NULL only computes it.  At most 64 segments (rectangle x
 * plane). */
#define BMFR_HALO_NOISY 1
#define BMFR_HALO_SPP 2
#define BMFR_HALO_FILTERED 4
#define BMFR_HALO_RESULT 8
#define BMFR_HALO_STATE (BMFR_HALO_NOISY | BMFR_HALO_SPP | BMFR_HALO_FILTERED)
#define BMFR_HALO_ALL (BMFR_HALO_STATE | BMFR_HALO_RESULT)
bmfr_status bmfr_halo_copy(bmfr_ctx *ctx, void *stream, const int *rects, int n, void *buffer, int unpack,
    size_t *bytes);

/* What frame `frame_number` of a tiled configuration reads of the previous
 * frame's state ({x, y, width, height}, inside the region; host only, no
 * context): state_rect for noisy_accumulated / spp / filtered_accumulated --
 * the pixels of the frame's K1 blocks (its shifted block grid, bmfr.cl:
 * 267-285; mirrored at the frame border) grown by tile_halo - 33 --, and
 * result_rect for the TAA output -- the tile grown by tile_halo - 33.
 * Before frame_number the caller must refresh the parts of these
 * rectangles outside the tile (refreshing the whole halo ring is also
 * correct); the kernels check the reprojection taps against them.  Both
 * depend on frame_number % 16 only. */
bmfr_status bmfr_halo_need(const bmfr_config *cfg, int frame_number, int state_rect[4], int result_rect[4]);

/* ---- Multi-GPU halo exchange (SURVEY.md 5 "Distributed communication
 * backend", 8e; no reference counterpart: the reference drives one GPU,
 * bmfr.cpp:183-191) ----
 * A tile grid is ntiles rectangles tiles[4 r .. 4 r + 3] = {x, y, width,
 * height} partitioning the frame; rank r runs a tiled context whose
 * bmfr_config has tile_* = tile r (same tile_halo for every rank).
 *
 * bmfr_halo_plan: what rank `rank` exchanges before frame_number (host only):
 * for each of the *n_peers neighbours, peers[k], then send_counts[k]
 * bmfr_halo_copy records of its own tile that the neighbour's frame reads,
 * then recv_counts[k] records of the neighbour's tile its own frame reads,
 * all in `records` (5 ints each, at most max_records).  peers = records =
 * NULL only counts.  Depends on frame_number % 16.  (bmfr_amd/tiling.py
 * TileGrid.frame_plan is the same plan.) */
bmfr_status bmfr_halo_plan(const bmfr_config *cfg, const int *tiles, int ntiles, int rank, int frame_number,
    int *peers, int *send_counts, int *recv_counts, int *records, int max_records, int *n_peers);

/* RCCL communicator of one rank (RCCL is loaded at run time; without it the
 * calls return BMFR_ERROR_UNSUPPORTED).  One process per GPU: rank 0 makes
 * the id (bmfr_comm_unique_id), every rank receives it out of band (e.g.
 * torch.distributed / MPI broadcast) and calls bmfr_comm_create.  One
 * process driving several GPUs: bmfr_comm_create_all (out[i] = rank i, on
 * devices[i]). */
typedef struct bmfr_comm bmfr_comm;
bmfr_status bmfr_comm_unique_id(unsigned char id[128]);
bmfr_status bmfr_comm_create(const unsigned char id[128], int nranks, int rank, int hip_device, bmfr_comm **out);
bmfr_status bmfr_comm_create_all(int ndev, const int *devices, bmfr_comm **out);
bmfr_status bmfr_comm_destroy(bmfr_comm *comm);

/* The per-frame exchange of one rank: the plans of all 16 block-grid shifts
 * and device send / receive buffers are made once here (cfg = the rank's
 * context configuration; comm = its communicator, or NULL for an in-process
 * grid).  bmfr_exchange_run, before frame_number > 0 of the context (after the
 * previous frame, before bmfr_process_frame_border -- or before
 * bmfr_process_frame), enqueues on `stream`: one pack kernel
 * (bmfr_halo_copy), one ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd
 * batch to the neighbours, one unpack kernel.  bmfr_exchange_run_all: every
 * rank of a grid held by this process -- with communicators
 * (bmfr_comm_create_all) all messages in one group, streams[i] rank i's
 * stream; without, every context on one device and everything on
 * streams[0] as device copies (single-GPU runs of a tiled grid). */
typedef struct bmfr_exchange bmfr_exchange;
bmfr_status bmfr_exchange_create(bmfr_ctx *ctx, const bmfr_config *cfg, const int *tiles, int ntiles, int rank,
    bmfr_comm *comm, bmfr_exchange **out);
bmfr_status bmfr_exchange_run(bmfr_exchange *x, void *stream, int frame_number);
bmfr_status bmfr_exchange_run_all(bmfr_exchange *const *xs, int n, void *const *streams, int frame_number);
/* Bytes rank x sends / receives before frame_number. */
bmfr_status bmfr_exchange_bytes(const bmfr_exchange *x, int frame_number, size_t *sent, size_t *received);
bmfr_status bmfr_exchange_destroy(bmfr_exchange *x);

/* Tiled contexts: waits for the last enqueued frame and returns
 * BMFR_ERROR_HALO_EXCEEDED if any frame since frame 0 read reprojection taps
 * past its valid state (see tile_halo), BMFR_OK otherwise; *overshoot
 * (nullable) receives the largest distance in pixels.  Untiled: BMFR_OK.
 * BMFR_ERROR_SYNC_TIMEOUT takes precedence (see bmfr_frame_status). */
bmfr_status bmfr_halo_status(bmfr_ctx *ctx, unsigned *overshoot);

/* Waits for the last enqueued frame and returns the context's sticky report:
 * BMFR_ERROR_SYNC_TIMEOUT if, in any frame since frame 0, a bounded wait of
 * the fused kernels gave up -- a K1 wave waiting for the pivot column another
 * wave of its work-group publishes in LDS, or (one-launch frame) a TAA tile
 * waiting for the completion flags of the K1 blocks under it; the kernels run
 * to their end regardless (no wave waits forever), so that frame's output and
 * state are not valid --, else BMFR_ERROR_HALO_EXCEEDED as bmfr_halo_status,
 * else BMFR_OK.  Every bmfr_process_frame* / bmfr_process_sequence call
 * returns the same report, without waiting, once the host has seen it, until
 * frame_number 0 starts a new sequence (frame 0 first waits for every frame
 * enqueued before it, then clears the reports).  The wait is an event the
 * library records at that point on the stream of the last enqueued frame
 * (none between frames: a marker between two frames' kernels costs GPU time),
 * so it also waits for work the caller queued on that stream after the frame;
 * if that stream no longer exists it waits for the whole device. */
bmfr_status bmfr_frame_status(bmfr_ctx *ctx);

/* Device pointer to the last processed frame's output (TAA result, float3,
 * W*H, the buffer the reference reads back at bmfr.cpp:479-480).  Valid until
 * the next bmfr_process_frame. */
const float *bmfr_output(const bmfr_ctx *ctx);

/* Device pointers to the context's temporal state of the last frame, for
 * inspection / multi-GPU halo exchange: accumulated noisy colour (float3),
 * spp (u8), accumulated filtered colour (float3), prev-frame pixel (float2).
 * tone_mapped is only materialised by the generic-feature fallback (the
 * canonical path tone-maps inside the TAA kernel) and accept bits never are
 * (NULL). */
typedef struct bmfr_state_view {
    float *noisy_accumulated;
    uint8_t *spp;
    float *filtered_accumulated;
    float *tone_mapped;
    float *prev_frame_pixel;
    uint8_t *accept;
    float *result;
} bmfr_state_view;
bmfr_status bmfr_state(const bmfr_ctx *ctx, int previous, bmfr_state_view *out);

/* ---- Profiling: the CL_QUEUE_PROFILING_ENABLE + GPUTimer analogue ----
 * (bmfr.cpp:191, 386-412, 488-517).  When enabled, bmfr_process_frame records
 * HIP events around its two kernels; bmfr_get_profile synchronises on them and
 * returns per-frame device durations in ms, oldest first (at most `capacity`
 * frames are kept; enabling again clears the record). */
typedef struct bmfr_frame_profile {
    int frame_number;
    float fused_block_ms; /* K1: accumulate_noisy .. accumulate_filtered, fused */
    float taa_ms;         /* K2: taa */
    float total_ms;       /* start of K1 -> end of K2 (bmfr.cpp:497-502) */
} bmfr_frame_profile;
bmfr_status bmfr_set_profiling(bmfr_ctx *ctx, int enable, int capacity);
/* Record only frames whose frame_number is a multiple of `stride` (default
 * 1): per-kernel timings sampled inside a long timed run at a small cost. */
bmfr_status bmfr_set_profiling_stride(bmfr_ctx *ctx, int stride);
bmfr_status bmfr_get_profile(bmfr_ctx *ctx, bmfr_frame_profile *out, int max_frames, int *count);

/* ---- Synthetic scene (stands in for the external EXR dataset) ---- */

/* Camera of frame `frame`: column-major view-projection matrix and the
 * pixel offset (jitter) in [0,1)^2, i.e. camera_matrices[frame] and
 * pixel_offsets[frame] of the dataset's camera_matrices.h (bmfr.cpp:44-53). */
void bmfr_synth_camera(int image_width, int image_height, int frame, float vp[16],
    float pixel_offset[2]);

/* Render frame `frame` of the synthetic sequence into float3 planes.  `clean`
 * (nullable) receives the noise-free tone-mapped reference image used for
 * PSNR.  _host runs on the CPU (host pointers), _device on the GPU. */
bmfr_status bmfr_synth_frame_host(int image_width, int image_height, int frame, uint32_t seed,
    float *noisy, float *normals, float *positions, float *albedo, float *clean);
bmfr_status bmfr_synth_frame_device(int image_width, int image_height, int frame, uint32_t seed,
    float *noisy, float *normals, float *positions, float *albedo, float *clean, void *stream);
/* The region [x0, x0+w) x [y0, y0+h) of the same frame into planes of row
 * stride w (a tiled context's inputs). */
bmfr_status bmfr_synth_region_device(int image_width, int image_height, int x0, int y0, int w, int h,
    int frame, uint32_t seed, float *noisy, float *normals, float *positions, float *albedo, float *clean,
    void *stream);

#ifdef __cplusplus
}
#endif
#endif /* BMFR_H */
