/* bmfr_debug.h -- diagnostics of libbmfr (not part of the drop-in boundary).
 *
 * bmfr_debug_stamps: per-block phase timestamps (s_memtime, shader clock) of
 * the last fused frame, 8 per block: start, after accumulate_noisy, after
 * scaling, after QR, after back substitution, end.  Only the diagnostic
 * build (libbmfr_diag.so, -DBMFR_STAMPS) with BMFR_STAMPS set in the
 * environment at bmfr_create records them; otherwise BMFR_ERROR_UNSUPPORTED.
 * bmfr_debug_sync: see below.
 */
#ifndef BMFR_DEBUG_H
#define BMFR_DEBUG_H
#include "bmfr.h"
#ifdef __cplusplus
extern "C" {
#endif
bmfr_status bmfr_debug_stamps(const bmfr_ctx *ctx, unsigned long long *host, size_t count);
/* bmfr_debug_sync: the fused kernels' bounded waits for the frames enqueued
 * from now on.  max_polls = how many sleeps a K1 pivot wait polls before it
 * gives up (a TAA tile's completion-flag wait: 4x that); < 0 restores the
 * default (2^20); 0 gives up at the first unready flag, which forces the
 * BMFR_ERROR_SYNC_TIMEOUT path.  k1_delay > 0: in the one-launch frame, one
 * K1 block in 61 sleeps k1_delay x ~8K shader cycles before it publishes its
 * completion flag, so the TAA tiles really wait (results must not change). */
bmfr_status bmfr_debug_sync(bmfr_ctx *ctx, int max_polls, int k1_delay);
/* bmfr_debug_frame_launches: kernel launches of the untiled bmfr_process_frame
 * from now on -- 0: by the frame's size (bmfr_sizes.frame_launches, the
 * default), 1: one launch (K1 blocks, then the TAA tiles on completion
 * flags) at any size, 2: K1, then K2.  Results are the same bit for bit;
 * the tests use it to run the one-launch kernel at 4K. */
bmfr_status bmfr_debug_frame_launches(bmfr_ctx *ctx, int launches);
#ifdef __cplusplus
}
#endif
#endif
