/* bmfr_debug.h -- diagnostics of libbmfr (not part of the drop-in boundary).
 *
 * bmfr_debug_stamps: per-block phase timestamps (s_memtime, shader clock) of
 * the last fused frame, 8 per block: start, after accumulate_noisy, after
 * scaling, after QR, after back substitution, end.  Only the diagnostic
 * build (libbmfr_diag.so, -DBMFR_STAMPS) with BMFR_STAMPS set in the
 * environment at bmfr_create records them; otherwise BMFR_ERROR_UNSUPPORTED.
 */
#ifndef BMFR_DEBUG_H
#define BMFR_DEBUG_H
#include "bmfr.h"
#ifdef __cplusplus
extern "C" {
#endif
bmfr_status bmfr_debug_stamps(const bmfr_ctx *ctx, unsigned long long *host, size_t count);
#ifdef __cplusplus
}
#endif
#endif
