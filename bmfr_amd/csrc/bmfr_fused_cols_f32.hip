// bmfr_fused_cols_f32.hip -- the column-split K1 for f32 tmp_data
// (USE_HALF_PRECISION_IN_TMP_DATA 0), compiled apart from the half kernels.
#define BMFR_COLS_F32 1
#include "bmfr_fused_cols.hip"
