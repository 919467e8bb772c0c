// bmfr_generic_ns4.hip -- feature-count kernels for FEATURES_NOT_SCALED = 4 (bmfr_generic.h).
#define BMFR_GENERIC_NS 4
#include "bmfr_generic.h"
