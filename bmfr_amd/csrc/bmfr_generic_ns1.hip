// bmfr_generic_ns1.hip -- feature-count kernels for FEATURES_NOT_SCALED = 1 (bmfr_generic.h).
#define BMFR_GENERIC_NS 1
#include "bmfr_generic.h"
