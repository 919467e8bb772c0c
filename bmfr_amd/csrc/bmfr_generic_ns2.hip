// bmfr_generic_ns2.hip -- feature-count kernels for FEATURES_NOT_SCALED = 2 (bmfr_generic.h).
#define BMFR_GENERIC_NS 2
#include "bmfr_generic.h"
