// bmfr_generic_ns3.hip -- feature-count kernels for FEATURES_NOT_SCALED = 3 (bmfr_generic.h).
#define BMFR_GENERIC_NS 3
#include "bmfr_generic.h"
