// The small-s kernel compiled with -fno-slp-vectorize (build.py) for
// same-process A/B against the default build (HOP_SMALL_VARIANT=1).
#define HOP_SMALL_NS small_noslp
#define HOP_SMALL_DISPATCH dispatch_lft_small_noslp
#include "lft_small.hip"
