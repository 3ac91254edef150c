// stencilk_k12.hip -- sweepk_kernel<12> (stencilk.h)
#include "stencilk.h"
SMI_SWEEPK_INSTANCE(12)
