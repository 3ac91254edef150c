// stencilk_k6.hip -- sweepk_kernel<6> (stencilk.h)
#include "stencilk.h"
SMI_SWEEPK_INSTANCE(6)
