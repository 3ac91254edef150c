// stencilk_k4.hip -- sweepk_kernel<4> (stencilk.h)
#include "stencilk.h"
SMI_SWEEPK_INSTANCE(4)
