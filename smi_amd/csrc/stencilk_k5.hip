// stencilk_k5.hip -- sweepk_kernel<5> (stencilk.h)
#include "stencilk.h"
SMI_SWEEPK_INSTANCE(5)
