// stencilk_k7.hip -- sweepk_kernel<7> (stencilk.h)
#include "stencilk.h"
SMI_SWEEPK_INSTANCE(7)
