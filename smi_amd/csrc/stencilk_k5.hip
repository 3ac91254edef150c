// stencilk_k5.hip -- sweepk_kernel<5> (stencilk.h) and bandk_kernel<5> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_SWEEPK_INSTANCE(5)
SMI_BANDK_INSTANCE(5)
