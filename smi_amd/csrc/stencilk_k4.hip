// stencilk_k4.hip -- sweepk_kernel<4> (stencilk.h) and bandk_kernel<4> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_SWEEPK_INSTANCE(4)
SMI_BANDK_INSTANCE(4)
