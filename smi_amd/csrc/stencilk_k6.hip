// stencilk_k6.hip -- sweepk_kernel<6> (stencilk.h) and bandk_kernel<6> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_SWEEPK_INSTANCE(6)
SMI_BANDK_INSTANCE(6)
