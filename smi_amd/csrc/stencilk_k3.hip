// stencilk_k3.hip -- sweepk_kernel<3> (stencilk.h) and bandk_kernel<3> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_SWEEPK_INSTANCE(3)
SMI_BANDK_INSTANCE(3)
