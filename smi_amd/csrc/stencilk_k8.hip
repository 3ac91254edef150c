// stencilk_k8.hip -- sweepk_kernel<8> (stencilk.h) and bandk_kernel<8> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_SWEEPK_INSTANCE(8)
SMI_BANDK_INSTANCE(8)
