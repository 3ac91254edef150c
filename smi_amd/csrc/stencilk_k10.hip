// stencilk_k10.hip -- sweepk_kernel<10> (stencilk.h) and bandk_kernel<10> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_SWEEPK_INSTANCE(10)
SMI_BANDK_INSTANCE(10)
