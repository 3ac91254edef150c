// stencilk_k7.hip -- sweepk_kernel<7> (stencilk.h) and bandk_kernel<7> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_SWEEPK_INSTANCE(7)
SMI_BANDK_INSTANCE(7)
