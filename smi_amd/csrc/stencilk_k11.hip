// stencilk_k11.hip -- sweepk_kernel<11> (stencilk.h) and bandk_kernel<11> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_SWEEPK_INSTANCE(11)
SMI_BANDK_INSTANCE(11)
