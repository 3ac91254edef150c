// stencilk_k12.hip -- sweepk_kernel<12> (stencilk.h) and bandk_kernel<12> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_SWEEPK_INSTANCE(12)
SMI_BANDK_INSTANCE(12)
