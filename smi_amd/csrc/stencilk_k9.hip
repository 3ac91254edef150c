// stencilk_k9.hip -- sweepk_kernel<9> (stencilk.h) and bandk_kernel<9> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_SWEEPK_INSTANCE(9)
SMI_BANDK_INSTANCE(9)
