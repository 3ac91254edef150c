// stencild_k20.hip -- sweepd_kernel<20> (stencild.h) and bandk_kernel<20> (stencil_bandk.h)
#include "stencil_bandk.h"
#include "stencild.h"
SMI_SWEEPD_INSTANCE(20)
SMI_BANDK_INSTANCE(20)
