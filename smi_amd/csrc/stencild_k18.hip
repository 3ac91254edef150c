// stencild_k18.hip -- sweepd_kernel<18> (stencild.h) and bandk_kernel<18> (stencil_bandk.h)
#include "stencil_bandk.h"
#include "stencild.h"
SMI_SWEEPD_INSTANCE(18)
SMI_BANDK_INSTANCE(18)
