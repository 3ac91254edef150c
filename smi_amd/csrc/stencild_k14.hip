// stencild_k14.hip -- sweepd_kernel<14> (stencild.h) and bandk_kernel<14> (stencil_bandk.h)
#include "stencil_bandk.h"
#include "stencild.h"
SMI_SWEEPD_INSTANCE(14)
SMI_BANDK_INSTANCE(14)
