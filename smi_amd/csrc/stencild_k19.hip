// stencild_k19.hip -- sweepd_kernel<19> (stencild.h) and bandk_kernel<19> (stencil_bandk.h)
#include "stencil_bandk.h"
#include "stencild.h"
SMI_SWEEPD_INSTANCE(19)
SMI_BANDK_INSTANCE(19)
