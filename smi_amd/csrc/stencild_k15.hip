// stencild_k15.hip -- sweepd_kernel<15> (stencild.h) and bandk_kernel<15> (stencil_bandk.h)
#include "stencil_bandk.h"
#include "stencild.h"
SMI_SWEEPD_INSTANCE(15)
SMI_BANDK_INSTANCE(15)
