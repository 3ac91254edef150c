// stencild_k16.hip -- sweepd_kernel<16> (stencild.h) and bandk_kernel<16> (stencil_bandk.h)
#include "stencil_bandk.h"
#include "stencild.h"
SMI_SWEEPD_INSTANCE(16)
SMI_BANDK_INSTANCE(16)
