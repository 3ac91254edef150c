// stencild_k17.hip -- sweepd_kernel<17> (stencild.h) and bandk_kernel<17> (stencil_bandk.h)
#include "stencil_bandk.h"
#include "stencild.h"
SMI_SWEEPD_INSTANCE(17)
SMI_BANDK_INSTANCE(17)
