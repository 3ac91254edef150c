// stencild_k13.hip -- sweepd_kernel<13> (stencild.h) and bandk_kernel<13> (stencil_bandk.h)
#include "stencil_bandk.h"
#include "stencild.h"
SMI_SWEEPD_INSTANCE(13)
SMI_BANDK_INSTANCE(13)
