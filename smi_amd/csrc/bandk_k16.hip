// bandk_k16.hip -- bandk_kernel<16> and the lean bandl_kernel<16> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(16)
SMI_BANDL_INSTANCE(16)
