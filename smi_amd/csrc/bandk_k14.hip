// bandk_k14.hip -- bandk_kernel<14> and the lean bandl_kernel<14> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(14)
SMI_BANDL_INSTANCE(14)
