// bandk_k20.hip -- bandk_kernel<20> and the lean bandl_kernel<20> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(20)
SMI_BANDL_INSTANCE(20)
