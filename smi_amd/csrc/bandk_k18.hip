// bandk_k18.hip -- bandk_kernel<18> and the lean bandl_kernel<18> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(18)
SMI_BANDL_INSTANCE(18)
