// bandk_k15.hip -- bandk_kernel<15> and the lean bandl_kernel<15> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(15)
SMI_BANDL_INSTANCE(15)
