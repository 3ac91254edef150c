// bandk_k19.hip -- bandk_kernel<19> and the lean bandl_kernel<19> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(19)
SMI_BANDL_INSTANCE(19)
