// bandk_k13.hip -- bandk_kernel<13> and the lean bandl_kernel<13> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(13)
SMI_BANDL_INSTANCE(13)
