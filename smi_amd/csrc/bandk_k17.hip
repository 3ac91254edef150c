// bandk_k17.hip -- bandk_kernel<17> and the lean bandl_kernel<17> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(17)
SMI_BANDL_INSTANCE(17)
