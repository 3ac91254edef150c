// bandk_k4.hip -- bandk_kernel<4> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(4)
