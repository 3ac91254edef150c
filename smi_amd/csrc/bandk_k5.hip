// bandk_k5.hip -- bandk_kernel<5> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(5)
