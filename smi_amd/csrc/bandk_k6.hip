// bandk_k6.hip -- bandk_kernel<6> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(6)
