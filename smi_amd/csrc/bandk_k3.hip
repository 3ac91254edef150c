// bandk_k3.hip -- bandk_kernel<3> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(3)
