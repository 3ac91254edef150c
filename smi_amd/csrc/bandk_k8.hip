// bandk_k8.hip -- bandk_kernel<8> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(8)
