// bandk_k10.hip -- bandk_kernel<10> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(10)
