// bandk_k7.hip -- bandk_kernel<7> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(7)
