// bandk_k11.hip -- bandk_kernel<11> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(11)
