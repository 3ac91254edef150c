// bandk_k12.hip -- bandk_kernel<12> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(12)
