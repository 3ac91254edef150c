// bandk_k9.hip -- bandk_kernel<9> (stencil_bandk.h)
#include "stencil_bandk.h"
SMI_BANDK_INSTANCE(9)
