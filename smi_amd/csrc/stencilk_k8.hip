// stencilk_k8.hip -- sweepk_kernel<8> (stencilk.h)
#include "stencilk.h"
SMI_SWEEPK_INSTANCE(8)
