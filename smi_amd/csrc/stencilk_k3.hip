// stencilk_k3.hip -- sweepk_kernel<3> (stencilk.h)
#include "stencilk.h"
SMI_SWEEPK_INSTANCE(3)
