// stencilk_k11.hip -- sweepk_kernel<11> (stencilk.h)
#include "stencilk.h"
SMI_SWEEPK_INSTANCE(11)
