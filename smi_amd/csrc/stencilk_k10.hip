// stencilk_k10.hip -- sweepk_kernel<10> (stencilk.h)
#include "stencilk.h"
SMI_SWEEPK_INSTANCE(10)
