// stencilk_k9.hip -- sweepk_kernel<9> (stencilk.h)
#include "stencilk.h"
SMI_SWEEPK_INSTANCE(9)
