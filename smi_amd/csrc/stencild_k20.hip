// stencild_k20.hip -- sweepd_kernel<20> (stencild.h)
#include "stencild.h"
SMI_SWEEPD_INSTANCE(20)
