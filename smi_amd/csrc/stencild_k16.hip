// stencild_k16.hip -- sweepd_kernel<16> (stencild.h)
#include "stencild.h"
SMI_SWEEPD_INSTANCE(16)
