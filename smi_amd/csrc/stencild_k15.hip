// stencild_k15.hip -- sweepd_kernel<15> (stencild.h)
#include "stencild.h"
SMI_SWEEPD_INSTANCE(15)
