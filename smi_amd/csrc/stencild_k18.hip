// stencild_k18.hip -- sweepd_kernel<18> (stencild.h)
#include "stencild.h"
SMI_SWEEPD_INSTANCE(18)
