// stencild_k14.hip -- sweepd_kernel<14> (stencild.h)
#include "stencild.h"
SMI_SWEEPD_INSTANCE(14)
