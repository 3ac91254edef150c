// stencild_k19.hip -- sweepd_kernel<19> (stencild.h)
#include "stencild.h"
SMI_SWEEPD_INSTANCE(19)
