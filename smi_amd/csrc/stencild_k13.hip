// stencild_k13.hip -- sweepd_kernel<13> (stencild.h)
#include "stencild.h"
SMI_SWEEPD_INSTANCE(13)
