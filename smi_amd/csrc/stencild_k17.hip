// stencild_k17.hip -- sweepd_kernel<17> (stencild.h)
#include "stencild.h"
SMI_SWEEPD_INSTANCE(17)
