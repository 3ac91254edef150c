/*
 * smi.h -- umbrella header of the MI355X-native SMI hot path.
 *
 * Drop-in for the reference umbrella include/smi.h:1-21 (ryutakashino/SMI).
 * The reference declares device-side OpenCL primitives that are specialised
 * per port by a code generator; this build exposes the same channel surface
 * as a host-callable C ABI (libsmi_amd.so) whose bulk entry points run
 * hand-written gfx950 HIP kernels and move data with RCCL over xGMI.
 * No HIP or torch type appears in any signature: device buffers are plain
 * pointers, streams are opaque `SMI_Stream` handles (a hipStream_t).
 */
#ifndef SMI_H
#define SMI_H

#include "smi/status.h"
#include "smi/data_types.h"
#include "smi/operation_type.h"
#include "smi/communicator.h"
#include "smi/channel_descriptor.h"
#include "smi/push.h"
#include "smi/pop.h"
#include "smi/stencil.h"
#include "smi/reduce.h"
#include "smi/bcast.h"
#include "smi/scatter.h"
#include "smi/gather.h"
#include "smi/gesummv.h"
#include "smi/kmeans.h"
#include "smi/profiling.h"

#endif /* SMI_H */
