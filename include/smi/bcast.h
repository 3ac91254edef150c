/*
 * bcast.h -- SMI_Bcast on whole buffers.
 *
 * Replaces SMI_Open_bcast_channel / SMI_Bcast (include/smi/bcast.h:43-63) and
 * the support kernel smi_kernel_bcast_<port> (codegen/templates/bcast.cl:
 * 3-149), a linear fan-out of 7-element packets from the root.  Contract:
 * bitwise copy of the root's buffer into every rank's buffer.
 */
#ifndef SMI_BCAST_H
#define SMI_BCAST_H

#include <stddef.h>
#include "communicator.h"
#include "data_types.h"
#include "channel_descriptor.h"

#ifdef __cplusplus
extern "C" {
#endif

/* `buf`: device buffer of `count` elements; read on root, overwritten on the
 * other ranks.  Enqueued on `stream`. */
int smi_bcast(SMI_Comm comm, void *buf, size_t count, SMI_Datatype type,
              int root, int port, SMI_Stream stream);

/* Element API, same names and argument meaning as the reference
 * (include/smi/bcast.h:43-63): every rank calls SMI_Bcast `count` times; on
 * the root `data` is the element sent, elsewhere it receives the element. */
SMI_BChannel SMI_Open_bcast_channel(int count, SMI_Datatype data_type, int port, int root, SMI_Comm comm);
SMI_BChannel SMI_Open_bcast_channel_ad(int count, SMI_Datatype data_type, int port, int root,
                                       SMI_Comm comm, int asynch_degree);
void SMI_Bcast(SMI_BChannel *chan, void *data);

/* Size in bytes of one element of `type` (0 for an unknown type). */
size_t smi_type_size(SMI_Datatype type);

#ifdef __cplusplus
}
#endif
#endif /* SMI_BCAST_H */
