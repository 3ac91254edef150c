/*
 * gather.h -- SMI_Gather (element API) and smi_gather (whole buffers).
 *
 * Element API: same names and argument meaning as the reference
 * include/smi/gather.h:47-68 (implementation codegen/templates/gather.cl:
 * 3-162): every rank calls SMI_Gather send_count times with its element in
 * send_data; the root calls it recv_count*num_ranks times and receives rank
 * 0's elements, then rank 1's, ... in rcv_data (its own segment is copied
 * from send_data).
 */
#ifndef SMI_GATHER_H
#define SMI_GATHER_H

#include <stddef.h>
#include "channel_descriptor.h"

#ifdef __cplusplus
extern "C" {
#endif

SMI_GatherChannel SMI_Open_gather_channel(int send_count, int recv_count, SMI_Datatype data_type,
                                          int port, int root, SMI_Comm comm);
SMI_GatherChannel SMI_Open_gather_channel_ad(int send_count, int recv_count, SMI_Datatype data_type,
                                             int port, int root, SMI_Comm comm, int asynch_degree);
void SMI_Gather(SMI_GatherChannel *chan, void *send_data, void *rcv_data);

/* Device buffers: every rank's sendbuf holds count elements; the root's
 * recvbuf receives size*count elements in rank order.  Enqueued on `stream`. */
int smi_gather(SMI_Comm comm, const void *sendbuf, void *recvbuf, size_t count, SMI_Datatype type,
               int root, int port, SMI_Stream stream);

#ifdef __cplusplus
}
#endif
#endif /* SMI_GATHER_H */
