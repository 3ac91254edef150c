/*
 * scatter.h -- SMI_Scatter (element API) and smi_scatter (whole buffers).
 *
 * Element API: same names and argument meaning as the reference
 * include/smi/scatter.h:49-72 (implementation codegen/templates/scatter.cl:
 * 3-164): the root calls SMI_Scatter send_count*num_ranks times, its
 * elements going to rank 0, 1, ... in turn (during its own segment the
 * element is copied to data_rcv); every other rank calls it recv_count
 * times and receives in data_rcv.
 */
#ifndef SMI_SCATTER_H
#define SMI_SCATTER_H

#include <stddef.h>
#include "channel_descriptor.h"

#ifdef __cplusplus
extern "C" {
#endif

SMI_ScatterChannel SMI_Open_scatter_channel(int send_count, int recv_count, SMI_Datatype data_type,
                                            int port, int root, SMI_Comm comm);
SMI_ScatterChannel SMI_Open_scatter_channel_ad(int send_count, int recv_count, SMI_Datatype data_type,
                                               int port, int root, SMI_Comm comm, int asynch_degree);
void SMI_Scatter(SMI_ScatterChannel *chan, void *data_snd, void *data_rcv);

/* Device buffers: the root's sendbuf holds size*count elements, rank r gets
 * elements [r*count, (r+1)*count) in recvbuf.  Enqueued on `stream`. */
int smi_scatter(SMI_Comm comm, const void *sendbuf, void *recvbuf, size_t count, SMI_Datatype type,
                int root, int port, SMI_Stream stream);

#ifdef __cplusplus
}
#endif
#endif /* SMI_SCATTER_H */
