/*
 * pop.h -- receive side of a point-to-point transient channel (host-callable).
 *
 * Same names and argument meaning as the reference include/smi/pop.h:20-39
 * (implementation codegen/templates/pop.cl:3-83).  Messages are FIFO per
 * (source, destination, port); SMI_Pop blocks until the next element of
 * this channel has arrived and writes it to `data` (host memory).
 */
#ifndef SMI_POP_H
#define SMI_POP_H

#include "channel_descriptor.h"

#ifdef __cplusplus
extern "C" {
#endif

SMI_Channel SMI_Open_receive_channel(int count, SMI_Datatype data_type, int source, int port,
                                     SMI_Comm comm);
SMI_Channel SMI_Open_receive_channel_ad(int count, SMI_Datatype data_type, int source, int port,
                                        SMI_Comm comm, int asynch_degree);
void SMI_Pop(SMI_Channel *chan, void *data);

/* Bulk, device-buffer form of a receive channel: `count` elements from
 * `source` into `buf` (device memory), enqueued on `stream`.  Replaces a
 * SMI_Open_receive_channel + count x SMI_Pop loop (bandwidth_1.cl:12-44). */
int smi_recv(SMI_Comm comm, void *buf, size_t count, SMI_Datatype data_type, int source, int port,
             SMI_Stream stream);

#ifdef __cplusplus
}
#endif
#endif /* SMI_POP_H */
