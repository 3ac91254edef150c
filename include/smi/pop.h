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

#ifdef __cplusplus
}
#endif
#endif /* SMI_POP_H */
