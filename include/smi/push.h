/*
 * push.h -- send side of a point-to-point transient channel (host-callable).
 *
 * Same names and argument meaning as the reference include/smi/push.h:19-48
 * (implementation codegen/templates/push.cl:3-70): elements are packed into
 * packets (here 16,368-byte payloads instead of 28-byte ones) and a packet is
 * sent when it is full, when the message is complete, or on an immediate
 * flush.  Sends are buffered (32 packets per communicator in flight), the
 * counterpart of the reference's credit window, so a rank may push before its
 * peer pops.  `data` points to ONE element in host memory.
 */
#ifndef SMI_PUSH_H
#define SMI_PUSH_H

#include "channel_descriptor.h"

#ifdef __cplusplus
extern "C" {
#endif

SMI_Channel SMI_Open_send_channel(int count, SMI_Datatype data_type, int destination, int port,
                                  SMI_Comm comm);
/* asynch_degree (elements; the reference's channel FIFO depth,
 * codegen/rewrite.py:26-35): at most this many elements are packed before a
 * message leaves (capped at one 16,368-byte payload); <= 0 = the default. */
SMI_Channel SMI_Open_send_channel_ad(int count, SMI_Datatype data_type, int destination, int port,
                                     SMI_Comm comm, int asynch_degree);
void SMI_Push_flush(SMI_Channel *chan, void *data, int immediate);
void SMI_Push(SMI_Channel *chan, void *data);

/* Bulk, device-buffer form of a send channel: `count` elements of `buf`
 * (device memory) to `destination`, enqueued on `stream`.  Replaces a
 * SMI_Open_send_channel + count x SMI_Push loop (bandwidth_0.cl:13-35).
 * Pairs with smi_recv on the destination; messages between two ranks are
 * matched in issue order (the port is informational). */
int smi_send(SMI_Comm comm, const void *buf, size_t count, SMI_Datatype data_type, int destination,
             int port, SMI_Stream stream);

#ifdef __cplusplus
}
#endif
#endif /* SMI_PUSH_H */
