/*
 * channel_descriptor.h -- transient channel descriptors of the element API.
 *
 * Replaces the reference descriptors, which carried a 32-byte network
 * packet inline and were specialised per port by the code generator:
 *   SMI_Channel         include/smi/channel_descriptor.h:17-31
 *   SMI_BChannel        include/smi/bcast.h:17-32
 *   SMI_RChannel        include/smi/reduce.h:27-42
 *   SMI_ScatterChannel  include/smi/scatter.h:20-37
 *   SMI_GatherChannel   include/smi/gather.h:18-35
 * Here a descriptor is a small value type (returned by value, caller-owned,
 * like the reference's) whose `handle` names the runtime's staging state.
 * A channel is transient: it ends by itself after its element count, as in
 * the reference (stencil_smi.cl:241-248 re-opens one per message).
 * `status` holds the SMI_Status of the last call on the channel (the
 * reference primitives are void and cannot report errors).
 */
#ifndef SMI_CHANNEL_DESCRIPTOR_H
#define SMI_CHANNEL_DESCRIPTOR_H

#include "communicator.h"
#include "data_types.h"

#define SMI_CHANNEL_FIELDS                                                   \
    int handle;             /* runtime state, 0 once the channel ended     */ \
    int status;             /* SMI_Status of the last operation            */ \
    int my_rank;                                                             \
    int num_ranks;                                                           \
    int peer;               /* destination / source / root                 */ \
    int port;                                                                \
    SMI_Datatype data_type;                                                  \
    unsigned int message_size;        /* elements in this transient channel */ \
    unsigned int processed_elements;  /* elements pushed/popped so far      */

typedef struct { SMI_CHANNEL_FIELDS } SMI_Channel;
typedef struct { SMI_CHANNEL_FIELDS } SMI_BChannel;
typedef struct { SMI_CHANNEL_FIELDS int reduce_op; } SMI_RChannel;
typedef struct { SMI_CHANNEL_FIELDS unsigned int recv_count; } SMI_ScatterChannel;
typedef struct { SMI_CHANNEL_FIELDS unsigned int recv_count; } SMI_GatherChannel;

#endif /* SMI_CHANNEL_DESCRIPTOR_H */
