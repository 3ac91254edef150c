/*
 * communicator.h -- communicator and runtime bring-up.
 *
 * Replaces:
 *   - SMI_Comm = char2{rank, size} and SMI_Comm_rank/SMI_Comm_size
 *     (include/smi/communicator.h:12-31);
 *   - the generated host initialiser SMI_Comm SmiInit_<program>(rank,
 *     ranks_count, routing_dir, context, program, buffers)
 *     (codegen/templates/host_hlslib.cl:8-90), which loaded routing tables
 *     and launched the never-terminating CK_S/CK_R/support kernels.
 * On one 8xMI355X node there is nothing to route: rank r drives GPU r and
 * every pair of GPUs is one xGMI hop, so initialisation is just an RCCL
 * communicator (or, for single-GPU testing, an in-process group whose ranks
 * are host threads sharing one device).
 *
 * Ordering and threads.  A communicator carries two independent matching
 * spaces:
 *   - bulk operations (smi_reduce, smi_bcast, smi_scatter, smi_gather,
 *     smi_send/smi_recv, smi_gesummv, the stencil exchanges) are matched with
 *     the other ranks' in issue order per rank pair, as RCCL matches them:
 *     every rank issues its bulk operations in the same order, from one host
 *     thread at a time (concurrent callers are serialised per transport
 *     group, but a second thread's operation would still interleave in the
 *     issue order and share the communicator's staging workspace).  The
 *     `port` argument of a bulk call is informational: bulk operations that
 *     must run concurrently from different threads (the reference's
 *     collectives on different ports) each take a communicator of their own
 *     from smi_comm_dup.
 *   - element-granular channels (SMI_Push/SMI_Pop, SMI_Bcast, SMI_Reduce,
 *     SMI_Scatter, SMI_Gather) travel on a communicator of their own (an
 *     RCCL communicator split off at smi_init, pre-connected to every peer),
 *     tagged by port and demultiplexed into one FIFO per (source, port), like
 *     the reference's per-port channels: a packet pushed before a collective
 *     is never consumed by it, and channels on different ports may be driven
 *     from different host threads.
 */
#ifndef SMI_COMMUNICATOR_H
#define SMI_COMMUNICATOR_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Opaque stream handle (a hipStream_t; NULL = the device's null stream). */
typedef void *SMI_Stream;

/* Communicator, passed by value like the reference's char2.  `handle`
 * indexes the runtime's table of live communicators. */
typedef struct {
    int rank;
    int size;
    int handle;
} SMI_Comm;

static inline int SMI_Comm_rank(SMI_Comm comm) { return comm.rank; }
static inline int SMI_Comm_size(SMI_Comm comm) { return comm.size; }

#define SMI_UNIQUE_ID_BYTES 128

/* Fill `id` (SMI_UNIQUE_ID_BYTES bytes) with a fresh RCCL unique id; call on
 * rank 0 and distribute the bytes to every rank (the Python host uses the
 * torch.distributed store). */
int smi_get_unique_id(void *id, int id_bytes);

/* One process per GPU: RCCL communicator over xGMI.  Selects `device` for
 * the calling thread.  Collective: every rank must call it. */
int smi_init(int rank, int size, int device, const void *unique_id, int id_bytes,
             SMI_Comm *comm);

/* In-process group: `size` ranks are host threads of this process, all on
 * one device (the first rank's `device`; smi_init_local returns
 * SMI_ERR_INVALID_ARG for any other).  smi_local_group_create returns a
 * group id; each rank thread then calls smi_init_local with it.  Transfers
 * are device-side copies ordered by HIP events -- a GPU transport used to run
 * multi-rank parity tests on a single GPU. */
int smi_local_group_create(int size, int *group_id);
int smi_init_local(int group_id, int rank, int device, SMI_Comm *comm);

/* A new communicator over the same ranks, with its own matching spaces,
 * comm stream and staging (MPI_Comm_dup; an RCCL communicator split off
 * this one, or a new in-process group).  Collective: every rank calls it,
 * in the same order relative to its other dups.  Bulk operations on
 * different communicators are matched independently, so a communicator per
 * port lets host threads drive bulk collectives on different ports at the
 * same time -- what the reference's distinct ports give its concurrent
 * collectives (microbenchmarks/kernels/multi_collectives.cl:50-76).
 * Finalize every dup like any communicator. */
int smi_comm_dup(SMI_Comm comm, SMI_Comm *out);

int smi_finalize(SMI_Comm comm);

/* Devices visible to this process. */
int smi_device_count(int *count);

/* Block until all work queued on `stream` has finished. */
int smi_stream_synchronize(SMI_Stream stream);

#ifdef __cplusplus
}
#endif
#endif /* SMI_COMMUNICATOR_H */
