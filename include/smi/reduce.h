/*
 * reduce.h -- SMI_Reduce on whole buffers.
 *
 * Replaces SMI_Open_reduce_channel / SMI_Reduce (include/smi/reduce.h:55-76)
 * and the root-side support kernel smi_kernel_reduce_<port>
 * (codegen/templates/reduce.cl:3-245), which reduced one element per 32-byte
 * packet with a 16-deep credit window.
 *
 * Arithmetic contract: for every element the contributions are folded in
 * rank order through an S-slot rotating accumulator (S = 4 for float/double,
 * 1 for int/short/char, codegen/ops.py:110-116; init 0 / *_MIN / *_MAX,
 * codegen/ops.py:124-141):  q[S] = op(d_k, q[0]); shift; then
 * result = op(...op(init, q[0])..., q[S-1])  (reduce.cl:65-69,100-105,120-125).
 * Integer types wrap.  The result is defined on `root` only.
 */
#ifndef SMI_REDUCE_H
#define SMI_REDUCE_H

#include <stddef.h>
#include "communicator.h"
#include "data_types.h"
#include "channel_descriptor.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Same enumerators and values as include/smi/reduce.h:18-22. */
typedef enum {
    SMI_ADD = 0,
    SMI_MAX = 1,
    SMI_MIN = 2
} SMI_Op;

/* Reduce `count` elements of every rank's device buffer `sendbuf` into the
 * root's device buffer `recvbuf` (ignored on other ranks), enqueued on
 * `stream`.  `port` is informational: like every bulk operation of a
 * communicator (include/smi/communicator.h), a reduce is matched with the
 * other ranks' in issue order, so all ranks issue their bulk operations in
 * the same order (the reference orders them by port).
 * Schedule: owner-chunk exchange -> canonical rank-order fold on each owner
 * -> gather on the root, pipelined over pieces of smi_set_pipeline_bytes()
 * bytes per owner chunk (the fold of one piece overlaps the exchange of the
 * next).  Messages up to 256 KiB (latency-bound) take a direct fan-in
 * instead: every rank's buffer to the root in one transfer group and one
 * rank-order fold there.  Results depend on neither the path nor the piece
 * size: every element is folded over the ranks in rank order. */
int smi_reduce(SMI_Comm comm, const void *sendbuf, void *recvbuf, size_t count,
               SMI_Datatype type, SMI_Op op, int root, int port,
               SMI_Stream stream);

/* Element API, same names and argument meaning as the reference
 * (include/smi/reduce.h:55-76): every rank calls SMI_Reduce `count` times;
 * the root receives each element's reduction in data_rcv on return.  The
 * root folds the n contributions of the element with the same HIP fold
 * kernel as smi_reduce (one launch per element: a compatibility path, use
 * smi_reduce for throughput). */
SMI_RChannel SMI_Open_reduce_channel(int count, SMI_Datatype data_type, SMI_Op op, int port, int root,
                                     SMI_Comm comm);
SMI_RChannel SMI_Open_reduce_channel_ad(int count, SMI_Datatype data_type, SMI_Op op, int port, int root,
                                        SMI_Comm comm, int asynch_degree);
void SMI_Reduce(SMI_RChannel *chan, void *data_snd, void *data_rcv);

/* Piece size (bytes per owner chunk) of the pipelined smi_reduce/smi_bcast;
 * 0 = one piece per chunk.  Default 4 MiB.  Process-wide; set it between
 * operations, identically on every rank. */
int smi_set_pipeline_bytes(size_t piece_bytes);
int smi_get_pipeline_bytes(size_t *piece_bytes);

/* The local fold kernel: contribs holds `nranks` rows of `count` elements
 * (row r = rank r's contribution, row pitch `ld` elements); out[i] = fold of
 * column i in row order.  Used by smi_reduce on each chunk owner. */
int smi_reduce_fold(const void *contribs, void *out, int nranks, size_t count,
                    size_t ld, SMI_Datatype type, SMI_Op op, SMI_Stream stream);

#ifdef __cplusplus
}
#endif
#endif /* SMI_REDUCE_H */
