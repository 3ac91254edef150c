/*
 * kmeans.h -- the kmeans_smi consumer of SMI_Reduce / SMI_Bcast.
 *
 * Replaces the three kernels of examples/kernels/kmeans_smi.cl and the
 * device part of examples/host/kmeans_smi.cpp (ryutakashino/SMI):
 *   SendCentroids    kmeans_smi.cl:14-34    centroids of iteration i: the
 *                                            initial ones, then the updated ones
 *   ComputeDistance  kmeans_smi.cl:36-88    per point and cluster k a squared
 *                                            distance; the first k with the
 *                                            strictly smallest one wins
 *   ComputeMeans     kmeans_smi.cl:90-209   per-cluster sums and counts,
 *                                            SMI_Reduce to rank 0 (fp32 add on
 *                                            port 0, int add on port 2),
 *                                            SMI_Bcast (ports 1, 3), divide
 *
 * Arithmetic contract (the reference's semantics, quirks included):
 *   - distance: points are read as `width`-wide vectors (W, VTYPE in
 *     examples/include/kmeans.h.in; 16 in the reference build,
 *     examples/CMakeLists.txt:5) and the inner loop ASSIGNS the squared
 *     difference instead of adding it (kmeans_smi.cl:68-71), so only the
 *     last lane of every vector counts:
 *       dist_k = ((0 + d_{W-1}^2) + d_{2W-1}^2) + ...   (fp32, mul then add)
 *     width = 1 is the plain squared Euclidean distance.
 *   - assignment: min starts at +inf and cluster k replaces it only if
 *     dist_k < min (kmeans_smi.cl:75-83): ties keep the lower k, NaN never
 *     wins, a point whose distances are all NaN / +inf goes to cluster 0.
 *   - sums: per cluster and dimension, this rank's points in point order,
 *     fp32 adds from +0 (kmeans_smi.cl:113-127); counts exact.  Assignments
 *     outside [0, clusters) belong to no cluster (`index == k` never holds).
 *   - across ranks: the fold of reduce.h (canonical rank order), then
 *     centroid = sum / (float)count with IEEE division (kmeans_smi.cl:200);
 *     an empty cluster becomes 0/0 = NaN, as in the reference.
 */
#ifndef SMI_KMEANS_H
#define SMI_KMEANS_H

#include "communicator.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ComputeDistance on n points (row-major n x dims, device memory):
 * assignment[p] = cluster of point p under `centroids` (clusters x dims).
 * dims must be a multiple of width, 1 <= clusters <= 256 and
 * clusters * dims / width <= 16384. */
int smi_kmeans_assign(const float *points, int n, int dims, const float *centroids, int clusters,
                      int width, int *assignment, SMI_Stream stream);

/* The accumulation half of ComputeMeans on one rank: sums (clusters x dims)
 * and counts (clusters) of the points assigned to each cluster, in point
 * order.  Scratch is stream-ordered device memory. */
int smi_kmeans_accumulate(const float *points, int n, int dims, const int *assignment, int clusters,
                          float *sums, int *counts, SMI_Stream stream);

/* The whole kmeans_smi program on this rank's n_local points: `iterations`
 * rounds of assign, accumulate, SMI_Reduce to rank 0, SMI_Bcast and divide.
 * `centroids` (clusters x dims, device) holds the initial centroids on entry
 * -- the same on every rank, as after the host's MPI_Bcast
 * (kmeans_smi.cpp:164) -- and the final ones on return, on every rank.  All
 * work is enqueued on `stream`; the call does not synchronise the host. */
int smi_kmeans(SMI_Comm comm, const float *points, int n_local, int dims, int clusters, int width,
               float *centroids, int iterations, SMI_Stream stream);

#ifdef __cplusplus
}
#endif
#endif /* SMI_KMEANS_H */
