// kmeans.hip -- the kmeans_smi program on MI355X.
//
// Reference replaced (ryutakashino/SMI):
//   SendCentroids    examples/kernels/kmeans_smi.cl:14-34
//   ComputeDistance  kmeans_smi.cl:36-88   per point: K squared distances over
//                    W-wide vectors, the first strictly smallest wins
//   ComputeMeans     kmeans_smi.cl:90-209  per-cluster sums and counts in point
//                    order, SMI_Reduce to rank 0 (ports 0, 2), SMI_Bcast
//                    (ports 1, 3), centroid = sum / count
// The FPGA version is three single-work-item kernels joined by channels.  On
// MI355X one iteration is:
//   assign_kernel    one thread per point; the centroid lanes the distance
//                    reads are staged in LDS
//   count_kernel     per 256-point block, a cluster histogram (LDS atomics)
//   scan_kernel      per cluster, exclusive prefix over the blocks
//   base_kernel      exclusive prefix over the clusters
//   scatter_kernel   order-preserving compaction: list = the points of
//                    cluster 0 in point order, then those of cluster 1, ...
//   fold_kernel      one workgroup per (cluster, 16 dimensions): all waves
//                    gather the cluster's rows into an LDS tile, wave 0 adds
//                    them in point order while the next tile is in flight
//   smi_reduce / smi_bcast (collectives.hip), divide_kernel
// The per-cluster sums are sequential fp32 chains (the reference's order), so
// each chain is serial by definition; the compaction makes a chain only as
// long as its cluster and runs every (cluster, dimension) chain at once.
// Adding +0 for the points of other clusters (kmeans_smi.cl:122) never
// changes an fp32 sum that starts at +0 (such a sum is never -0), so the
// chains skip those points; the oracle restates the literal form and the GPU
// tests compare bitwise.
#include <algorithm>

#include "smi_internal.h"

namespace smi {

constexpr int kPtsPerBlock = 256;  // assign / count / scatter
constexpr int kMaxClusters = 256;
constexpr int kQReg = 16;          // distance lanes held in registers
constexpr int kFoldWaves = 8;
constexpr int kFoldDims = 8;                        // dimensions per workgroup (32-B row pieces)
constexpr int kRowsPerLoad = 64 / kFoldDims;        // rows one wave-load covers
constexpr int kLoadsPerWave = 32;
constexpr int kRowsPerWave = kLoadsPerWave * kRowsPerLoad;
constexpr int kFoldRows = kFoldWaves * kRowsPerWave;  // rows per LDS tile (64 KiB)

// ComputeDistance (kmeans_smi.cl:54-85): per W-wide vector only the last
// lane's squared difference is added (the unrolled `=` of :68-71).
template <bool REG>
__global__ __launch_bounds__(kPtsPerBlock) void assign_kernel(const float *__restrict__ pts, int n, int dims,
                                                             const float *__restrict__ cen, int clusters,
                                                             int width, int *__restrict__ idx) {
    extern __shared__ float cl[];  // [clusters][q]: the centroid lanes the distance reads
    const int q = dims / width;
    for (int i = threadIdx.x; i < clusters * q; i += kPtsPerBlock) {
        const int k = i / q, j = i - k * q;
        cl[i] = cen[(size_t)k * dims + (size_t)j * width + width - 1];
    }
    __syncthreads();
    const int p = blockIdx.x * kPtsPerBlock + threadIdx.x;
    if (p >= n) return;
    const float *x = pts + (size_t)p * dims + width - 1;
    float min_dist = __builtin_inff();
    int best = 0;
    if constexpr (REG) {
        float xv[kQReg];
#pragma unroll
        for (int j = 0; j < kQReg; ++j) xv[j] = x[(size_t)min(j, q - 1) * width];
        for (int k = 0; k < clusters; ++k) {
            const float *c = cl + k * q;
            float dist = 0.f;
#pragma unroll
            for (int j = 0; j < kQReg; ++j) {
                if (j < q) {
                    const float diff = __fadd_rn(xv[j], -c[j]);
                    dist = __fadd_rn(dist, __fmul_rn(diff, diff));
                }
            }
            if (dist < min_dist) {
                min_dist = dist;
                best = k;
            }
        }
    } else {
        for (int k = 0; k < clusters; ++k) {
            const float *c = cl + k * q;
            float dist = 0.f;
            for (int j = 0; j < q; ++j) {
                const float diff = __fadd_rn(x[(size_t)j * width], -c[j]);
                dist = __fadd_rn(dist, __fmul_rn(diff, diff));
            }
            if (dist < min_dist) {
                min_dist = dist;
                best = k;
            }
        }
    }
    idx[p] = best;
}

// Per-block cluster histogram.  Assignments outside [0, clusters) count for
// no cluster (the reference's `index == k` never holds for them).
__global__ __launch_bounds__(kPtsPerBlock) void count_kernel(const int *__restrict__ idx, int n, int clusters,
                                                            int nblocks, int *__restrict__ bcount) {
    __shared__ int h[kMaxClusters];
    for (int k = threadIdx.x; k < clusters; k += kPtsPerBlock) h[k] = 0;
    __syncthreads();
    const int p = blockIdx.x * kPtsPerBlock + threadIdx.x;
    if (p < n) {
        const int k = idx[p];
        if (k >= 0 && k < clusters) atomicAdd(&h[k], 1);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < clusters; k += kPtsPerBlock) bcount[(size_t)k * nblocks + blockIdx.x] = h[k];
}

// Per cluster: exclusive prefix of its block counts (in place); the total
// is the cluster's count.
__global__ __launch_bounds__(1024) void scan_kernel(int *__restrict__ bcount, int nblocks,
                                                    int *__restrict__ counts) {
    __shared__ int wsum[16];
    int *row = bcount + (size_t)blockIdx.x * nblocks;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int carry = 0;
    for (int b0 = 0; b0 < nblocks; b0 += 1024) {
        const int i = b0 + threadIdx.x;
        const int v = i < nblocks ? row[i] : 0;
        int s = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(s, o);
            if (lane >= o) s += t;
        }
        if (lane == 63) wsum[w] = s;
        __syncthreads();
        int before = 0, total = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            before += j < w ? wsum[j] : 0;
            total += wsum[j];
        }
        if (i < nblocks) row[i] = carry + before + s - v;
        carry += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) counts[blockIdx.x] = carry;
}

// Exclusive prefix over the clusters: where each cluster's list starts.
__global__ __launch_bounds__(kMaxClusters) void base_kernel(const int *__restrict__ counts, int clusters,
                                                           int *__restrict__ base) {
    __shared__ int s[kMaxClusters];
    const int k = threadIdx.x;
    const int v = k < clusters ? counts[k] : 0;
    s[k] = v;
    __syncthreads();
    for (int o = 1; o < kMaxClusters; o <<= 1) {
        const int t = k >= o ? s[k - o] : 0;
        __syncthreads();
        s[k] += t;
        __syncthreads();
    }
    if (k < clusters) base[k] = s[k] - v;
}

// Order-preserving compaction: point p of cluster k goes to
// list[base[k] + (points of k in earlier blocks) + (earlier points of k in
// this block)].
__global__ __launch_bounds__(kPtsPerBlock) void scatter_kernel(const int *__restrict__ idx, int n, int clusters,
                                                              int nblocks, const int *__restrict__ boff,
                                                              const int *__restrict__ base,
                                                              int *__restrict__ list) {
    constexpr int NW = kPtsPerBlock / 64;
    __shared__ int wcnt[NW][kMaxClusters];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int k = threadIdx.x; k < clusters; k += kPtsPerBlock)
        for (int j = 0; j < NW; ++j) wcnt[j][k] = 0;
    __syncthreads();
    const int p = blockIdx.x * kPtsPerBlock + threadIdx.x;
    int k = p < n ? idx[p] : -1;
    if (k < 0 || k >= clusters) k = -1;
    // rank among the lanes of this wave with the same cluster (lane order =
    // point order); one ballot per distinct cluster present in the wave
    int rank = 0;
    unsigned long long rem = __ballot(k >= 0);
    while (rem) {
        const int kk = __shfl(k, __builtin_ctzll(rem));
        const unsigned long long m = __ballot(k == kk);
        if (k == kk) rank = __popcll(m & ((1ull << lane) - 1));
        if (lane == 0) wcnt[w][kk] = __popcll(m);
        rem &= ~m;
    }
    __syncthreads();
    if (k >= 0) {
        int off = base[k] + boff[(size_t)k * nblocks + blockIdx.x] + rank;
        for (int j = 0; j < w; ++j) off += wcnt[j][k];
        list[off] = p;
    }
}

// ComputeMeans accumulation (kmeans_smi.cl:113-127): sums[k][d] = the fp32
// chain over the points of cluster k in point order, from +0.  The chain is
// serial, so the workgroup's job is to keep it fed.  A CU fetches ~11 B/cycle,
// so one workgroup per cluster would cap a chain at ~10 ns per point for 64
// dims: each workgroup takes 16 dimensions (64-B row pieces, 4 rows per
// wave-load) and all its waves gather rows two tiles ahead into registers and stage them into a double-buffered
// LDS tile, while wave 0 adds the current tile in point order.  One barrier
// per tile: tile t+1 goes into the buffer tile t-1 used, which every wave
// finished with before the previous barrier.
__global__ __launch_bounds__(64 * kFoldWaves) void fold_kernel(const float *__restrict__ pts, int dims,
                                                              const int *__restrict__ list,
                                                              const int *__restrict__ counts,
                                                              const int *__restrict__ base,
                                                              float *__restrict__ sums) {
    // transposed tile [dim][row]: a chain reads 4 rows per ds_read_b128; the
    // +8 pad puts the 8 dims x 8 rows of one wave-store in 64 distinct banks
    constexpr int TS = kFoldRows + 8;
    __shared__ __attribute__((aligned(16))) float tile[2][kFoldDims][TS];
    const int k = blockIdx.x;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int sub = lane / kFoldDims;                 // row within a wave-load
    const int d = blockIdx.y * kFoldDims + (lane % kFoldDims);
    const int dc = min(d, dims - 1);
    const int cnt = counts[k];
    const int *lst = list + base[k];
    const int ntiles = (cnt + kFoldRows - 1) / kFoldRows;
    float va[kLoadsPerWave], vb[kLoadsPerWave];
    auto gather = [&](float (&v)[kLoadsPerWave], int t) {
#pragma unroll
        for (int r = 0; r < kLoadsPerWave; ++r) {
            const int j = min(t * kFoldRows + w * kRowsPerWave + r * kRowsPerLoad + sub, cnt - 1);
            v[r] = pts[(size_t)lst[j] * dims + dc];
        }
    };
    auto put = [&](const float (&v)[kLoadsPerWave], int t) {
#pragma unroll
        for (int r = 0; r < kLoadsPerWave; ++r)
            tile[t & 1][lane % kFoldDims][w * kRowsPerWave + r * kRowsPerLoad + sub] = v[r];
    };
    float acc = 0.f;
    auto add = [&](int t) {
        if (w == 0) {
            const int rows = min(kFoldRows, cnt - t * kFoldRows);
            const int c = lane % kFoldDims;  // lanes >= kFoldDims repeat lane c's chain
            const float *tl = tile[t & 1][c];
            // 16 LDS reads in flight ahead of the dependent adds (lgkmcnt holds 15)
            int r = 0;
            for (; r + 16 <= rows; r += 16) {
                float4 x4[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) x4[i] = *reinterpret_cast<const float4 *>(tl + r + 4 * i);
                const float *x = reinterpret_cast<const float *>(x4);
#pragma unroll
                for (int i = 0; i < 16; ++i) acc = __fadd_rn(acc, x[i]);
            }
            for (; r < rows; ++r) acc = __fadd_rn(acc, tl[r]);
        }
    };
    // one pipeline step: tile t is in LDS, `cur` holds tile t+1, `nxt` gets t+2
    auto step = [&](float (&cur)[kLoadsPerWave], float (&nxt)[kLoadsPerWave], int t) {
        if (t + 2 < ntiles) gather(nxt, t + 2);
        add(t);
        if (t + 1 < ntiles) put(cur, t + 1);
        __syncthreads();
    };
    if (ntiles > 0) {
        gather(va, 0);
        if (ntiles > 1) gather(vb, 1);
        put(va, 0);
        __syncthreads();
        for (int t = 0; t < ntiles; t += 2) {
            step(vb, va, t);
            if (t + 1 < ntiles) step(va, vb, t + 1);
        }
    }
    if (w == 0 && lane < kFoldDims && d < dims) sums[(size_t)k * dims + d] = acc;
}

// centroid = sum / (float)count, IEEE division (kmeans_smi.cl:196-205)
__global__ void divide_kernel(const float *__restrict__ sums, const int *__restrict__ counts,
                              float *__restrict__ cen, int clusters, int dims) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= clusters * dims) return;
    cen[i] = __fdiv_rn(sums[i], (float)counts[i / dims]);
}

// ---------------------------------------------------------------- host ----
static size_t up256(size_t b) { return (b + 255) & ~(size_t)255; }

struct KmeansWork {
    int *idx, *bcount, *list, *counts, *base;
    float *sums;
    size_t bytes;
};

static KmeansWork kmeans_layout(char *ws, int n, int dims, int clusters) {
    const size_t nb = ((size_t)n + kPtsPerBlock - 1) / kPtsPerBlock;
    KmeansWork w{};
    size_t o = 0;
    auto take = [&](size_t b) {
        char *p = ws ? ws + o : nullptr;
        o += up256(std::max(b, (size_t)4));
        return p;
    };
    w.idx = (int *)take((size_t)n * 4);
    w.list = (int *)take((size_t)n * 4);
    w.bcount = (int *)take((size_t)clusters * nb * 4);
    w.counts = (int *)take((size_t)clusters * 4);
    w.base = (int *)take((size_t)clusters * 4);
    w.sums = (float *)take((size_t)clusters * dims * 4);
    w.bytes = o;
    return w;
}

static int check_shape(int n, int dims, int clusters, int width) {
    SMI_ARG_CHECK(n >= 0 && dims >= 1, "need n >= 0 and dims >= 1");
    SMI_ARG_CHECK(clusters >= 1 && clusters <= kMaxClusters, "clusters must be in [1, 256]");
    SMI_ARG_CHECK(width >= 1 && dims % width == 0, "dims must be a multiple of width");
    SMI_ARG_CHECK((long)clusters * (dims / width) <= 16384, "clusters * dims / width must be <= 16384");
    SMI_ARG_CHECK((long)n * dims < (1L << 40), "points too large");
    return SMI_SUCCESS;
}

static int launch_assign(const float *pts, int n, int dims, const float *cen, int clusters, int width, int *idx,
                         hipStream_t s) {
    if (n == 0) return SMI_SUCCESS;
    const int q = dims / width;
    const size_t lds = (size_t)clusters * q * sizeof(float);
    const int nb = (n + kPtsPerBlock - 1) / kPtsPerBlock;
    int tok = -1;
    if (prof_enabled()) SMI_TRY(prof_begin(SMI_PROF_KMEANS_ASSIGN, s, &tok));
    if (q <= kQReg)
        hipLaunchKernelGGL(assign_kernel<true>, dim3(nb), dim3(kPtsPerBlock), lds, s, pts, n, dims, cen, clusters,
                           width, idx);
    else
        hipLaunchKernelGGL(assign_kernel<false>, dim3(nb), dim3(kPtsPerBlock), lds, s, pts, n, dims, cen, clusters,
                           width, idx);
    SMI_HIP_CHECK(hipGetLastError());
    if (tok >= 0) SMI_TRY(prof_end(tok, s));
    return SMI_SUCCESS;
}

static int launch_accumulate(const float *pts, int n, int dims, const int *idx, int clusters, float *sums,
                             int *counts, const KmeansWork &w, hipStream_t s) {
    const int nb = (n + kPtsPerBlock - 1) / kPtsPerBlock;
    if (nb > 0)
        hipLaunchKernelGGL(count_kernel, dim3(nb), dim3(kPtsPerBlock), 0, s, idx, n, clusters, nb, w.bcount);
    hipLaunchKernelGGL(scan_kernel, dim3(clusters), dim3(1024), 0, s, w.bcount, nb, counts);
    hipLaunchKernelGGL(base_kernel, dim3(1), dim3(kMaxClusters), 0, s, counts, clusters, w.base);
    if (nb > 0)
        hipLaunchKernelGGL(scatter_kernel, dim3(nb), dim3(kPtsPerBlock), 0, s, idx, n, clusters, nb, w.bcount,
                           w.base, w.list);
    int tok = -1;
    if (prof_enabled()) SMI_TRY(prof_begin(SMI_PROF_KMEANS_FOLD, s, &tok));
    hipLaunchKernelGGL(fold_kernel, dim3(clusters, (dims + kFoldDims - 1) / kFoldDims), dim3(64 * kFoldWaves), 0, s, pts, dims,
                       w.list, counts, w.base, sums);
    SMI_HIP_CHECK(hipGetLastError());
    if (tok >= 0) SMI_TRY(prof_end(tok, s));
    return SMI_SUCCESS;
}

static int launch_divide(const float *sums, const int *counts, float *cen, int clusters, int dims,
                         hipStream_t s) {
    const int total = clusters * dims;
    hipLaunchKernelGGL(divide_kernel, dim3((total + 255) / 256), dim3(256), 0, s, sums, counts, cen, clusters,
                       dims);
    SMI_HIP_CHECK(hipGetLastError());
    return SMI_SUCCESS;
}

}  // namespace smi

using namespace smi;

extern "C" {

int smi_kmeans_assign(const float *points, int n, int dims, const float *centroids, int clusters, int width,
                      int *assignment, SMI_Stream stream) {
    SMI_TRY(check_shape(n, dims, clusters, width));
    if (n == 0) return SMI_SUCCESS;
    SMI_ARG_CHECK(points && centroids && assignment, "NULL buffer");
    return launch_assign(points, n, dims, centroids, clusters, width, assignment, (hipStream_t)stream);
}

int smi_kmeans_accumulate(const float *points, int n, int dims, const int *assignment, int clusters, float *sums,
                          int *counts, SMI_Stream stream) {
    SMI_TRY(check_shape(n, dims, clusters, 1));
    SMI_ARG_CHECK(sums && counts && (n == 0 || (points && assignment)), "NULL buffer");
    hipStream_t s = (hipStream_t)stream;
    const KmeansWork sz = kmeans_layout(nullptr, n, dims, clusters);
    void *ws = nullptr;
    SMI_HIP_CHECK(hipMallocAsync(&ws, sz.bytes, s));
    const KmeansWork w = kmeans_layout((char *)ws, n, dims, clusters);
    const int rc = launch_accumulate(points, n, dims, assignment, clusters, sums, counts, w, s);
    SMI_HIP_CHECK(hipFreeAsync(ws, s));
    return rc;
}

int smi_kmeans(SMI_Comm comm, const float *points, int n, int dims, int clusters, int width, float *centroids,
               int iterations, SMI_Stream stream) {
    Comm *c = lookup_comm(comm);
    if (!c) {
        set_error("unknown communicator");
        return SMI_ERR_BAD_COMM;
    }
    SMI_TRY(check_shape(n, dims, clusters, width));
    SMI_ARG_CHECK(iterations >= 0, "iterations < 0");
    SMI_ARG_CHECK(centroids && (n == 0 || points), "NULL buffer");
    if (iterations == 0) return SMI_SUCCESS;
    hipStream_t s = (hipStream_t)stream;
    const size_t kd = (size_t)clusters * dims;
    const KmeansWork sz = kmeans_layout(nullptr, n, dims, clusters);
    const size_t extra = up256(kd * 4) + up256((size_t)clusters * 4);  // reduced sums / counts
    void *ws = nullptr;
    SMI_HIP_CHECK(hipMallocAsync(&ws, sz.bytes + extra, s));
    const KmeansWork w = kmeans_layout((char *)ws, n, dims, clusters);
    float *rsums = (float *)((char *)ws + sz.bytes);
    int *rcounts = (int *)((char *)rsums + up256(kd * 4));
    int rc = SMI_SUCCESS;
    for (int it = 0; it < iterations && rc == SMI_SUCCESS; ++it) {
        rc = launch_assign(points, n, dims, centroids, clusters, width, w.idx, s);
        if (rc == SMI_SUCCESS) rc = launch_accumulate(points, n, dims, w.idx, clusters, w.sums, w.counts, w, s);
        // ComputeMeans' collectives with the reference's ports and order
        // (kmeans_smi.cl:132-192); the result reaches every rank
        if (rc == SMI_SUCCESS) rc = smi_reduce(comm, w.sums, rsums, kd, SMI_FLOAT, SMI_ADD, 0, 0, stream);
        if (rc == SMI_SUCCESS) rc = smi_bcast(comm, rsums, kd, SMI_FLOAT, 0, 1, stream);
        if (rc == SMI_SUCCESS) rc = smi_reduce(comm, w.counts, rcounts, clusters, SMI_INT, SMI_ADD, 0, 2, stream);
        if (rc == SMI_SUCCESS) rc = smi_bcast(comm, rcounts, clusters, SMI_INT, 0, 3, stream);
        if (rc == SMI_SUCCESS) rc = launch_divide(rsums, rcounts, centroids, clusters, dims, s);
    }
    const hipError_t fe = hipFreeAsync(ws, s);
    if (rc == SMI_SUCCESS && fe != hipSuccess) {
        set_error(std::string("hipFreeAsync: ") + hipGetErrorString(fe));
        rc = SMI_ERR_HIP;
    }
    return rc;
}

}  // extern "C"
