// gesummv.hip -- the gesummv_smi hot path: y = alpha*A*x + beta*B*x.
//
// Reference replaced (ryutakashino/SMI):
//   gemv  examples/kernels/gesummv_rank0.cl:53-181 (and gesummv_rank1.cl:50-187)
//         row-streamed GEMV, W=64, TILE_M=128: per 64-element chunk a
//         sequential dot product c_k (:137-149), per 128-column tile
//         acc = (0 + alpha*c_{2t}) + alpha*c_{2t+1} (:111,158), and the row
//         result y = ((0 + acc_0) + acc_1) + ... (:126-127,171)
//   axpy  gesummv_rank0.cl:184-203: y = (alpha*A*x)_i + (beta*B*x)_i with the
//         beta*B*x stream SMI_Pushed from rank 1 (gesummv_rank1.cl:95,182)
// MI355X design: the functional split (A on rank 0, B on rank 1) becomes a
// row split over all ranks -- each rank owns contiguous rows of both A and B
// and computes both terms locally, so only the y chunks travel (to the root).
// One workgroup per row: every lane owns one 64-element chunk and forms c_k
// in the reference order; lane pairs form the tile sums through DPP; the
// strictly sequential row fold runs in one lane per matrix.
#include <algorithm>

#include "smi_internal.h"

namespace smi {

__device__ __forceinline__ float dpp_from_next(float v) {  // lane i <- lane i+1
    return __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, false));
}

// c_k for chunk k of row `a` (64 products, summed sequentially from 0).
__device__ __forceinline__ float chunk_dot(const float *__restrict__ a, const float *__restrict__ x, int k) {
    const float4 *ap = reinterpret_cast<const float4 *>(a + 64 * (size_t)k);
    const float4 *xp = reinterpret_cast<const float4 *>(x + 64 * (size_t)k);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const float4 av = ap[j], xv = xp[j];
        acc = __fadd_rn(acc, __fmul_rn(av.x, xv.x));
        acc = __fadd_rn(acc, __fmul_rn(av.y, xv.y));
        acc = __fadd_rn(acc, __fmul_rn(av.z, xv.z));
        acc = __fadd_rn(acc, __fmul_rn(av.w, xv.w));
    }
    return acc;
}

// One block per row.  LDS holds the per-tile sums of A (and B).
template <bool HAS_B>
__global__ __launch_bounds__(256) void gemv_rows_kernel(const float *__restrict__ A,
                                                        const float *__restrict__ B,
                                                        const float *__restrict__ x, float *__restrict__ y,
                                                        int m, int lda, float alpha, float beta) {
    extern __shared__ __attribute__((aligned(16))) float tiles[];
    const int row = blockIdx.x;
    const int nchunks = m / 64;
    const int ntiles = (nchunks + 1) / 2;
    float *tA = tiles;
    float *tB = tiles + ntiles;
    const float *a = A + (size_t)row * lda;
    const float *b = HAS_B ? B + (size_t)row * lda : nullptr;
    // Rounds of 256 chunks; every lane of the block takes part in the DPP.
    for (int base = 0; base < nchunks; base += 256) {
        const int k = base + threadIdx.x;
        const bool valid = k < nchunks;
        const int kc = valid ? k : nchunks - 1;  // in-bounds even if speculated
        const float cA = valid ? chunk_dot(a, x, kc) : 0.f;  // missing chunk: c = +0
        const float nA = dpp_from_next(cA);
        float cB = 0.f, nB = 0.f;
        if constexpr (HAS_B) {
            cB = valid ? chunk_dot(b, x, kc) : 0.f;
            nB = dpp_from_next(cB);
        }
        if (valid && (k & 1) == 0) {
            const int t = k >> 1;
            tA[t] = __fadd_rn(__fadd_rn(0.f, __fmul_rn(alpha, cA)), __fmul_rn(alpha, nA));
            if constexpr (HAS_B)
                tB[t] = __fadd_rn(__fadd_rn(0.f, __fmul_rn(beta, cB)), __fmul_rn(beta, nB));
        }
    }
    __syncthreads();
    // sequential row folds: lane 0 folds A, lane 64 (next wave) folds B
    if (threadIdx.x == 0 || (HAS_B && threadIdx.x == 64)) {
        const float *t = threadIdx.x == 0 ? tA : tB;
        float acc = 0.f;
        for (int i = 0; i < ntiles; ++i) acc = __fadd_rn(acc, t[i]);
        if (threadIdx.x == 64) tB[0] = acc;  // hand yB to lane 0 (tB[0] already consumed)
        else tA[0] = acc;
    }
    __syncthreads();
    if (threadIdx.x == 0) y[row] = HAS_B ? __fadd_rn(tA[0], tB[0]) : tA[0];
}

static int launch_gemv(const float *A, const float *B, const float *x, float *y, int n, int m, int lda,
                       float alpha, float beta, hipStream_t s) {
    if (n == 0) return SMI_SUCCESS;
    const int ntiles = (m / 64 + 1) / 2;
    const size_t lds = (size_t)2 * std::max(ntiles, 1) * sizeof(float);
    SMI_ARG_CHECK(lds <= 64 * 1024, "m too large for one row per workgroup");
    int tok = -1;
    if (prof_enabled()) SMI_TRY(prof_begin(SMI_PROF_GEMV, s, &tok));
    if (B)
        hipLaunchKernelGGL(gemv_rows_kernel<true>, dim3(n), dim3(256), lds, s, A, B, x, y, m, lda, alpha, beta);
    else
        hipLaunchKernelGGL(gemv_rows_kernel<false>, dim3(n), dim3(256), lds, s, A, B, x, y, m, lda, alpha,
                           beta);
    SMI_HIP_CHECK(hipGetLastError());
    if (tok >= 0) SMI_TRY(prof_end(tok, s));
    return SMI_SUCCESS;
}

}  // namespace smi

using namespace smi;

extern "C" {

int smi_gemv_rows(const float *A, const float *B, const float *x, float *y, int n, int m, int lda,
                  float alpha, float beta, SMI_Stream stream) {
    SMI_ARG_CHECK(n >= 0 && m >= 0 && m % 64 == 0, "m must be a multiple of 64");
    SMI_ARG_CHECK(lda >= m && lda % 4 == 0, "lda must be >= m and a multiple of 4");
    if (n == 0) return SMI_SUCCESS;
    SMI_ARG_CHECK(A && x && y, "NULL buffer");
    SMI_ARG_CHECK(((uintptr_t)A & 15u) == 0 && ((uintptr_t)x & 15u) == 0 && (!B || ((uintptr_t)B & 15u) == 0),
                  "A, B, x must be 16-byte aligned");
    return launch_gemv(A, B, x, y, n, m, lda, alpha, beta, (hipStream_t)stream);
}

int smi_gesummv(SMI_Comm comm, const float *A_rows, const float *B_rows, const float *x, float *y,
                int n_global, int m, float alpha, float beta, int root, SMI_Stream stream_) {
    Comm *c = lookup_comm(comm);
    if (!c) {
        set_error("unknown communicator");
        return SMI_ERR_BAD_COMM;
    }
    const int n = c->size, me = c->rank;
    SMI_ARG_CHECK(root >= 0 && root < n, "root out of range");
    SMI_ARG_CHECK(n_global >= 0, "n_global < 0");
    SMI_ARG_CHECK(me != root || y, "NULL y on root");
    hipStream_t s = (hipStream_t)stream_;
    auto row0 = [&](int r) { return (int)((long)n_global * r / n); };
    const int my0 = row0(me), my_n = row0(me + 1) - my0;
    float *ychunk = nullptr;
    if (me == root) {
        ychunk = y + my0;
    } else {
        void *ws = nullptr;
        SMI_TRY(comm_workspace(c, (size_t)std::max(my_n, 1) * sizeof(float), &ws));
        ychunk = (float *)ws;
    }
    SMI_TRY(smi_gemv_rows(A_rows, B_rows, x, ychunk, my_n, m, m, alpha, beta, stream_));
    if (n == 1) return SMI_SUCCESS;
    // stream the partial y chunks to the root (the rank-1 SMI_Push of
    // beta*B*x and rank-0 SMI_Pop in the reference)
    Transport *tp = c->transport.get();
    SMI_TRY(tp->begin(s));
    if (me == root) {
        for (int k = 0; k < n; ++k)
            if (k != root) SMI_TRY(tp->recv(y + row0(k), (size_t)(row0(k + 1) - row0(k)) * sizeof(float), k));
    } else {
        SMI_TRY(tp->send(ychunk, (size_t)my_n * sizeof(float), root));
    }
    return tp->end();
}

}  // extern "C"
