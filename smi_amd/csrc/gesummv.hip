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
//
// One wave per row (A and B).  The row is walked in slabs of 64 chunks
// (16 KiB): the wave reads a slab with fully coalesced float4 loads, forms
// the products a*x in that layout, and transposes them through LDS so that
// lane l holds chunk l and sums its 64 products sequentially (the reference
// order).  Lane pairs form the tile sums through DPP, and the sequential row
// fold consumes the slab's tiles in order from lane 0 (readlane), so no tile
// array is kept and m is unbounded.
#include <algorithm>

#include "smi_internal.h"

namespace smi {

__device__ __forceinline__ float dpp_from_next(float v) {  // lane i <- lane i+1
    return __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, false));
}

__device__ __forceinline__ float4 mul4(float4 a, float4 b) {
    return make_float4(__fmul_rn(a.x, b.x), __fmul_rn(a.y, b.y), __fmul_rn(a.z, b.z), __fmul_rn(a.w, b.w));
}

// LDS between the writes and reads of other lanes of the same wave
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float4 ld_stream(const float *p) {
    using V4 = float __attribute__((ext_vector_type(4)));
    const V4 v = __builtin_nontemporal_load(reinterpret_cast<const V4 *>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}

constexpr int kGemvWaves = 4;
constexpr int kSlabStride = 17;  // float4s per chunk in LDS (64 floats + 4 pad: conflict-free)

// c for the chunk this lane owns: products of slab `pv` (coalesced layout:
// pv[j] = elements 4*(64j + lane) .. +3 of the slab) transposed through `wb`.
__device__ __forceinline__ float chunk_sum(float4 *wb, const float4 (&pv)[16], int lane) {
#pragma unroll
    for (int j = 0; j < 16; ++j) wb[(4 * j + (lane >> 4)) * kSlabStride + (lane & 15)] = pv[j];
    wave_lds_sync();
    float c = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const float4 p = wb[lane * kSlabStride + q];
        c = __fadd_rn(c, p.x);
        c = __fadd_rn(c, p.y);
        c = __fadd_rn(c, p.z);
        c = __fadd_rn(c, p.w);
    }
    wave_lds_sync();  // reads done before the next slab overwrites
    return c;
}

template <bool HAS_B>
__global__ __launch_bounds__(64 * kGemvWaves) void gemv_rows_kernel(const float *__restrict__ A,
                                                                   const float *__restrict__ B,
                                                                   const float *__restrict__ x,
                                                                   float *__restrict__ y, int n, int m, int lda,
                                                                   float alpha, float beta) {
    __shared__ float4 lds[kGemvWaves][64 * kSlabStride];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * kGemvWaves + wave;
    if (row >= n) return;  // wave-uniform; the kernel has no block barrier
    float4 *wb = lds[wave];
    const int nchunks = m >> 6;
    const float *a = A + (size_t)row * lda;
    const float *b = HAS_B ? B + (size_t)row * lda : a;
    float accA = 0.f, accB = 0.f;
    for (int cbase = 0; cbase < nchunks; cbase += 64) {
        float4 pa[16], pb[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int ch = min(cbase + 4 * j + (lane >> 4), nchunks - 1);  // clamped: the tail
            const int e = ch * 64 + (lane & 15) * 4;                       // chunk's c is replaced
            const float4 xv = *reinterpret_cast<const float4 *>(x + e);
            pa[j] = mul4(ld_stream(a + e), xv);  // A, B streamed once; x stays cached
            if constexpr (HAS_B) pb[j] = mul4(ld_stream(b + e), xv);
        }
        const bool valid = cbase + lane < nchunks;
        // every lane writes slots of other lanes' chunks: transpose on all
        // lanes, then replace a missing chunk's c by +0
        float cA = chunk_sum(wb, pa, lane);
        cA = valid ? cA : 0.f;
        const float nA = dpp_from_next(cA);
        const float tA = __fadd_rn(__fadd_rn(0.f, __fmul_rn(alpha, cA)), __fmul_rn(alpha, nA));
        float tB = 0.f;
        if constexpr (HAS_B) {
            float cB = chunk_sum(wb, pb, lane);
            cB = valid ? cB : 0.f;
            const float nB = dpp_from_next(cB);
            tB = __fadd_rn(__fadd_rn(0.f, __fmul_rn(beta, cB)), __fmul_rn(beta, nB));
        }
        // tiles of this slab live in the even lanes, in order
        const int ntl = min(32, (nchunks - cbase + 1) >> 1);
        for (int k = 0; k < ntl; ++k) {
            accA = __fadd_rn(accA, __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                                                                 __builtin_bit_cast(int, tA), 2 * k)));
            if constexpr (HAS_B)
                accB = __fadd_rn(accB, __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                                                                     __builtin_bit_cast(int, tB), 2 * k)));
        }
    }
    if (lane == 0) y[row] = HAS_B ? __fadd_rn(accA, accB) : accA;
}

static int launch_gemv(const float *A, const float *B, const float *x, float *y, int n, int m, int lda,
                       float alpha, float beta, hipStream_t s) {
    if (n == 0) return SMI_SUCCESS;
    int tok = -1;
    if (prof_enabled()) SMI_TRY(prof_begin(SMI_PROF_GEMV, s, &tok));
    const dim3 grid((n + kGemvWaves - 1) / kGemvWaves), block(64 * kGemvWaves);
    if (B)
        hipLaunchKernelGGL(gemv_rows_kernel<true>, grid, block, 0, s, A, B, x, y, n, m, lda, alpha, beta);
    else
        hipLaunchKernelGGL(gemv_rows_kernel<false>, grid, block, 0, s, A, B, x, y, n, m, lda, alpha, beta);
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
    Group grp(tp);
    SMI_TRY(grp.begin(s));
    if (me == root) {
        for (int k = 0; k < n; ++k)
            if (k != root) SMI_TRY(tp->recv(y + row0(k), (size_t)(row0(k + 1) - row0(k)) * sizeof(float), k));
    } else {
        SMI_TRY(tp->send(ychunk, (size_t)my_n * sizeof(float), root));
    }
    return grp.end();
}

}  // extern "C"
