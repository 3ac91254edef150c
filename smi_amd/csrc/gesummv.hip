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
#include <cstdlib>

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

// c for the chunk this lane owns, continued over one pass of a slab: `pv`
// holds the pass's products in the coalesced layout (load j = chunks
// CPL*j .. CPL*j + CPL-1 of the slab, LPC lanes x float4 each) and is
// transposed through `wb` so that lane l sums chunk l's 64/H elements of this
// pass in order, continuing `c` (the reference's sequential chunk sum,
// gesummv_rank0.cl:137-149).
template <int H>
struct SlabPass {
    static constexpr int J = 16 / H;       // float4 loads per matrix per lane and pass
    static constexpr int LPC = 16 / H;     // lanes per chunk in a load
    static constexpr int CPL = 64 / LPC;   // chunks per load instruction
    static constexpr int SS = LPC + 1;     // float4 stride of a chunk in LDS (+1 pad: conflict-free)
    static constexpr int LDS_F4 = 64 * SS; // per wave
};

template <int H>
__device__ __forceinline__ float chunk_sum(float4 *wb, const float4 (&pv)[SlabPass<H>::J], int lane, float c) {
    using P = SlabPass<H>;
#pragma unroll
    for (int j = 0; j < P::J; ++j) wb[(P::CPL * j + lane / P::LPC) * P::SS + (lane % P::LPC)] = pv[j];
    wave_lds_sync();
#pragma unroll
    for (int q = 0; q < P::LPC; ++q) {
        const float4 p = wb[lane * P::SS + q];
        c = __fadd_rn(c, p.x);
        c = __fadd_rn(c, p.y);
        c = __fadd_rn(c, p.z);
        c = __fadd_rn(c, p.w);
    }
    wave_lds_sync();  // reads done before the next pass overwrites
    return c;
}

// Tile values of one slab (64 chunks = 32 tiles from chunk cbase on), read
// in H passes of 64/H elements per chunk: tile k of the slab ends up in lane
// 2k of tA (and tB), in the reference's per-tile order
// acc_t = (0 + alpha*c_{2t}) + alpha*c_{2t+1} (gesummv_rank0.cl:111,158);
// a chunk past the row's end counts as c = 0.
template <bool HAS_B, int H>
__device__ __forceinline__ void slab_tiles(const float *a, const float *b, const float *x, float4 *wb, int cbase,
                                           int nchunks, int lane, float alpha, float beta, float &tA, float &tB) {
    using P = SlabPass<H>;
    float cA = 0.f, cB = 0.f;
#pragma unroll
    for (int h = 0; h < H; ++h) {
        float4 pa[P::J], pb[P::J];
#pragma unroll
        for (int j = 0; j < P::J; ++j) {
            const int ch = min(cbase + P::CPL * j + lane / P::LPC, nchunks - 1);  // clamped: the tail
            const int e = ch * 64 + h * (64 / H) + (lane % P::LPC) * 4;            // chunk's c is replaced
            const float4 xv = *reinterpret_cast<const float4 *>(x + e);
            pa[j] = mul4(ld_stream(a + e), xv);  // A, B streamed once; x stays cached
            if constexpr (HAS_B) pb[j] = mul4(ld_stream(b + e), xv);
        }
        // every lane writes slots of other lanes' chunks: transpose on all lanes
        cA = chunk_sum<H>(wb, pa, lane, cA);
        if constexpr (HAS_B) cB = chunk_sum<H>(wb, pb, lane, cB);
    }
    const bool valid = cbase + lane < nchunks;  // replace a missing chunk's c by +0
    cA = valid ? cA : 0.f;
    const float nA = dpp_from_next(cA);
    tA = __fadd_rn(__fadd_rn(0.f, __fmul_rn(alpha, cA)), __fmul_rn(alpha, nA));
    tB = 0.f;
    if constexpr (HAS_B) {
        cB = valid ? cB : 0.f;
        const float nB = dpp_from_next(cB);
        tB = __fadd_rn(__fadd_rn(0.f, __fmul_rn(beta, cB)), __fmul_rn(beta, nB));
    }
}

// One wave per row: the slabs are walked in order and each slab's tiles are
// folded into the row sum straight from the even lanes (readlane), so no
// tile array is kept and m is unbounded.  Used for rows longer than
// kSplitMaxCols.
template <bool HAS_B>
__global__ __launch_bounds__(64 * kGemvWaves) void gemv_rows_kernel(const float *__restrict__ A,
                                                                   const float *__restrict__ B,
                                                                   const float *__restrict__ x,
                                                                   float *__restrict__ y, int n, int m, int lda,
                                                                   float alpha, float beta) {
    __shared__ float4 lds[kGemvWaves][SlabPass<1>::LDS_F4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * kGemvWaves + wave;
    if (row >= n) return;  // wave-uniform; the kernel has no block barrier
    float4 *wb = lds[wave];
    const int nchunks = m >> 6;
    const float *a = A + (size_t)row * lda;
    const float *b = HAS_B ? B + (size_t)row * lda : a;
    float accA = 0.f, accB = 0.f;
    for (int cbase = 0; cbase < nchunks; cbase += 64) {
        float tA, tB;
        slab_tiles<HAS_B, 1>(a, b, x, wb, cbase, nchunks, lane, alpha, beta, tA, tB);
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

// Row split over the workgroup's waves (rows up to kSplitMaxCols): wave w
// computes slabs w, w + 4, ... and parks their tile values in LDS at their
// place in the row; after one barrier wave 0 folds the row's tiles in order.
// A workgroup is a quarter of the old one-wave-per-row work unit, so the
// grid has 4x the units: a 4096-row shard (BASELINE config 5 per GPU) is
// 8 rounds of resident workgroups instead of 2, and no CU idles through a
// long last round.  The tile values and the fold order are those of
// gemv_rows_kernel, so the two are bit-identical.
constexpr int kSplitMaxCols = 32768;  // 2 KiB of tiles: 4 workgroups of 4 waves fill a CU's LDS
constexpr int kSplitMaxTiles = kSplitMaxCols / 128;
template <bool HAS_B, int H>
__global__ __launch_bounds__(64 * kGemvWaves) void gemv_split_kernel(const float *__restrict__ A,
                                                                    const float *__restrict__ B,
                                                                    const float *__restrict__ x,
                                                                    float *__restrict__ y, int n, int m, int lda,
                                                                    float alpha, float beta) {
    __shared__ float4 lds[kGemvWaves][SlabPass<H>::LDS_F4];
    __shared__ __attribute__((aligned(16))) float tiles[2][kSplitMaxTiles];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x;
    float4 *wb = lds[wave];
    const int nchunks = m >> 6;
    const float *a = A + (size_t)row * lda;
    const float *b = HAS_B ? B + (size_t)row * lda : a;
    for (int s = wave; s * 64 < nchunks; s += kGemvWaves) {
        float tA, tB;
        slab_tiles<HAS_B, H>(a, b, x, wb, s * 64, nchunks, lane, alpha, beta, tA, tB);
        // tile k of slab s -> tiles[s*32 + k]; missing tiles of the last
        // slab read +0 (acc is never -0, so + 0 leaves it unchanged)
        const int ntl = min(32, (nchunks - s * 64 + 1) >> 1);
        if ((lane & 1) == 0) {
            tiles[0][s * 32 + (lane >> 1)] = (lane >> 1) < ntl ? tA : 0.f;
            if constexpr (HAS_B) tiles[1][s * 32 + (lane >> 1)] = (lane >> 1) < ntl ? tB : 0.f;
        }
    }
    __syncthreads();
    if (wave != 0) return;
    const int nt4 = (((nchunks + 1) >> 1) + 3) >> 2;  // tiles, in float4 groups
    const float4 *tA4 = reinterpret_cast<const float4 *>(tiles[0]);
    const float4 *tB4 = reinterpret_cast<const float4 *>(tiles[1]);
    float accA = 0.f, accB = 0.f;
    for (int q = 0; q < nt4; ++q) {
        const float4 ta = tA4[q];  // every lane reads the same address: broadcast
        accA = __fadd_rn(__fadd_rn(__fadd_rn(__fadd_rn(accA, ta.x), ta.y), ta.z), ta.w);
        if constexpr (HAS_B) {
            const float4 tb = tB4[q];
            accB = __fadd_rn(__fadd_rn(__fadd_rn(__fadd_rn(accB, tb.x), tb.y), tb.z), tb.w);
        }
    }
    if (lane == 0) y[row] = HAS_B ? __fadd_rn(accA, accB) : accA;
}

// Launch variant (experiment build only, switch SMI_GEMV_VARIANT; the library: 0, the default):
// 1 = one wave per row for every shape; row split with 2 = whole-slab
// passes, 3 = quarter-slab passes (default: half-slab passes).
static int gemv_variant() {
#ifdef SMI_EXPERIMENTS  // experiment build only (smi_amd/build.py --experiments)
    static int v = [] {
        const char *e = getenv("SMI_GEMV_VARIANT");
        return e ? atoi(e) : 0;
    }();
    return v;
#else
    return 0;
#endif
}

template <int H>
static void launch_split(const float *A, const float *B, const float *x, float *y, int n, int m, int lda,
                         float alpha, float beta, hipStream_t s) {
    if (B)
        hipLaunchKernelGGL((gemv_split_kernel<true, H>), dim3(n), dim3(64 * kGemvWaves), 0, s, A, B, x, y, n, m, lda,
                           alpha, beta);
    else
        hipLaunchKernelGGL((gemv_split_kernel<false, H>), dim3(n), dim3(64 * kGemvWaves), 0, s, A, B, x, y, n, m,
                           lda, alpha, beta);
}

static int launch_gemv(const float *A, const float *B, const float *x, float *y, int n, int m, int lda,
                       float alpha, float beta, hipStream_t s) {
    if (n == 0) return SMI_SUCCESS;
    int tok = -1;
    if (prof_enabled()) SMI_TRY(prof_begin(SMI_PROF_GEMV, s, &tok));
    const dim3 block(64 * kGemvWaves);
    if (m <= kSplitMaxCols && gemv_variant() != 1) {
        const int v = gemv_variant();
        if (v == 2) launch_split<1>(A, B, x, y, n, m, lda, alpha, beta, s);
        else if (v == 3) launch_split<4>(A, B, x, y, n, m, lda, alpha, beta, s);
        else launch_split<2>(A, B, x, y, n, m, lda, alpha, beta, s);
        SMI_HIP_CHECK(hipGetLastError());
        if (tok >= 0) SMI_TRY(prof_end(tok, s));
        return SMI_SUCCESS;
    }
    const dim3 grid((n + kGemvWaves - 1) / kGemvWaves);
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
