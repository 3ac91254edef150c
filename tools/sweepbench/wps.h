// wps.h -- experiment: wave-pipelined K-step sweep (K = P x L steps per HBM
// pass).  A workgroup of P waves owns one 256-column window of one row
// block; wave p evaluates levels pL+1 .. (p+1)L of every input row and hands
// its top level to wave p+1 through a two-slot LDS ring, so each wave keeps
// only L levels in registers (3-slot rings, as in stencilk.h) and a pass
// covers P times more steps than one wave's register file allows.  Waves
// advance in lockstep, one raw s_barrier per row; wave p runs p rows behind
// wave 0.  Wave 0 streams the input rows from HBM (loads 3 rows ahead), the
// last wave stores level K through per-row buffer descriptors.
//
// Rows before a level's first needed row are evaluated on clamped inputs and
// never reach a stored cell (level l at input t is needed only for t >= 2l).
// EDGE: per-cell copy selects for global edge rows / columns (blocks and
// strips that touch them); the plain variant has none.
#pragma once

#include <type_traits>

#include "stencil_common.h"

namespace smi {

typedef float wf32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int wu32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float wshr1(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float wshl1(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x130, 0xf, 0xf, true));
}

template <int I, int N, typename F>
__device__ __forceinline__ void wfor_from(F &f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        wfor_from<I + 1, N>(f);
    }
}
template <int N, typename F>
__device__ __forceinline__ void wfor(F &&f) {
    wfor_from<0, N>(f);
}

__device__ __forceinline__ void wps_barrier() {
    // LDS writes of this step done, then the workgroup barrier; the memory
    // clobber keeps the compiler from moving LDS accesses across it
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

#ifndef WPS_BATCH
#define WPS_BATCH 3  // rows per barrier interval (1 or 3)
#endif
#ifndef WPS_APRON_LANES
#define WPS_APRON_LANES(K) (((K) + 3) / 4)
#endif

template <int P, int L, bool EDGE>
struct Wps {
    static constexpr int K = P * L;
    static constexpr int LL = WPS_APRON_LANES(K);
    static constexpr int KC = 4 * LL;

    const float *__restrict__ in;
    float *__restrict__ out;
    int rows, cols;
    int o0, o1, r_begin;
    int cl, voff, row_bytes;
    bool copyL, copyR, gT, gB;
    float4 W[L][3];   // local level 0 (= global level pL, the input) .. L-1
    float4 A[3];      // wave 0: input rows in flight (3 ahead)
    float4 *ring;     // [P-1][2][64] float4

    __device__ __forceinline__ float4 ld(int t) const {
        const int r = min(max(r_begin + t, 0), rows - 1);
        return *reinterpret_cast<const float4 *>(in + (size_t)r * cols + cl);
    }

    __device__ __forceinline__ float4 step(int i, const float4 &n, const float4 &c, const float4 &s) const {
        const float w = wshr1(c.w);
        const float e = wshl1(c.x);
        wf32x2 sw01 = {__fadd_rn(s.x, w), __fadd_rn(s.y, c.x)};
        wf32x2 sw23 = {__fadd_rn(s.z, c.y), __fadd_rn(s.w, c.z)};
        wf32x2 swe01 = {__fadd_rn(sw01.x, c.y), __fadd_rn(sw01.y, c.z)};
        wf32x2 swe23 = {__fadd_rn(sw23.x, c.w), __fadd_rn(sw23.y, e)};
        const wf32x2 q = {0.25f, 0.25f};
        const wf32x2 o01 = (swe01 + wf32x2{n.x, n.y}) * q;
        const wf32x2 o23 = (swe23 + wf32x2{n.z, n.w}) * q;
        float4 o;
        o.x = o01.x;
        o.y = o01.y;
        o.z = o23.x;
        o.w = o23.y;
        if constexpr (EDGE) {
            const bool rcopy = (i == 0 && gT) || (i == rows - 1 && gB);
            o.x = (rcopy || copyL) ? c.x : o.x;
            o.y = rcopy ? c.y : o.y;
            o.z = rcopy ? c.z : o.z;
            o.w = (rcopy || copyR) ? c.w : o.w;
        }
        return o;
    }

    __device__ __forceinline__ void store_row(int t, const float4 &v) const {
        const int j = o0 + (t - 2 * K);
        const int jj = __builtin_amdgcn_readfirstlane(min(max(j, 0), rows - 1));
        const int nrec = __builtin_amdgcn_readfirstlane((j >= o0 && j < o1) ? row_bytes : 0);
        __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(out + (size_t)jj * cols, (short)0, nrec, 0x00020000);
        const wu32x4 d = {__builtin_bit_cast(unsigned int, v.x), __builtin_bit_cast(unsigned int, v.y),
                          __builtin_bit_cast(unsigned int, v.z), __builtin_bit_cast(unsigned int, v.w)};
        __builtin_amdgcn_raw_buffer_store_b128(d, rs, voff, 0, 2);
    }

    // one input row t of wave `p` (compile-time slot phase PH = t mod 3)
    template <int PH, int ROLE>  // ROLE: 0 first wave, 1 middle, 2 last (P == 1: 3 = both)
    __device__ __forceinline__ void row(int t, int p, int lane) {
        float4 x;
        // ring slot of row t: 2 batches of 3 rows per wave boundary
        const int slot = (((t / 3) & 1) * 3 + PH) * 64 + lane;
        if constexpr (ROLE == 0 || ROLE == 3) {
            x = A[PH];
            A[PH] = ld(t + 3);
        } else {
            x = ring[(p - 1) * 6 * 64 + slot];
        }
        W[0][PH] = x;
        float4 v;
        wfor<L>([&](auto J) {
            constexpr int j = J + 1;
            const int gl = p * L + j;  // global level
            v = step(r_begin + t - gl, W[j - 1][(PH + 1) % 3], W[j - 1][(PH + 2) % 3], W[j - 1][PH]);
            if constexpr (j < L) W[j][PH] = v;
        });
        if constexpr (ROLE == 2 || ROLE == 3)
            store_row(t, v);
        else
            ring[p * 6 * 64 + slot] = v;
#if WPS_BATCH == 1
        wps_barrier();
#endif
    }

    template <int ROLE>
    __device__ __forceinline__ void run(int p, int lane, int n_pad) {
#pragma unroll
        for (int j = 0; j < L; ++j)
#pragma unroll
            for (int k = 0; k < 3; ++k) W[j][k] = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (ROLE == 0 || ROLE == 3)
#pragma unroll
            for (int k = 0; k < 3; ++k) A[k] = ld(k);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // drain: the loop header sees no pending prologue loads
        for (int t = 0; t < n_pad; t += 3) {
            row<0, ROLE>(t, p, lane);
            row<1, ROLE>(t + 1, p, lane);
            row<2, ROLE>(t + 2, p, lane);
#if WPS_BATCH == 3
            wps_barrier();
#endif
        }
    }
};

template <int P, int L, bool EDGE>
__global__ __launch_bounds__(64 * P) void wps_kernel(SweepKArgs a, int nstrips, int nrb) {
    using S = Wps<P, L, EDGE>;
    constexpr int SW = 256 - 2 * S::KC;
    __shared__ float4 ring[(P > 1 ? P - 1 : 1) * 6 * 64];
    const int task = xcd_remap(blockIdx.x, gridDim.x);
    const int rb = task / nstrips;
    const int strip = task - rb * nstrips;
    if (rb >= nrb) return;  // workgroup-uniform
    const int p = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    S w;
    w.ring = ring;
    w.in = a.in;
    w.out = a.out;
    w.rows = a.rows;
    w.cols = a.cols;
    const int out_rows = a.row_hi - a.row_lo;
    w.o0 = a.row_lo + (int)((long)rb * out_rows / nrb);
    w.o1 = a.row_lo + (int)((long)(rb + 1) * out_rows / nrb);
    w.r_begin = w.o0 - S::K;
    const int cs = a.col_lo + strip * SW;
    const int cb = cs - S::KC + 4 * lane;
    w.cl = min(max(cb, 0), a.cols - 4);
    const bool st = lane >= S::LL && lane < 64 - S::LL && cb < a.col_hi;
    w.row_bytes = a.cols * 4;
    w.voff = st ? cb * 4 : 0x7ffffff0;
    w.copyL = a.gL && cb == 0;
    w.copyR = a.gR && cb + 4 == a.cols;
    w.gT = a.gT;
    w.gB = a.gB;
    const int n_in = (w.o1 - w.o0) + 2 * S::K;
    const int n_pad = (n_in + 2) / 3 * 3;
    // every wave executes the same number of barriers: p lead-in (wave p
    // runs one barrier interval = WPS_BATCH rows behind wave p-1), the loop,
    // P-1-p trailing
    for (int k = 0; k < p; ++k) wps_barrier();
    if constexpr (P == 1) {
        w.template run<3>(p, lane, n_pad);
    } else {
        if (p == 0)
            w.template run<0>(p, lane, n_pad);
        else if (p == P - 1)
            w.template run<2>(p, lane, n_pad);
        else
            w.template run<1>(p, lane, n_pad);
    }
    for (int k = p; k < P - 1; ++k) wps_barrier();
}

}  // namespace smi
