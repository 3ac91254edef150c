// stencilk.h -- K Jacobi steps per pass over HBM (deep temporal blocking).
//
// Same per-cell arithmetic as every other stencil kernel here
// (stencil_smi.cl:153-156, global-edge cells copied per :143-151), applied K
// times inside one streaming pass.  Each wave owns a 256-column window of the
// input and walks it down a block of rows; every incoming input row advances
// a pipeline of K levels and only level K is stored.  The window is 256 input
// columns wide and stores the central 256-2KC (KC = K rounded up to whole
// float4 lanes): each level loses one valid column per side, so adjacent
// windows overlap by 2KC columns instead of fetching strip-edge extras (no
// cross-lane broadcasts).  HBM traffic per pass is that of a single step, so
// the algorithmic 8 B/cell/step move up to K times faster.
//
// Software pipeline (one input row per step, pinned by sched_barrier):
//   * the input rows stream into a per-wave LDS ring of D+3 rows (1 KiB
//     each) by LDS-DMA (global_load_lds_dwordx4: no VGPR holds a row in
//     flight).  Step t issues the DMA of row t+D into the slot of row t-3
//     (dead), waits with an exact s_waitcnt vmcnt for row t's DMA and reads
//     it into registers (ds_read_b128), evaluates the levels and stores
//     level K.  The barrier after every step keeps the compiler from sinking
//     the loads to their use (the round-1 kernel issued each batch right
//     before it was consumed, so every wave waited a full HBM latency per
//     batch).
//   * levels 0..K-1 keep their last three rows in a 3-slot register ring
//     (slot = t mod 3); the loop is unrolled over D+3 rows (a multiple of 3),
//     so every slot index is a compile-time constant and no value moves
//     between registers.
//   * the levels of a step form G independent groups (SweepK::levels): group
//     g evaluates input t - g, so the scheduler interleaves G dependency
//     chains of K/G levels instead of stalling on one chain of K.
//   * the first 2K+G steps prime the pipeline, unrolled with compile-time
//     row indices; level l is evaluated only from input row 2l on.
//
// Edges.  The fast kernel has ONE code path: windows whose cone never meets
// a global edge row or column.  The host keeps the interior rectangle K rows
// / KC columns clear of every side and computes those bands with the ring
// kernel (stencil_ringk.hip) beside the sweep, on the high-priority comm
// stream; tiles too small for that take the FULL kernel (per-cell copy
// selects).  Every extra code path in the fast kernel costs registers for
// all waves: the register allocator handles a kernel body holding several
// variants worse than each alone (197 VGPRs at K = 12 for variants of <= 160
// each), and a per-lane select on one half of a packed pair costs 50-80
// VGPRs -- each time a wave per SIMD.
#pragma once

#include <type_traits>

#include "stencil_common.h"

namespace smi {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// lane i <- lane i-1 / i+1 (DPP wave_shr:1 / wave_shl:1).  Lanes 0 / 63 get
// whatever the hardware leaves (they only ever feed non-stored columns), so
// the destination needs no initialisation.
__device__ __forceinline__ float shr1_any(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float shl1_any(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x130, 0xf, 0xf, true));
}

template <int I, int N, typename F>
__device__ __forceinline__ void static_for_from(F &f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for_from<I + 1, N>(f);
    }
}
// f(integral_constant<0>) ... f(integral_constant<N-1>), fully unrolled
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    static_for_from<0, N>(f);
}

constexpr int pmod(int a, int m) { return ((a % m) + m) % m; }

#ifndef SMI_SWEEPK_D
#define SMI_SWEEPK_D 6
#endif
#ifndef SMI_SWEEPK_GROUPS
#define SMI_SWEEPK_GROUPS 2  // independent level groups per step (see SweepK::levels)
#endif
#ifndef SMI_SWEEPK_LOAD_AUX
#define SMI_SWEEPK_LOAD_AUX 0  // cache policy of the row DMAs (2 = nt)
#endif
constexpr int SWEEPK_D = SMI_SWEEPK_D;  // input rows loaded ahead of the row being evaluated

// s_waitcnt vmcnt(N) / a ds_read_b128 the compiler cannot see.  The LDS
// ring is filled by LDS-DMA, which the compiler's wait-count pass treats as
// aliasing every LDS read (it would put vmcnt(0) before each one and drain
// the whole prefetch); the read is therefore inline asm that waits for its
// own data (lgkmcnt(0)), and the DMA waits are placed by hand with exact
// counts (see SweepK::vm_count).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt is a 6-bit counter");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ float4 lds_read_b128(unsigned addr) {
    float4 v;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return v;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const float *base, int nbytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(base), (short)0, nbytes, 0x00020000);
}

template <int K, int D, int G_MAX, bool FULL>
struct SweepK {
    static_assert(K >= 1 && K <= 12, "1 <= K <= 12");
    static_assert(D % 3 == 0, "the input ring must be a multiple of the 3-slot level rings");
    static constexpr int LL = (K + 3) / 4;  // lanes per window side that never store
    static constexpr int KC = 4 * LL;       // window apron in columns (>= K)
    static constexpr int G = K < G_MAX ? K : G_MAX;  // independent level groups per step
    static constexpr int PRO = 2 * K + G;   // prologue steps (the last stores the first output row)
    // level L belongs to group gof(L); group g evaluates input t - g in step t
    static constexpr int gof(int L) { return (L - 1) * G / K; }
    static constexpr int R0 = D + 3;        // LDS input-row ring (rows)

    const float *__restrict__ in;
    float *__restrict__ out;
    int rows, cols;
    int o0, o1;       // output rows of this wave
    int r_begin;      // input row of step 0 (o0 - K)
    unsigned loff;    // byte offset of this lane's first load column (clamped into the row)
    float4 *ring;     // this wave's LDS ring: R0 rows of 64 float4
    unsigned rd;      // LDS byte address of this lane's float4 in ring row 0
    int voff;         // store byte offset in the row (out of range: no store)
    int row_bytes;
    bool copyL, copyR, gT, gB;  // FULL kernel only
    float4 W[K][3];   // levels 0..K-1 (level 0 = input rows), slot = t mod 3

    // the level-L row produced by input t, where PH == t (mod R0)
    template <int L, int PH>
    __device__ __forceinline__ float4 &at() {
        return W[L][pmod(PH, 3)];
    }

    // Issue the LDS-DMA of input row t into ring slot t mod R0 (PH == t).
    template <int PH>
    __device__ __forceinline__ void dma(int t) const {
        const int r = __builtin_amdgcn_readfirstlane(min(max(r_begin + t, 0), rows - 1));
        const char *row = reinterpret_cast<const char *>(in + (size_t)r * cols);
        __builtin_amdgcn_global_load_lds(row + loff, ring + pmod(PH, R0) * 64, 16, 0, SMI_SWEEPK_LOAD_AUX);
    }

    // Vector-memory ops issued after the DMA of input t, at the point where
    // step t waits for it: the D DMAs of inputs t+1..t+D and the stores of
    // steps t-D..t-1 (the first store is issued in step PRO-1).  vmcnt
    // counts loads, DMAs and stores together, in issue order.
    static constexpr int vm_count(int t) {
        const int st = t - (PRO - 1) < 0 ? 0 : (t - (PRO - 1) > D ? D : t - (PRO - 1));
        return D + st;
    }

    template <int PH>
    __device__ __forceinline__ float4 ring_read() const {
        return lds_read_b128(rd + (unsigned)(pmod(PH, R0) * 1024));
    }

    // one cell-step on four columns: row i of the output, N / C / S rows
    __device__ __forceinline__ float4 step(int i, const float4 &n, const float4 &c, const float4 &s) const {
        const float w = shr1_any(c.w);
        const float e = shl1_any(c.x);
        float4 o;
        if constexpr (!FULL) {
            // ((S + W) + E) element-wise, then (+ N) and (x 0.25) on packed
            // pairs (v_pk_add_f32 / v_pk_mul_f32: same IEEE single-precision
            // round-to-nearest results as the scalar ops, never contracted)
            f32x2 sw01 = {__fadd_rn(s.x, w), __fadd_rn(s.y, c.x)};
            f32x2 sw23 = {__fadd_rn(s.z, c.y), __fadd_rn(s.w, c.z)};
            f32x2 swe01 = {__fadd_rn(sw01.x, c.y), __fadd_rn(sw01.y, c.z)};
            f32x2 swe23 = {__fadd_rn(sw23.x, c.w), __fadd_rn(sw23.y, e)};
            const f32x2 q = {0.25f, 0.25f};
            const f32x2 o01 = (swe01 + f32x2{n.x, n.y}) * q;
            const f32x2 o23 = (swe23 + f32x2{n.z, n.w}) * q;
            o.x = o01.x;
            o.y = o01.y;
            o.z = o23.x;
            o.w = o23.y;
        } else {
            // per-cell copy selects for the global edge rows / columns
            o.x = jacobi(s.x, w, c.y, n.x);
            o.y = jacobi(s.y, c.x, c.z, n.y);
            o.z = jacobi(s.z, c.y, c.w, n.z);
            o.w = jacobi(s.w, c.z, e, n.w);
            const bool rcopy = (i == 0 && gT) || (i == rows - 1 && gB);
            o.x = (rcopy || copyL) ? c.x : o.x;
            o.y = rcopy ? c.y : o.y;
            o.z = rcopy ? c.z : o.z;
            o.w = (rcopy || copyR) ? c.w : o.w;
        }
        return o;
    }

    // level L (1..K) at input u (PH == u mod R0) from the level L-1 rows of
    // inputs u-2 (N), u-1 (C), u (S)
    template <int L, int PH>
    __device__ __forceinline__ float4 level(int u) {
        return step(r_begin + u - L, at<L - 1, PH - 2>(), at<L - 1, PH - 1>(), at<L - 1, PH>());
    }

    // Branch-free predicated store of the level-K row produced by input u:
    // a buffer store through a per-row descriptor whose record count is the
    // row's bytes (0 for rows outside [o0, o1)); lanes that must not store
    // carry an offset beyond it and the hardware range check drops them.
    __device__ __forceinline__ void store_row(int u, const float4 &v) const {
        const int j = o0 + (u - 2 * K);
        const int jj = __builtin_amdgcn_readfirstlane(min(max(j, 0), rows - 1));
        const int nrec = __builtin_amdgcn_readfirstlane(j < o1 ? row_bytes : 0);
        const u32x4 d = {__builtin_bit_cast(unsigned int, v.x), __builtin_bit_cast(unsigned int, v.y),
                         __builtin_bit_cast(unsigned int, v.z), __builtin_bit_cast(unsigned int, v.w)};
        __builtin_amdgcn_raw_buffer_store_b128(d, row_rsrc(out + (size_t)jj * cols, nrec), voff, 0, 2 /* nt */);
    }

    // The K levels of step t.  Level L of group g evaluates input u = t - g
    // (its output row lags one more row per group), so the G groups of a
    // step read only rows earlier steps wrote: G independent dependency
    // chains of K/G levels for the scheduler to interleave, instead of one
    // chain of K (a wave issuing a single chain stalls on every dependent
    // add).  Groups run last to first in program order: a group reads its
    // predecessor's oldest row before the predecessor overwrites that slot.
    // PRO_T >= 0: prologue step (compile-time t), levels only from input 2L.
    template <int PH, int PRO_T>
    __device__ __forceinline__ float4 levels(int t) {
        float4 vk = make_float4(0.f, 0.f, 0.f, 0.f);
        static_for<G>([&](auto GI) {
            constexpr int g = G - 1 - GI;
            static_for<K>([&](auto I) {
                constexpr int L = I + 1;
                if constexpr (gof(L) == g && (PRO_T < 0 || PRO_T - g >= 2 * L)) {
                    const float4 v = level<L, PH - g>(t - g);
                    if constexpr (L < K)
                        at<L, PH - g>() = v;
                    else
                        vk = v;
                }
            });
        });
        return vk;
    }

    // one steady-state step t (PH == t mod R0, VMC = vm_count(t))
    template <int PH, int VMC>
    __device__ __forceinline__ void advance(int t) {
        dma<PH + D>(t + D);  // into the slot of input t-3
        wait_vmcnt<VMC>();
        at<0, PH>() = ring_read<PH>();
        const float4 v = levels<PH, -1>(t);
        store_row(t - (G - 1), v);
    }

    __device__ __forceinline__ void run() {
        static_for<D>([&](auto U) { dma<U>(U); });
        // prologue: steps 0 .. PRO-1, compile-time indices
        static_for<PRO>([&](auto T) {
            constexpr int t = T;
            dma<t + D>(t + D);
            wait_vmcnt<vm_count(t)>();
            at<0, t>() = ring_read<t>();
            const float4 v = levels<t, t>(t);
            if constexpr (t == PRO - 1) store_row(t - (G - 1), v);
            __builtin_amdgcn_sched_barrier(0);
        });
        // steady state: R0 steps per iteration (slot phases repeat).  No
        // per-step guard: a conditional step would keep every ring slot's
        // old value alive across it (phis), i.e. three rows per level instead
        // of two.  A block whose height is not 1 mod R0 runs up to R0-1 extra
        // steps whose stores the row descriptor drops (the host picks heights
        // of 1 mod R0: n_in - PRO = height - 1).  The first iteration is
        // peeled: its wait counts still ramp up with the stores issued so far.
        const int n_in = (o1 - o0) + 2 * K + G - 1;  // steps
        if (PRO < n_in) {
            static_for<R0>([&](auto V) {
                advance<PRO + V, vm_count(PRO + V)>(PRO + V);
                __builtin_amdgcn_sched_barrier(0);
            });
        }
        for (int base = PRO + R0; base < n_in; base += R0) {
            static_for<R0>([&](auto V) {
                advance<PRO + V, 2 * D>(base + V);
                __builtin_amdgcn_sched_barrier(0);
            });
        }
        wait_vmcnt<0>();  // no DMA may land in LDS after the wave has exited
    }
};

// FULL = false: the fast kernel (the host guarantees no window's cone meets
// a global edge row or column).  FULL = true: per-cell copy selects for the
// global edges (small tiles); its own kernel, so its register peak never sets
// the fast kernel's occupancy.
template <int K, bool FULL>
__global__ __launch_bounds__(256) void sweepk_kernel(SweepKArgs a, int nstrips, int nrb, int ht) {
    using S = SweepK<K, SWEEPK_D, SMI_SWEEPK_GROUPS, FULL>;
    constexpr int SW = 256 - 2 * S::KC;  // output columns per window
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int lane = threadIdx.x & 63;
    const int task = __builtin_amdgcn_readfirstlane(lb * 4 + (int)(threadIdx.x >> 6));
    const int rb = task / nstrips;
    const int strip = task - rb * nstrips;
    if (rb >= nrb) return;  // wave-uniform

    __shared__ float4 lds_ring[4][S::R0][64];  // one ring per wave of the workgroup
    S w;
    w.ring = &lds_ring[threadIdx.x >> 6][0][0];
    w.rd = (unsigned)(uintptr_t)(w.ring + lane);
    w.in = a.in;
    w.out = a.out;
    w.rows = a.rows;
    w.cols = a.cols;
    // row blocks of ht rows (the last one shorter)
    w.o0 = a.row_lo + rb * ht;
    w.o1 = min(w.o0 + ht, a.row_hi);
    const int cs = a.col_lo + strip * SW;
    const int cb = cs - S::KC + 4 * lane;
    const int cl = min(max(cb, 0), a.cols - 4);
    const bool st = lane >= S::LL && lane < 64 - S::LL && cb < a.col_hi;
    w.loff = (unsigned)cl * 4u;
    w.row_bytes = a.cols * 4;
    w.voff = st ? cb * 4 : 0x7ffffff0;
    w.copyL = a.gL && cb == 0;
    w.copyR = a.gR && cb + 4 == a.cols;
    w.gT = a.gT;
    w.gB = a.gB;
    w.r_begin = w.o0 - K;
    w.run();
}

template <int K>
int sweepk_launch_impl(const SweepKArgs &a, int nstrips, int nrb, int ht, int blocks, bool full, hipStream_t s) {
    if (full)
        hipLaunchKernelGGL((sweepk_kernel<K, true>), dim3(blocks), dim3(256), 0, s, a, nstrips, nrb, ht);
    else
        hipLaunchKernelGGL((sweepk_kernel<K, false>), dim3(blocks), dim3(256), 0, s, a, nstrips, nrb, ht);
    SMI_HIP_CHECK(hipGetLastError());
    return SMI_SUCCESS;
}

// resident waves of the fast sweepk<K> on the current device (one round of the grid)
template <int K>
int sweepk_resident_impl() {
    static int cached[64] = {};  // per device
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    if (cached[dev]) return cached[dev];
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, sweepk_kernel<K, false>, 256, 0) != hipSuccess)
        return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cached[dev] = per_cu * cus * 4;
    return cached[dev];
}

}  // namespace smi

// One translation unit per K (stencilk_k<K>.hip) so the ten instantiations
// compile in parallel.
#define SMI_SWEEPK_INSTANCE(K)                                                                         \
    namespace smi {                                                                                    \
    int sweepk_launch_k##K(const SweepKArgs &a, int nstrips, int nrb, int ht, int blocks, bool full,  \
                           hipStream_t s) {                                                            \
        return sweepk_launch_impl<K>(a, nstrips, nrb, ht, blocks, full, s);                            \
    }                                                                                                  \
    int sweepk_resident_k##K() { return sweepk_resident_impl<K>(); }                                   \
    }
