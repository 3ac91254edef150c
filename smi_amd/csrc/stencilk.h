// stencilk.h -- K Jacobi steps per pass over HBM (deep temporal blocking).
//
// Same per-cell arithmetic as every other stencil kernel here
// (stencil_smi.cl:153-156, global-edge cells copied per :143-151), applied K
// times inside one streaming pass.  Each wave owns a 256-column window of the
// input and walks it down a block of rows; every incoming input row advances
// a pipeline of K levels (level l lags l rows behind the input) and only
// level K is stored.  The window is 256 input columns wide but stores only
// the central 256-2KC (KC = K rounded up to whole float4 lanes): each level
// loses one valid column per side, so adjacent windows overlap by 2KC
// columns instead of fetching strip-edge extras (no cross-lane broadcasts).
// HBM traffic per pass is that of a single step, so the algorithmic
// 8 B/cell/step move up to K times faster.
//
// Register pipeline.  Level l keeps its last three rows in a 3-slot ring,
// slot = (input row index) mod 3; the loop body covers 6 input rows (two
// batches of 3, each batch's loads issued one batch ahead), so every slot
// index is a compile-time constant and no value is ever moved between
// registers.  The first 2K+1 input rows of a row block prime the pipeline;
// that prologue is unrolled with compile-time row indices and evaluates
// level l only from input row 2l on (the rows it must produce).  Global-edge
// copy rules cost nothing in the loop (ROW_* below); only the strips holding
// column 0 or Y-1 add a per-lane select.
//
// The kernel computes an arbitrary output rectangle [row_lo,row_hi) x
// [col_lo,col_hi) of the tile from input cells within K of it, so it is the
// single-tile sweep (whole tile) and, in multi-rank runs, the interior sweep
// that stays K rows / KC columns clear of every halo-facing side.
//
// Window apron: K >= 9 uses 16 columns (4 lanes) per side, so a window
// stores 224 columns = 7 whole 128-byte lines at a line-aligned offset
// (strip starts are multiples of 224 columns); smaller K keep the minimal
// float4 apron.  Round 2 (tools/sweepbench, 8192^2, K=12, ping-pong): the
// aligned apron + the pre-loop drain + the batch issue barrier run a pass in
// 0.117 ms vs 0.122 ms; the same grid streaming its loads and stores with no
// levels takes 0.106 ms and the levels alone (cache-resident inputs) 0.094
// ms, so the pass is now within ~10 % of its memory floor for this traffic
// (594 MB, 1.1x the 537 MB minimum: window and row-block aprons).
//
// Measured alternative (round 2, tools/sweepbench): an LDS-DMA input ring
// with hand-placed vmcnt waits and independent level groups reached 3
// waves/SIMD at 145 VGPRs but ran 0.129 ms per 12-step pass at 8192^2 vs
// 0.110 ms for this kernel in the same harness (2 waves/SIMD; single-buffer
// timing): the per-step ds_read + sched barriers turned
// the pass issue-stall bound (SQ_WAIT_INST_ANY 2.7x, VALU instructions 1.23x;
// profiles/r02/).
//
// Scaled levels (round 2).  x 0.25 is a power-of-two scaling, and IEEE
// round-to-nearest commutes with power-of-two scaling whenever nothing
// overflows and no rounding happens in the subnormal range.  So level l can
// carry u_l = 4^l v_l: u_l = ((S'+W')+E')+N' over the level-(l-1) values u,
// with no multiply (copied edge cells: u_l = 4 u_{l-1}), and the store
// writes u_K * 4^-K.  This is bit-identical to the reference arithmetic
// when every finite nonzero input of the wave's cone has magnitude in
// [2^-100, 2^101): then every level-l value is a multiple of 2^(-123-2l)
// (>= 2^-147 for l <= 12, so each x 0.25 of the reference order is exact,
// subnormal or not), and |u| < 2^(2K+101) <= 2^125 never overflows; Inf and
// NaN propagate the same either way.  Each wave checks its inputs as they
// stream in (frexp exponents) and a block that fails walks again with the
// exact arithmetic.  The multiply was 2 of the 12 VALU instructions of a
// level step (4 of 16.3 issue-slot units, packed ops at half rate).
#pragma once

#include <type_traits>

#include <hip/hip_ext.h>

#include "stencil_common.h"

#ifndef SMI_SWEEPK_SCALED
#define SMI_SWEEPK_SCALED 1
#endif
// experiment switches (tools/sweepbench builds; the library uses the defaults)
#ifndef SMI_SWEEPK_NT_LOADS
#define SMI_SWEEPK_NT_LOADS 0
#endif
#ifndef SMI_SWEEPK_TASK_ORDER
#define SMI_SWEEPK_TASK_ORDER 0
#endif
#ifndef SMI_SWEEPK_ALT
#define SMI_SWEEPK_ALT 0
#endif

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

// How a wave treats the global edge rows (stencil_smi.cl:143-151: rows 0 and
// X-1 are copied unchanged every step).
//   ROW_NONE  the wave's cone never reaches an edge row: no selects at all.
//   ROW_TOP   the wave's first output row is row 0 (walk downwards).  Row 0
//             of level l is produced at input t = K + l <= 2K, i.e. only in
//             the compile-time prologue, so the copy is a handful of
//             constant-index register moves there -- nothing in the loop.
//   ROW_BOT   the wave's last output row is row X-1: the wave walks UPWARDS
//             (N and S swap roles in the loads, never in the arithmetic
//             order), so row X-1 is again its prologue row t - l = K.
//   ROW_FULL  anything else that touches an edge row (blocks spanning both
//             edges, tiny row blocks from a tuning override): per-cell
//             row selects.
// Column edges add one per-lane select per level step: CE bit 0 for the
// strip holding column 0, bit 1 for the one holding column Y-1 (both only
// when one window spans the whole tile); every other wave runs the plain
// 12-instruction step.
enum { ROW_NONE = 0, ROW_TOP = 1, ROW_BOT = 2, ROW_FULL = 3, ROW_UP = 4 };
// ROW_UP: a ROW_NONE block that walks upwards (alternating walk directions,
// SMI_SWEEPK_ALT): row block rb walks down for even rb and up for odd rb, so
// the 2K apron rows two neighbouring blocks share are read by both at the
// same time (the ends of both walks, or the starts of both) and the second
// read hits L2.  Needs an even number of row blocks (launch_sweepk_ex).
__host__ __device__ constexpr bool walks_up(int row) { return row == ROW_BOT || row == ROW_UP; }

template <int K, int U>
struct SweepK {
    static_assert(K >= SWEEPK_MIN && K <= SWEEPK_MAX, "3 <= K <= 12");
    static_assert(U % 3 == 0, "batch must be a multiple of the 3-slot ring");
    static constexpr int LL = sweepk_apron_lanes(K);  // lanes per window side that never store
    static constexpr int KC = 4 * LL;                  // window apron in columns (>= K)
    static constexpr int PRO = 2 * K + 1;   // prologue input rows (the last one stores the first output row)
    static constexpr bool kScaled = SMI_SWEEPK_SCALED != 0;
    static constexpr int kExpLo = -99, kExpHi = 101;      // frexp exponent range of the scaled walk's inputs
    static constexpr float kUnscale = 1.0f / (float)(1u << (2 * K));  // 4^-K (exact: K <= 12)

    const float *__restrict__ in;
    float *__restrict__ out;
    int rows, cols;
    int o0, o1;       // output rows of this wave
    int r_begin;      // input row of t = 0 (o0 - K walking down, o1 - 1 + K walking up)
    int cl;           // clamped load column of this lane
    int voff;         // store byte offset in the row (out of range: no store)
    int row_bytes;
    bool copyL, copyR, gT, gB;
    float4 W[K][3];   // level 0..K-1, slot = input row index mod 3

    template <bool REV>
    __device__ __forceinline__ float4 ld(int t) const {
        const int r = min(max(REV ? r_begin - t : r_begin + t, 0), rows - 1);
#if SMI_SWEEPK_NT_LOADS
        typedef float V4 __attribute__((ext_vector_type(4)));
        const V4 v = __builtin_nontemporal_load(reinterpret_cast<const V4 *>(in + (size_t)r * cols + cl));
        return make_float4(v.x, v.y, v.z, v.w);
#else
        return *reinterpret_cast<const float4 *>(in + (size_t)r * cols + cl);
#endif
    }

    // One level step of 4 cells per lane.  SC (scaled): the operands carry
    // 4^(l-1) times their level-(l-1) values, so the sum ((S+W)+E)+N is
    // 4^l times the level-l value and the x 0.25 is skipped (copied edge
    // cells are scaled by 4 instead); see "Scaled levels" above.
    template <int ROW, int CE, bool SC>
    __device__ __forceinline__ float4 step(int i, const float4 &n, const float4 &c, const float4 &s) const {
        const float w = shr1_any(c.w);
        const float e = shl1_any(c.x);
        // ((S + W) + E) element-wise, then (+ N) (and x 0.25) on packed
        // pairs (v_pk_add_f32 / v_pk_mul_f32: same IEEE single-precision
        // round-to-nearest results as the scalar ops, never contracted)
        float b0 = __fadd_rn(__fadd_rn(s.x, w), c.y);
        float b1 = __fadd_rn(__fadd_rn(s.y, c.x), c.z);
        float b2 = __fadd_rn(__fadd_rn(s.z, c.y), c.w);
        float b3 = __fadd_rn(__fadd_rn(s.w, c.z), e);
        if constexpr (SC) {
            // opaque: keeps the instruction selector from re-pairing the
            // scalar adds into v_pk_add_f32 with register moves for operands
            asm("" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3));
        }
        f32x2 o01 = f32x2{b0, b1} + f32x2{n.x, n.y};
        f32x2 o23 = f32x2{b2, b3} + f32x2{n.z, n.w};
        if constexpr (!SC) {
            const f32x2 q = {0.25f, 0.25f};
            o01 = o01 * q;
            o23 = o23 * q;
        }
        float4 o;
        o.x = o01.x;
        o.y = o01.y;
        o.z = o23.x;
        o.w = o23.y;
        if constexpr (ROW == ROW_FULL) {
            static_assert(!SC, "ROW_FULL blocks run the exact arithmetic only");
            const bool rcopy = (i == 0 && gT) || (i == rows - 1 && gB);
            o.x = (rcopy || copyL) ? c.x : o.x;
            o.y = rcopy ? c.y : o.y;
            o.z = rcopy ? c.z : o.z;
            o.w = (rcopy || copyR) ? c.w : o.w;
        } else {
            if constexpr (CE & 1) o.x = copyL ? (SC ? c.x * 4.0f : c.x) : o.x;
            if constexpr (CE & 2) o.w = copyR ? (SC ? c.w * 4.0f : c.w) : o.w;
        }
        return o;
    }

    // level l (1..K) at input t from the level l-1 rows of inputs t-2, t-1, t
    // (slots PH+1, PH+2, PH mod 3).  Walking down, input t-2 is the upper
    // row (N) and input t the lower (S); walking up they swap.
    template <int ROW, int CE, bool SC, int PH>
    __device__ __forceinline__ float4 level(int l, int t, const float4 (&P)[3]) const {
        if constexpr (walks_up(ROW))
            return step<ROW, CE, SC>(r_begin - (t - l), P[PH], P[(PH + 2) % 3], P[(PH + 1) % 3]);
        else
            return step<ROW, CE, SC>(r_begin + t - l, P[(PH + 1) % 3], P[(PH + 2) % 3], P[PH]);
    }

    // Scaled-path guard: frexp exponents of every input the wave consumes
    // (0 for zeros, Inf and NaN); the scaled levels are exact when every one
    // lies in [-99, 101] (finite nonzero magnitudes in [2^-100, 2^101)).
    int emin, emax;
    __device__ __forceinline__ void note(const float4 &x) {
        const int e0 = __builtin_amdgcn_frexp_expf(x.x), e1 = __builtin_amdgcn_frexp_expf(x.y);
        const int e2 = __builtin_amdgcn_frexp_expf(x.z), e3 = __builtin_amdgcn_frexp_expf(x.w);
        emin = min(emin, min(e0, e1));
        emax = max(emax, max(e0, e1));
        emin = min(emin, min(e2, e3));
        emax = max(emax, max(e2, e3));
    }

    // Input row t arrives with value x; PH = t mod 3.
    template <int ROW, int CE, bool SC, int PH>
    __device__ __forceinline__ void advance(int t, const float4 &x) {
        W[0][PH] = x;
        if constexpr (SC) note(x);
        float4 v;
        static_for<K>([&](auto L) {
            constexpr int l = L + 1;
            v = level<ROW, CE, SC, PH>(l, t, W[l - 1]);
            if constexpr (l < K) W[l][PH] = v;
        });
        store_row<walks_up(ROW), SC>(t, v);
    }

    // Branch-free predicated store of the level-K row produced by input t:
    // a buffer store through a per-row descriptor whose record count is the
    // row's bytes (0 for rows outside [o0, o1)); lanes that must not store
    // carry an offset beyond it and the hardware range check drops them.  No
    // branch splits the unrolled rows, so the scheduler interleaves their
    // dependency chains.  Nontemporal: the output is not re-read this pass.
    template <bool REV, bool SC>
    __device__ __forceinline__ void store_row(int t, const float4 &vs) const {
        float4 v = vs;
        if constexpr (SC) {  // 4^K u -> u: exact (see "Scaled levels")
            const f32x2 q = {kUnscale, kUnscale};
            const f32x2 a = f32x2{vs.x, vs.y} * q, b = f32x2{vs.z, vs.w} * q;
            v = make_float4(a.x, a.y, b.x, b.y);
        }
        const int j = REV ? o1 - 1 - (t - 2 * K) : o0 + (t - 2 * K);
        const bool in_block = REV ? j >= o0 : j < o1;
        const int jj = __builtin_amdgcn_readfirstlane(min(max(j, 0), rows - 1));
        const int nrec = __builtin_amdgcn_readfirstlane(in_block ? row_bytes : 0);
        __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(out + (size_t)jj * cols, (short)0, nrec, 0x00020000);
        const u32x4 d = {__builtin_bit_cast(unsigned int, v.x), __builtin_bit_cast(unsigned int, v.y),
                         __builtin_bit_cast(unsigned int, v.z), __builtin_bit_cast(unsigned int, v.w)};
        __builtin_amdgcn_raw_buffer_store_b128(d, rs, voff, 0, 2 /* nt */);
    }

    // Walks the block; returns false (wave-uniform) when SC and some input
    // left the range where the scaled levels are exact -- the caller then
    // walks the block again with SC = false.
    template <int ROW, int CE, bool SC>
    __device__ __forceinline__ bool run() {
        constexpr bool REV = walks_up(ROW);
        emin = 0;
        emax = 0;
        // prologue: input rows 0 .. 2K, compile-time indices; level l starts
        // at input 2l (the first row it must produce)
        static_for<PRO>([&](auto T) {
            constexpr int t = T;
            W[0][t % 3] = ld<REV>(t);
            if constexpr (SC) note(W[0][t % 3]);
            float4 v;
            static_for<K>([&](auto L) {
                constexpr int l = L + 1;
                if constexpr (t >= 2 * l) {
                    v = level<ROW, CE, SC, t % 3>(l, t, W[l - 1]);
                    // the edge row (0 walking down, X-1 walking up) is input t - l == K
                    if constexpr ((ROW == ROW_TOP || ROW == ROW_BOT) && t - l == K) {
                        v = W[l - 1][(t + 2) % 3];
                        if constexpr (SC) v = make_float4(v.x * 4.0f, v.y * 4.0f, v.z * 4.0f, v.w * 4.0f);
                    }
                    if constexpr (l < K) W[l][t % 3] = v;
                }
            });
            if constexpr (t == 2 * K) store_row<REV, SC>(t, v);
        });
        // steady state: 2U input rows per iteration, loads one batch ahead
        const int n_in = (o1 - o0) + 2 * K;
        float4 A[U], B[U];
#pragma unroll
        for (int u = 0; u < U; ++u) A[u] = ld<REV>(PRO + u);
        // Drain before the loop.  Without it the wait-count pass merges the
        // loads pending from the prologue into the loop header's state and
        // waits there for the store issued a few instructions earlier (a full
        // store round trip per iteration); with it every wait in the loop
        // targets a load or store issued >= 2 rows of work before.
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
        for (int t = PRO; t < n_in; t += 2 * U) {
#pragma unroll
            for (int u = 0; u < U; ++u) B[u] = ld<REV>(t + U + u);
            __builtin_amdgcn_sched_barrier(0);  // issue the batch here, a whole batch ahead of its use
            static_for<U>([&](auto V) {
                constexpr int ph = (PRO + V) % 3;
                advance<ROW, CE, SC, ph>(t + V, A[V]);
            });
            if (t + U >= n_in) break;  // uniform
#pragma unroll
            for (int u = 0; u < U; ++u) A[u] = ld<REV>(t + 2 * U + u);
            __builtin_amdgcn_sched_barrier(0);
            static_for<U>([&](auto V) {
                constexpr int ph = (PRO + U + V) % 3;
                advance<ROW, CE, SC, ph>(t + U + V, B[V]);
            });
        }
        if constexpr (SC) {
            const bool bad = emin < kExpLo || emax > kExpHi;
            if (__builtin_amdgcn_ballot_w64(bad) != 0) {
                // the exact walk rewrites this block; its stores land after
                // the scaled walk's (same wave, drained first)
                __builtin_amdgcn_s_waitcnt(0x0F70);
                return false;
            }
        }
        return true;
    }

    // scaled walk first (SMI_SWEEPK_SCALED, default on), the exact walk for
    // blocks whose inputs leave its range
    template <int ROW, int CE>
    __device__ __forceinline__ void go() {
        if constexpr (kScaled && ROW != ROW_FULL) {
            if (run<ROW, CE, true>()) return;
        }
        run<ROW, CE, false>();
    }
};

// The interior task of one wave: row block rb of strip `strip`.
template <int K>
__device__ __forceinline__ void sweepk_task(const SweepKArgs &a, int strip, int rb, int nrb, int lane) {
    using S = SweepK<K, 3>;
    constexpr int SW = 256 - 2 * S::KC;  // output columns per window
    S w;
    w.in = a.in;
    w.out = a.out;
    w.rows = a.rows;
    w.cols = a.cols;
    // balanced row blocks: every block of a tall rectangle has >= ht/2 rows
    const int out_rows = a.row_hi - a.row_lo;
    w.o0 = a.row_lo + (int)((long)rb * out_rows / nrb);
    w.o1 = a.row_lo + (int)((long)(rb + 1) * out_rows / nrb);
    // strips start at whole 128-byte lines (col_lo rounded down to 32
    // columns): a multi-rank interior starts KC columns in, and windows
    // stored from there would straddle a line at both ends of every row
    const int cs = (a.col_lo & ~31) + strip * SW;
    const int cb = cs - S::KC + 4 * lane;
    w.cl = min(max(cb, 0), a.cols - 4);
    const bool st = lane >= S::LL && lane < 64 - S::LL && cb >= a.col_lo && cb < a.col_hi;
    w.row_bytes = a.cols * 4;
    w.voff = st ? cb * 4 : 0x7ffffff0;
    w.copyL = a.gL && cb == 0;
    w.copyR = a.gR && cb + 4 == a.cols;
    w.gT = a.gT;
    w.gB = a.gB;
    // rows any level touches: [o0 - 2K, o1 + K + 5); columns: [cs - KC, cs - KC + 256)
    const bool touchT = a.gT && w.o0 - 2 * K <= 0;
    const bool touchB = a.gB && w.o1 + K + 6 >= a.rows;
    const int ce = ((a.gL && cs - S::KC <= 0) ? 1 : 0) | ((a.gR && cs - S::KC + 256 >= a.cols) ? 2 : 0);
    int row = ROW_NONE;
    if (touchT && !touchB && w.o0 == 0)
        row = ROW_TOP;
    else if (touchB && !touchT && w.o1 == a.rows)
        row = ROW_BOT;
    else if (touchT || touchB)
        row = ROW_FULL;
#if SMI_SWEEPK_ALT
    if (row == ROW_NONE && (rb & 1)) row = ROW_UP;
#endif
    w.r_begin = walks_up(row) ? w.o1 - 1 + K : w.o0 - K;
    switch (row * 4 + ce) {
    case 0: w.template go<ROW_NONE, 0>(); break;
    case 1: w.template go<ROW_NONE, 1>(); break;
    case 2: w.template go<ROW_NONE, 2>(); break;
    case 3: w.template go<ROW_NONE, 3>(); break;
    case 4: w.template go<ROW_TOP, 0>(); break;
    case 5: w.template go<ROW_TOP, 1>(); break;
    case 6: w.template go<ROW_TOP, 2>(); break;
    case 7: w.template go<ROW_TOP, 3>(); break;
    case 8: w.template go<ROW_BOT, 0>(); break;
    case 9: w.template go<ROW_BOT, 1>(); break;
    case 10: w.template go<ROW_BOT, 2>(); break;
    case 11: w.template go<ROW_BOT, 3>(); break;
#if SMI_SWEEPK_ALT
    case 16: w.template go<ROW_UP, 0>(); break;
    case 17: w.template go<ROW_UP, 1>(); break;
    case 18: w.template go<ROW_UP, 2>(); break;
    case 19: w.template go<ROW_UP, 3>(); break;
#endif
    default: w.template go<ROW_FULL, 3>(); break;
    }
}

// experiment switch (tools/sweepbench builds): waves per SIMD the register
// allocation must allow (amdgpu_waves_per_eu); the library uses the default
#ifdef SMI_SWEEPK_WPE
#define SMI_SWEEPK_WPE_ATTR __attribute__((amdgpu_waves_per_eu(SMI_SWEEPK_WPE, SMI_SWEEPK_WPE)))
#else
#define SMI_SWEEPK_WPE_ATTR
#endif

template <int K>
__global__ __launch_bounds__(256) SMI_SWEEPK_WPE_ATTR void sweepk_kernel(SweepKArgs a, int nstrips, int nrb) {
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int lane = threadIdx.x & 63;
    const int task = __builtin_amdgcn_readfirstlane(lb * 4 + (int)(threadIdx.x >> 6));
#if SMI_SWEEPK_TASK_ORDER == 1  // experiment: consecutive tasks walk consecutive row blocks of one strip
    const int strip = task / nrb;
    const int rb = task - strip * nrb;
    if (strip >= nstrips) return;
#else
    const int rb = task / nstrips;
    const int strip = task - rb * nstrips;
#endif
    if (rb >= nrb) return;  // wave-uniform
    sweepk_task<K>(a, strip, rb, nrb, lane);
}

template <int K>
int sweepk_launch_impl(const SweepKArgs &a, int nstrips, int nrb, int blocks, hipStream_t s, hipEvent_t start,
                       hipEvent_t stop) {
    if (start || stop)  // events carried by the dispatch itself (no marker packets around it)
        hipExtLaunchKernelGGL((sweepk_kernel<K>), dim3(blocks), dim3(256), 0, s, start, stop, 0, a, nstrips, nrb);
    else
        hipLaunchKernelGGL((sweepk_kernel<K>), dim3(blocks), dim3(256), 0, s, a, nstrips, nrb);
    SMI_HIP_CHECK(hipGetLastError());
    return SMI_SUCCESS;
}

// resident waves of sweepk<K> on the current device (one round of the grid)
template <int K>
int sweepk_resident_impl() {
    static int cached[64] = {};  // per device
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    if (cached[dev]) return cached[dev];
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, sweepk_kernel<K>, 256, 0) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cached[dev] = per_cu * cus * 4;
    return cached[dev];
}

}  // namespace smi

// One translation unit per K (stencilk_k<K>.hip) so the ten instantiations
// compile in parallel.
#define SMI_SWEEPK_INSTANCE(K)                                                                           \
    namespace smi {                                                                                      \
    int sweepk_launch_k##K(const SweepKArgs &a, int nstrips, int nrb, int blocks, hipStream_t s,         \
                           hipEvent_t start, hipEvent_t stop) {                                          \
        return sweepk_launch_impl<K>(a, nstrips, nrb, blocks, s, start, stop);                           \
    }                                                                                                    \
    int sweepk_resident_k##K() { return sweepk_resident_impl<K>(); }                                     \
    }
