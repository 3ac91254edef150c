// stencild.h -- deep K-step sweep: a rotating two-row register ring.
//
// Same cell arithmetic as every stencil kernel here (stencil_smi.cl:153-156,
// global-edge cells copied per :143-151), K steps per pass over HBM, and the
// same wave geometry as stencilk.h (a wave = a 256-column window walking a
// row block, float4 per lane, W/E neighbours by DPP, scaled levels under a
// per-wave exactness guard).  What changes is the register pipeline.
//
// stencilk.h keeps three rows per level (slot = input row mod 3): 12 K
// VGPRs, so K = 12 needs 248 VGPRs (2 waves/SIMD) and K > 12 does not fit.
// Level l at input t needs the level-(l-1) rows of inputs t-2, t-1, t; the
// oldest of them dies as level l is formed, and that is where the new level-l
// row goes.  So the state is two rows per level (A_l older, B_l newer) plus
// the input row x: 2K + 1 float4.  Input t: level l = f(A_{l-1}, B_{l-1},
// new_{l-1}) lands in A_{l-1}'s register; the level-K row is stored and its
// register is free.  Named by position, every register moves one position
// up per input row around one cycle, so the position -> register map after
// j rows is p -> (p - j) mod N, compile-time inside an unrolled body.
//
// Loads join the same cycle: row t + D is loaded at row t into the register
// freed at the end of row t-1 and travels D positions before it is x, so the
// cycle has N = 2K + D + 1 positions (D in flight, x, then B_l / A_l of each
// level), a loop body of N rows leaves the rotation where it found it, and
// no register is ever copied.
//
// Scaled levels (see stencilk.h): level l carries 4^l v_l.  Exact when every
// finite nonzero input of the wave's cone has magnitude in [2^lo, 2^hi) with
//   level-l values multiples of 2^(lo-23-2l) >= 2^-147 for l < K:  lo >= 2K - 126,
//   |u_K| < 4^K 2^hi <= 2^127:                                   hi <= 127 - 2K,
// i.e. frexp exponents in [2K - 125 + 1, 127 - 2K - 1] (one spare binade at
// each end; K = 12 gives [-100, 102] vs stencilk.h's [-99, 101]).  A wave
// whose inputs leave that range walks its block again with the exact
// arithmetic (x 0.25 per level), as in stencilk.h.
#pragma once

#include "stencilk.h"

namespace smi {

// DeepGeom<K>: apron lanes per window side (KC = 4 LL >= K columns) and the
// rows loaded ahead D.
template <int K>
struct DeepGeom {
#ifdef SMI_DEEP_LL
    static constexpr int LL = SMI_DEEP_LL;
#else
    static constexpr int LL = (K + 3) / 4;
#endif
#ifdef SMI_DEEP_PAIR
    static constexpr bool PAIR = SMI_DEEP_PAIR;
#else
    // rows in interleaved pairs (SweepD::pair): off -- 1.5 % faster in the
    // interior-only timing variant at K = 20 with D = 7, 2.4 % slower in the
    // full kernel (236 vs 220 VGPRs; tools/deepbench interleaved A/B)
    static constexpr bool PAIR = false;
#endif
#ifdef SMI_DEEP_D
    static constexpr int D = SMI_DEEP_D;
#else
    // odd (the cycle 2K + D + 1 splits into pairs of rows); K <= 16 keeps 3
    // to stay at 3 waves/SIMD, the pairs of the deeper K want more rows in
    // flight (a pair issues its second row's load late)
    static constexpr int D = PAIR ? 7 : 3;
#endif
};

template <int K>
struct SweepD {
    static_assert(K >= 3 && K <= 24, "3 <= K <= 24");
    using Geom = DeepGeom<K>;
    static constexpr int LL = Geom::LL;
    static constexpr int KC = 4 * LL;
    static constexpr int D = Geom::D;       // rows loaded ahead
    static constexpr bool PAIR = Geom::PAIR; // rows processed in interleaved pairs
    static constexpr int N = 2 * K + D + 1;  // cycle length (registers, loop body rows)
    static constexpr int PRO = 2 * K + 1;    // prologue rows (the last stores the first output row)
    static constexpr int B = N;
#ifdef SMI_DEEP_G
    static constexpr int G = SMI_DEEP_G;
#else
    static constexpr int G = 2;  // rows per end-of-walk check (K = 20: 0.153 vs 0.162 ms for G = 1)
#endif
    static_assert(N % G == 0, "the loop body must hold whole groups");
    static_assert(KC >= K, "apron narrower than the cone");
    static constexpr int kExpLo = 2 * K - 124, kExpHi = 126 - 2 * K;
    static constexpr float kUnscale = 1.0f / (float)(1ull << (2 * K));  // 4^-K, exact

    const float *__restrict__ in;
    float *__restrict__ out;
    int rows, cols;
    int o0, o1;     // output rows of this wave
    int r_begin;    // input row of t = 0
    int n_in;       // input rows walked: (o1 - o0) + 2K
    int voff_ld;    // load byte offset of this lane in a row (clamped column)
    int voff;       // store byte offset (out of range: no store)
    int row_bytes;
    unsigned long long maskL, maskR;  // lanes holding column 0 / Y-1 of a global edge (copied)
    f32x2 quarter;                    // {0.25, 0.25} (exact walk)
    unsigned long long maskE;  // all lanes when the walk's first output row is a global edge row
    int emin, emax;
    float4 R[N];

    // register of ring position p after j rows
    static constexpr int ph(int p, int j) { return ((p - j) % N + N) % N; }

    // A wave-uniform row base (SGPRs) plus this lane's 32-bit byte offset:
    // global_load_dwordx4 in saddr form, no per-lane address arithmetic.
    // (Not __builtin_amdgcn_raw_buffer_load_b128: this toolchain's gfx950
    // backend emits a one-dword buffer_load_dword for it.)
    template <bool REV>
    __device__ __forceinline__ float4 ld(int t) const {
#ifdef SMI_DEEP_NOMEM  // experiment: levels only, no loads (timing)
        const float f = (float)(t & 7) * 0.125f + (float)voff_ld * 1e-6f;
        return make_float4(f, f + 0.25f, f + 0.5f, f + 0.75f);
#endif
        const int r = __builtin_amdgcn_readfirstlane(min(max(REV ? r_begin - t : r_begin + t, 0), rows - 1));
        const char *rowp = reinterpret_cast<const char *>(in + (size_t)r * cols);
        return *reinterpret_cast<const float4 *>(rowp + (unsigned)voff_ld);
    }

    __device__ __forceinline__ void note(const float4 &x) {
        const int e0 = __builtin_amdgcn_frexp_expf(x.x), e1 = __builtin_amdgcn_frexp_expf(x.y);
        const int e2 = __builtin_amdgcn_frexp_expf(x.z), e3 = __builtin_amdgcn_frexp_expf(x.w);
        emin = min(emin, min(e0, e1));
        emax = max(emax, max(e0, e1));
        emin = min(emin, min(e2, e3));
        emax = max(emax, max(e2, e3));
        // opaque: folded row by row (left alone, the compiler defers the
        // whole prologue's min/max tree to its end and keeps every row's
        // exponents live until then -- ~100 extra VGPRs at K = 10)
        asm("" : "+v"(emin), "+v"(emax));
    }

    // One level step of 4 cells per lane, ((S + W) + E) + N (x 0.25 unless
    // scaled), computed IN PLACE in the registers of the older operand row,
    // which dies here (tied asm operands).  Without this the register
    // allocator gives every new level row fresh registers and the cycle needs
    // ~60 more VGPRs than it holds (K = 16: 220 -> 156).  Walking down the
    // older row is N (the partial sums take temporaries, the + N lands in
    // N); walking up it is S (every add lands in S).  CE bit 0 / 1: the lanes
    // of maskL / maskR copy column 0 / Y-1 (stencil_smi.cl:143-151).
    template <bool REV, int CE, bool SC>
    __device__ __forceinline__ float4 step(const float4 &older, const float4 &c, const float4 &nw) const {
        f32x2 o01, o23;
        if constexpr (!REV) {
            const float4 &s = nw;
            const float w = shr1_any(c.w);
            const float e = shl1_any(c.x);
            float b0 = __fadd_rn(__fadd_rn(s.x, w), c.y);
            float b1 = __fadd_rn(__fadd_rn(s.y, c.x), c.z);
            float b2 = __fadd_rn(__fadd_rn(s.z, c.y), c.w);
            float b3 = __fadd_rn(__fadd_rn(s.w, c.z), e);
            // opaque: keeps the instruction selector from re-pairing the
            // scalar adds into v_pk_add_f32 with register moves for operands
            asm("" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3));
            o01 = f32x2{older.x, older.y};
            o23 = f32x2{older.z, older.w};
            asm("v_pk_add_f32 %0, %1, %0" : "+v"(o01) : "v"(f32x2{b0, b1}));
            asm("v_pk_add_f32 %0, %1, %0" : "+v"(o23) : "v"(f32x2{b2, b3}));
        } else {
            // W / E as separate v_mov_b32_dpp the compiler emits (it inserts
            // the DPP hazard wait states; it does not for DPP inside inline
            // asm), then every add in place in S
            const float w = shr1_any(c.w);
            const float e = shl1_any(c.x);
            float sx = older.x, sy = older.y, sz = older.z, sw = older.w;
            asm("v_add_f32 %0, %0, %1" : "+v"(sx) : "v"(w));
            asm("v_add_f32 %0, %0, %1" : "+v"(sy) : "v"(c.x));
            asm("v_add_f32 %0, %0, %1" : "+v"(sz) : "v"(c.y));
            asm("v_add_f32 %0, %0, %1" : "+v"(sw) : "v"(c.z));
            asm("v_add_f32 %0, %0, %1" : "+v"(sx) : "v"(c.y));
            asm("v_add_f32 %0, %0, %1" : "+v"(sy) : "v"(c.z));
            asm("v_add_f32 %0, %0, %1" : "+v"(sz) : "v"(c.w));
            asm("v_add_f32 %0, %0, %1" : "+v"(sw) : "v"(e));
            o01 = f32x2{sx, sy};
            o23 = f32x2{sz, sw};
            asm("v_pk_add_f32 %0, %0, %1" : "+v"(o01) : "v"(f32x2{nw.x, nw.y}));
            asm("v_pk_add_f32 %0, %0, %1" : "+v"(o23) : "v"(f32x2{nw.z, nw.w}));
        }
        if constexpr (!SC) {
            asm("v_pk_mul_f32 %0, %0, %1" : "+v"(o01) : "v"(quarter));
            asm("v_pk_mul_f32 %0, %0, %1" : "+v"(o23) : "v"(quarter));
        }
        float4 o = make_float4(o01.x, o01.y, o23.x, o23.y);
        if constexpr (CE & 1) {
            const float cx = SC ? c.x * 4.0f : c.x;
            asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(o.x) : "v"(cx), "s"(maskL));
        }
        if constexpr (CE & 2) {
            const float cw = SC ? c.w * 4.0f : c.w;
            asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(o.w) : "v"(cw), "s"(maskR));
        }
        return o;
    }

    template <bool REV, bool SC>
    __device__ __forceinline__ void store_row(int t, const float4 &vs) const {
        float4 v = vs;
        if constexpr (SC) {
            const f32x2 q = {kUnscale, kUnscale};
            const f32x2 a = f32x2{vs.x, vs.y} * q, b = f32x2{vs.z, vs.w} * q;
            v = make_float4(a.x, a.y, b.x, b.y);
        }
        const int j = REV ? o1 - 1 - (t - 2 * K) : o0 + (t - 2 * K);
        const bool in_block = REV ? (j >= o0 && j < o1) : (j < o1 && j >= o0);
        const int jj = __builtin_amdgcn_readfirstlane(min(max(j, 0), rows - 1));
        const int nrec = __builtin_amdgcn_readfirstlane(in_block ? row_bytes : 0);
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + (size_t)jj * cols, (short)0, nrec, 0x00020000);
        const u32x4 d = {__builtin_bit_cast(unsigned int, v.x), __builtin_bit_cast(unsigned int, v.y),
                         __builtin_bit_cast(unsigned int, v.z), __builtin_bit_cast(unsigned int, v.w)};
        __builtin_amdgcn_raw_buffer_store_b128(d, rs, voff, 0, 2 /* nt */);
    }

    // Input row t with the cycle rotated by J rows: issue the load of row
    // t + D into the register that became free at the end of the previous
    // row (clamped to the walk's last row: an L2 hit, not an HBM read), take
    // x = row t from position D, form the K levels in place.  TC >= 0: the
    // prologue's compile-time t (level l evaluated from t >= 2l on; the edge
    // row is input t - l == K).
    template <bool REV, int CE, bool SC, int J, int TC>
    __device__ __forceinline__ void row(int t) {
#ifdef SMI_DEEP_ROW_BARRIER
        __builtin_amdgcn_sched_barrier(0);
#endif
        R[ph(0, J)] = ld<REV>(min(t + D, n_in - 1));
        const float4 x = R[ph(D, J)];
        if constexpr (SC) note(x);
        float4 v = x;
        static_for<K>([&](auto L) {
            constexpr int l = L + 1;
            if constexpr (TC < 0 || TC >= 2 * l) {
                constexpr int ia = ph(D + 2 * l, J), ib = ph(D + 2 * l - 1, J);  // A_{l-1}, B_{l-1}
                const float4 older = R[ia], mid = R[ib];
                float4 nv = step<REV, CE, SC>(older, mid, v);
                if constexpr (TC >= 0 && TC - l == K) {
                    // the global edge row is copied (x 4 when scaled); maskE is
                    // all lanes or none (wave-uniform), the select stays in place
                    const float4 m = SC ? make_float4(mid.x * 4.0f, mid.y * 4.0f, mid.z * 4.0f, mid.w * 4.0f) : mid;
                    asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(nv.x) : "v"(m.x), "s"(maskE));
                    asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(nv.y) : "v"(m.y), "s"(maskE));
                    asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(nv.z) : "v"(m.z), "s"(maskE));
                    asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(nv.w) : "v"(m.w), "s"(maskE));
                }
                if constexpr (l < K) R[ia] = nv;
                v = nv;
            }
        });
        if constexpr (TC < 0 || TC == 2 * K) store_row<REV, SC>(t, v);
    }

    // Level l of the row at rotation J (TC as in row()): v = new_{l-1} in,
    // new_l out.
    template <bool REV, int CE, bool SC, int J, int TC, int l>
    __device__ __forceinline__ void level(float4 &v) {
        if constexpr (TC < 0 || TC >= 2 * l) {
            constexpr int ia = ph(D + 2 * l, J), ib = ph(D + 2 * l - 1, J);  // A_{l-1}, B_{l-1}
            const float4 older = R[ia], mid = R[ib];
            float4 nv = step<REV, CE, SC>(older, mid, v);
            if constexpr (TC >= 0 && TC - l == K) {
                const float4 m = SC ? make_float4(mid.x * 4.0f, mid.y * 4.0f, mid.z * 4.0f, mid.w * 4.0f) : mid;
                asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(nv.x) : "v"(m.x), "s"(maskE));
                asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(nv.y) : "v"(m.y), "s"(maskE));
                asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(nv.z) : "v"(m.z), "s"(maskE));
                asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(nv.w) : "v"(m.w), "s"(maskE));
            }
            if constexpr (l < K) R[ia] = nv;
            v = nv;
        }
    }

    // Rows t and t + 1 (rotations J, J + 1), their level chains interleaved
    // one level apart: row t + 1's level l - 1 needs row t's level l - 2
    // only, so each pair of steps is independent -- twice the ILP of one
    // chain, and the DPP / packed-result hazards of one chain are covered by
    // the other's instructions instead of s_nop.  Row t + 1's load goes out
    // after row t's level K (its register is row t's A_{K-1}).
    template <bool REV, int CE, bool SC, int J, int TC>
    __device__ __forceinline__ void pair(int t) {
        constexpr int TB = TC < 0 ? -1 : TC + 1;
        R[ph(0, J)] = ld<REV>(min(t + D, n_in - 1));
        float4 va = R[ph(D, J)];
        float4 vb = R[ph(D, J + 1)];
        if constexpr (SC) {
            note(va);
            note(vb);
        }
        level<REV, CE, SC, J, TC, 1>(va);
        static_for<K - 1>([&](auto L) {
            constexpr int l = L + 2;
            level<REV, CE, SC, J, TC, l>(va);
            level<REV, CE, SC, J + 1, TB, l - 1>(vb);
        });
        if constexpr (TC < 0 || TC == 2 * K) store_row<REV, SC>(t, va);
        R[ph(0, J + 1)] = ld<REV>(min(t + 1 + D, n_in - 1));
        level<REV, CE, SC, J + 1, TB, K>(vb);
        if constexpr (TB < 0 || TB == 2 * K) store_row<REV, SC>(t + 1, vb);
    }

    // Rows t + r .. t + N - 1 of one loop body (a whole cycle: the rotation
    // is the same at both ends, no register is ever copied), as a chain of
    // nested checks: the walk's end leaves the loop at once (the ring is dead
    // there), so no control-flow merge joins two rotation states.
    template <bool REV, int CE, bool SC, int r, int J0>
    __device__ __forceinline__ bool body(int t) {
        if constexpr (r == N) {
            return true;
        } else {
            // the walk's end is checked every G rows: the rows of a group
            // schedule together (a row past the end loads the clamped last row
            // and stores nothing)
            if constexpr (PAIR) {
            static_assert(N % 2 == 0, "pairs of rows need an even cycle (D odd)");
            if (t + r >= n_in) return false;
            pair<REV, CE, SC, (J0 + r) % N, -1>(t + r);
            return body<REV, CE, SC, r + 2, J0>(t);
            } else {
            if constexpr (r % G == 0) {
                if (t + r >= n_in) return false;
            }
            row<REV, CE, SC, (J0 + r) % N, -1>(t + r);
            return body<REV, CE, SC, r + 1, J0>(t);
            }
        }
    }

    template <bool REV, int CE, bool SC>
    __device__ __forceinline__ bool run() {
        emin = 0;
        emax = 0;
        // rows 0 .. D-1: loaded "at rows d - D" into position 0 of that row
        static_for<D>([&](auto Dd) {
            constexpr int d = Dd;
            R[ph(0, d - D)] = ld<REV>(d);
        });
#ifdef SMI_DEEP_NOPRO  // experiment: no triangular prologue (garbage levels, masked stores)
        static_for<2 * K>([&](auto P) { R[ph(D + 1 + P, 0)] = make_float4(0.f, 0.f, 0.f, 0.f); });
        for (int t = 0;; t += N)
            if (!body<REV, CE, SC, 0, 0>(t)) break;
#else
        // prologue: input rows 0 .. 2K, compile-time t (rotation j = t)
        if constexpr (PAIR) {
            row<REV, CE, SC, 0, 0>(0);
            static_for<K>([&](auto P) {
                constexpr int t = 2 * P + 1;
                __builtin_amdgcn_sched_barrier(0);
                pair<REV, CE, SC, t % N, t>(t);
            });
        } else {
            static_for<PRO>([&](auto T) {
                constexpr int t = T;
                // scheduling regions of G rows, as in the loop (one region of
                // 2K+1 rows costs minutes of compile time for nothing)
                if constexpr (t % G == 0 && t > 0) __builtin_amdgcn_sched_barrier(0);
                row<REV, CE, SC, t % N, t>(t);
            });
        }
        // steady state: N rows per iteration from rotation PRO mod N
        for (int t = PRO;; t += N)
            if (!body<REV, CE, SC, 0, PRO % N>(t)) break;
#endif
        if constexpr (SC) {
            const bool bad = emin < kExpLo || emax > kExpHi;
            if (__builtin_amdgcn_ballot_w64(bad) != 0) {
                __builtin_amdgcn_s_waitcnt(0x0F70);  // the exact walk's stores land after these
                return false;
            }
        }
        return true;
    }

    template <bool REV, int CE>
    __device__ __forceinline__ void go() {
        if (run<REV, CE, true>()) return;
#ifndef SMI_DEEP_NO_EXACT  // experiment switch (tools/deepbench register studies only)
        run<REV, CE, false>();
#endif
    }
};

// One wave: strip `strip`, block rb of nb.  The host guarantees that every
// block has at least K rows and that a tile with both global row edges has
// two blocks or more (so only the first block of a tile with gT reaches row
// 0, only the last with gB row X-1).
template <int K>
__device__ __forceinline__ void sweepd_task(const SweepKArgs &a, int strip, int rb, int nb, int wlast, int lane) {
    using S = SweepD<K>;
    constexpr int SW = 256 - 2 * S::KC;
    S w;
    w.in = a.in;
    w.out = a.out;
    w.rows = a.rows;
    w.cols = a.cols;
    sweepd_block_rows(a, rb, nb, wlast, &w.o0, &w.o1);
    w.n_in = (w.o1 - w.o0) + 2 * K;
    const int cs = (a.col_lo & ~31) + strip * SW;
    const int cb = cs - S::KC + 4 * lane;
    w.voff_ld = min(max(cb, 0), a.cols - 4) * 4;
    const bool st = lane >= S::LL && lane < 64 - S::LL && cb >= a.col_lo && cb < a.col_hi;
    w.row_bytes = a.cols * 4;
    w.voff = st ? cb * 4 : 0x7ffffff0;
    w.maskL = __builtin_amdgcn_ballot_w64(a.gL && cb == 0);
    w.maskR = __builtin_amdgcn_ballot_w64(a.gR && cb + 4 == a.cols);
    w.quarter = f32x2{0.25f, 0.25f};
    const int ce = ((a.gL && cs - S::KC <= 0) ? 1 : 0) | ((a.gR && cs - S::KC + 256 >= a.cols) ? 2 : 0);
    const bool top = a.gT && w.o0 == 0;
    const bool bot = a.gB && w.o1 == a.rows;
#ifdef SMI_DEEP_INTERIOR_ONLY  // experiment builds: every block walks down, edges not handled
    const bool rev = false;
#else
    const bool rev = bot && !top;  // the bottom block walks upwards (its edge row is then a prologue row)
#endif
    w.maskE = __builtin_amdgcn_ballot_w64(top || bot);  // uniform: all lanes or none
    w.r_begin = rev ? w.o1 - 1 + K : w.o0 - K;
    // column-edge strips run one variant for either side (the other side's
    // mask is empty): four walks per K instead of eight keep the build short
#ifdef SMI_DEEP_FORCE  // experiment: every wave runs variant SMI_DEEP_FORCE (timing only, wrong results)
    switch (SMI_DEEP_FORCE) {
#else
    switch ((rev ? 2 : 0) + (ce ? 1 : 0)) {
#endif
    case 0: w.template go<false, 0>(); break;
#ifndef SMI_DEEP_INTERIOR_ONLY
    case 1: w.template go<false, 3>(); break;
    case 2: w.template go<true, 0>(); break;
    default: w.template go<true, 3>(); break;
#else
    default: w.template go<false, 0>(); break;
#endif
    }
}

#ifndef SMI_DEEP_WPE
#define SMI_DEEP_WPE 1
#endif

// Task order: the interior strips' blocks row band by row band (the waves of
// a workgroup are neighbouring strips of one band: their overlapping window
// columns meet in L2), then the edge-column strips' blocks.
template <int K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SMI_DEEP_WPE, 8))) void sweepd_kernel(
    SweepKArgs a, SweepDGeom g) {
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int lane = threadIdx.x & 63;
    const int task = __builtin_amdgcn_readfirstlane(lb * 4 + (int)(threadIdx.x >> 6));
    if (task >= g.tasks) return;  // wave-uniform
    const int ti = g.n_int * g.nrb;
    if (task < ti) {
        const int rb = task / g.n_int;
        sweepd_task<K>(a, g.int0 + task - rb * g.n_int, rb, g.nrb, g.wlast, lane);
    } else {
        const int t2 = task - ti;
        const int k = t2 / g.nrb_ce;
        sweepd_task<K>(a, g.ce[k], t2 - k * g.nrb_ce, g.nrb_ce, g.wlast, lane);
    }
}

}  // namespace smi

// One translation unit per K (stencild_k<K>.hip): the eight instantiations
// compile in parallel.
#define SMI_SWEEPD_INSTANCE(K)                                                                           \
    namespace smi {                                                                                      \
    int sweepd_launch_k##K(const SweepKArgs &a, const SweepDGeom &g, int blocks, hipStream_t s,          \
                           hipEvent_t start, hipEvent_t stop) {                                          \
        if (start || stop)                                                                               \
            hipExtLaunchKernelGGL((sweepd_kernel<K>), dim3(blocks), dim3(256), 0, s, start, stop, 0, a, g); \
        else                                                                                             \
            hipLaunchKernelGGL((sweepd_kernel<K>), dim3(blocks), dim3(256), 0, s, a, g);                  \
        SMI_HIP_CHECK(hipGetLastError());                                                                \
        return SMI_SUCCESS;                                                                              \
    }                                                                                                    \
    int sweepd_resident_k##K() {                                                                         \
        static int cached[64] = {};                                                                      \
        int dev = 0;                                                                                     \
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;                          \
        if (cached[dev]) return cached[dev];                                                             \
        int per_cu = 0, cus = 0;                                                                         \
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, sweepd_kernel<K>, 256, 0) != hipSuccess) \
            return 0;                                                                                    \
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0; \
        cached[dev] = per_cu * cus * 4;                                                                  \
        return cached[dev];                                                                              \
    }                                                                                                    \
    }
