// stencil_bandk.h -- the halo-facing bands of a multi-rank K-step pass as
// short register walks, one cell per lane (instantiated per K in
// bandk_k<K>.hip; the lean variant bandl_kernel<K> for K = 13..20).
//
// In a multi-rank run with K steps per pass, every tile cell within K rows of
// a side with a neighbour, or within KC = 4 ceil(K/4) columns of one, depends
// on that neighbour's current cells; the interior sweep (stencilk.h) leaves
// those bands alone and this kernel computes them from the tile, the depth-K
// halos and the K x KC corner blocks of the diagonal neighbours, then tees the
// next exchange's packed columns and corner blocks out of its stores -- the
// reference's Write kernel sending each boundary row/column as it is produced
// (stencil_smi.cl:183-224).  Per-cell arithmetic and the global-edge copy
// rule are the sweep's (stencil_smi.cl:143-156), exact (x 0.25 every level).
//
// Shape.  The band kernel sits on the critical path of every pass twice: the
// exchange waits for it, and the next interior waits for it.  What bounds it
// is the length of one wave's dependent walk, not bytes or total VALU work
// (~5 MB and ~1 M wave-instructions at 8192^2, K = 12: a few us of the whole
// GPU).  Round 2's LDS ring (barrier per level) took ~30 us alone; a float4
// walk of 3K rows per wave with all rows staged in LDS took ~45 us alone
// (54 KiB of LDS per wave: one wave per CU pair of SIMDs, ~9 k dependent
// instructions each).  Here a lane owns ONE cell across the band, so a wave
// is 64 cells wide and walks only the band's depth:
//   top / bottom band: lanes = 64 columns, the wave walks rows [-K, 2K)
//     (bottom: [X-2K, X+K)), level l evaluated where the output cone needs
//     it (3K - 2l rows), the K output rows stored by lanes [K, 64-K)
//   left / right band: transposed -- lanes = 64 rows, the wave walks the
//     columns [-K, KC+K) (right: [Y-KC-K, Y+K)) of each lane's own row, N/S
//     neighbours by DPP, the KC output columns stored by lanes [K, 64-K)
// Every input of a wave is loaded up front into registers (one memory round
// trip; beside the HBM-saturating interior sweep a round trip takes
// microseconds, so a walk that waits on loads row by row is latency-bound),
// then the walk runs fully unrolled from registers: ~276 cell-levels per lane
// at K = 12, 4 VALU each (two of them DPP adds), ~800 waves of < 100 VGPRs.
#pragma once

#include "stencilk.h"

namespace smi {

// Level step on one cell per lane, in the reference order
// 0.25 * (((S + W) + E) + N).  ROWWALK: the wave walks down rows and its lanes
// are columns (W / E from lanes -1 / +1, N the older and S the newer input);
// else it walks along columns and its lanes are rows (N / S from lanes -1 /
// +1, W older, E newer).  Lanes 0 / 63 get whatever the DPP leaves: they are
// never stored and feed only lanes that are not either.
template <bool ROWWALK>
__device__ __forceinline__ float band_cell(float older, float c, float newer) {
    if constexpr (ROWWALK)
        return jacobi(newer, shr1_any(c), shl1_any(c), older);
    else
        return jacobi(shl1_any(c), older, newer, shr1_any(c));
}

// Source of one extended-tile cell (r, c), r in [-K, X+K), c in [-KC, Y+KC):
// tile, side halo ([row][KC]), top/bottom halo (K x Y) or corner block
// (K x KC).  Rows / columns past a global edge (no neighbour there) are
// clamped onto the tile: those cells only feed cells the copy rule overrides.
// a wave-uniform value the optimiser cannot trace back to its memory slot
template <typename T>
__device__ __forceinline__ T val(T x) {
    asm("" : "+s"(x));
    return x;
}

struct BandSrc {
    const float *in, *top, *bot, *left, *right, *c0, *c1, *c2, *c3;
    int X, Y, KC, K;
    bool hT, hB, hL, hR;
    __device__ __forceinline__ BandSrc(const BandKArgs &a, int K_)
        : in(a.in), top(a.h.top), bot(a.h.bot), left(a.h.left), right(a.h.right), c0(a.h.corner[0]),
          c1(a.h.corner[1]), c2(a.h.corner[2]), c3(a.h.corner[3]), X(a.rows), Y(a.cols), KC(a.kc), K(K_),
          hT(a.has[0]), hB(a.has[1]), hL(a.has[2]), hR(a.has[3]) {}
    __device__ __forceinline__ const float *at(int r, int c) const {
        r = min(max(r, hT ? -K : 0), hB ? X + K - 1 : X - 1);
        c = min(max(c, hL ? -KC : 0), hR ? Y + KC - 1 : Y - 1);
        const bool rin = r >= 0 && r < X, cin = c >= 0 && c < Y;
        const int rt = min(max(r, 0), X - 1), ct = min(max(c, 0), Y - 1);
        const int hr = r < 0 ? r + K : r - X;   // halo row (valid when !rin)
        const int hc = c < 0 ? c + KC : c - Y;  // halo column (valid when !cin)
        // (base, row index, row stride, column index) of the region
        // (selects between opaque values: a select between two fields would
        // be folded into a load from a computed address inside the struct,
        // which keeps it in scratch)
        const float *side = c < 0 ? val(left) : val(right);
        const float *vert = r < 0 ? val(top) : val(bot);
        const float *corn = r < 0 ? (c < 0 ? val(c0) : val(c1)) : (c < 0 ? val(c2) : val(c3));
        const float *base = rin ? (cin ? val(in) : side) : (cin ? vert : corn);
        const int ri = rin ? rt : hr, ci = cin ? ct : hc, stride = cin ? Y : KC;
        return base + (size_t)ri * stride + ci;
    }
};

template <int K>
struct BandW {
    static constexpr int KC = kc_of(K);
    static constexpr int SW = 64 - 2 * K;  // stored lanes (cells) per wave
    static constexpr int NR = 3 * K;       // inputs of a row walk
    static constexpr int NC = 2 * K + KC;  // inputs of a column walk
    static constexpr int G4 = 3 * KC / 4;  // float4 groups a column-walk lane loads

    // The walk over N register-resident inputs: level l at input t (t >= 2l)
    // is the cell at walk position t - l, from level l-1 at inputs t-2,
    // t-1, t (3-slot ring per level, slot = t mod 3, compile-time).  The
    // level-K value of input t (t >= 2K) goes to out(t - 2K, v).  CP: this
    // lane copies its cell every step (global edge across the walk).
    template <bool ROWWALK, bool CP, int N, typename Out>
    __device__ __forceinline__ static void walk(const float (&x)[N], bool cp, Out &&out) {
        float W[K][3];
        static_for<N>([&](auto T) {
            constexpr int t = T;
            W[0][t % 3] = x[t];
            float v = 0.0f;
            static_for<K>([&](auto L) {
                constexpr int l = L + 1;
                if constexpr (t >= 2 * l) {
                    const float c = W[l - 1][(t + 2) % 3];
                    v = band_cell<ROWWALK>(W[l - 1][(t + 1) % 3], c, W[l - 1][t % 3]);
                    if constexpr (CP) v = cp ? c : v;
                    if constexpr (l < K) W[l][t % 3] = v;
                }
            });
            if constexpr (t >= 2 * K) out(std::integral_constant<int, t - 2 * K>{}, v);
        });
    }

    // top (BOT = false) or bottom band: lane = column c, rows r0 + t
    template <bool BOT, bool CP>
    __device__ __forceinline__ static void rows(const BandKArgs &a, int w, int lane) {
        const int X = a.rows, Y = a.cols;
        const int c = w * SW - K + lane;
        const int r0 = BOT ? X - 2 * K : -K;
        // the lane's sources: halo rows (top: inputs [0, K); bottom: [2K, 3K))
        // from one base with one stride, tile rows from another
        const int th = BOT ? 2 * K : 0;  // first halo input
        const int tt = BOT ? 0 : K;      // first tile input
        const BandSrc src(a, K);
        const float *ph = src.at(r0 + th, c);
        const float *pt = src.at(r0 + tt, c);
        const int sh = (int)(src.at(r0 + th + 1, c) - ph);
        const int st = (int)(src.at(r0 + tt + 1, c) - pt);
        float x[NR];
        static_for<NR>([&](auto T) {
            constexpr int t = T;
            constexpr bool halo = BOT ? t >= 2 * K : t < K;
            x[t] = halo ? ph[(t - th) * sh] : pt[(t - tt) * st];
        });
        const bool store = lane >= K && lane < 64 - K && c < Y;
        const bool cp = (!a.has[2] && c == 0) || (!a.has[3] && c == Y - 1);
        const int KCr = a.kc;
        walk<true, CP>(x, cp, [&](auto Q, float v) {
            constexpr int q = Q;  // output row r0 + K + q
            if (!store) return;
            const int r = r0 + K + q;
            a.out[(size_t)r * Y + c] = v;
            if (!a.pack) return;
            // tee: packed side columns and this band's two K x KC corner blocks
            if (c < KCr) {
                a.h.send_left[(size_t)r * KCr + c] = v;
                a.h.send_corner[BOT ? 2 : 0][q * KCr + c] = v;
            }
            if (c >= Y - KCr) {
                a.h.send_right[(size_t)r * KCr + c - (Y - KCr)] = v;
                a.h.send_corner[BOT ? 3 : 1][q * KCr + c - (Y - KCr)] = v;
            }
        });
    }

    // left (RIGHT = false) or right band: lane = row r, columns c0 + t
    template <bool RIGHT, bool CP>
    __device__ __forceinline__ static void cols(const BandKArgs &a, int w, int lane) {
        const int X = a.rows, Y = a.cols;
        const int r = a.rlo + w * SW - K + lane;
        // float4 groups [-KC, 2KC) (right: [Y - 2KC, Y + KC)); the walk starts
        // KC - K columns in, at column -K (right: Y - KC - K)
        const int g0 = RIGHT ? Y - 2 * KC : -KC;
        const BandSrc src(a, K);
        float4 g[G4];
        static_for<G4>([&](auto G) {
            constexpr int j = G;
            g[j] = *reinterpret_cast<const float4 *>(src.at(r, g0 + 4 * j));
        });
        float x[NC];
        static_for<NC>([&](auto T) {
            constexpr int e = (KC - K) + T;
            const float4 &q = g[e / 4];
            x[T] = e % 4 == 0 ? q.x : e % 4 == 1 ? q.y : e % 4 == 2 ? q.z : q.w;
        });
        const bool store = lane >= K && lane < 64 - K && r < a.rhi;
        const bool cp = (!a.has[0] && r == 0) || (!a.has[1] && r == X - 1);
        float o[KC];
        walk<false, CP>(x, cp, [&](auto Q, float v) { o[Q] = v; });
        if (!store) return;
        const int c0 = RIGHT ? Y - KC : 0;
        float *send = RIGHT ? a.h.send_right : a.h.send_left;
        static_for<KC / 4>([&](auto G) {
            constexpr int j = 4 * G;
            const float4 v = make_float4(o[j], o[j + 1], o[j + 2], o[j + 3]);
            *reinterpret_cast<float4 *>(a.out + (size_t)r * Y + c0 + j) = v;
            if (a.pack) {
                *reinterpret_cast<float4 *>(send + (size_t)r * KC + j) = v;
                // corner blocks of rows this band owns (only when the top /
                // bottom side is a global edge, i.e. never sent)
                if (r < K) *reinterpret_cast<float4 *>(a.h.send_corner[RIGHT ? 1 : 0] + r * KC + j) = v;
                if (r >= X - K)
                    *reinterpret_cast<float4 *>(a.h.send_corner[RIGHT ? 3 : 2] + (r - (X - K)) * KC + j) = v;
            }
        });
    }
};

// Band segment wv: one wave per 64-cell run of a band; segments [first[0],
// first[1]) top, [first[1], first[2]) bottom, [first[2], first[3]) left,
// [first[3], first[4]) right.
template <int K>
__device__ __forceinline__ void bandk_wave(const BandKArgs &a, int wv, int lane) {
    using B = BandW<K>;
    const int band = (wv >= a.first[1]) + (wv >= a.first[2]) + (wv >= a.first[3]);
    // (no dynamic index into the kernel argument: that would copy it to scratch)
    const int w = wv - (band == 0 ? 0 : band == 1 ? a.first[1] : band == 2 ? a.first[2] : a.first[3]);
    const int X = a.rows, Y = a.cols;
    if (band < 2) {
        // does this wave hold column 0 or Y-1 of a global left / right edge?
        const int c_lo = w * B::SW - K, c_hi = c_lo + 63;
        const bool cp = (!a.has[2] && c_lo <= 0 && c_hi >= 0) || (!a.has[3] && c_lo <= Y - 1 && c_hi >= Y - 1);
        if (band == 0)
            cp ? B::template rows<false, true>(a, w, lane) : B::template rows<false, false>(a, w, lane);
        else
            cp ? B::template rows<true, true>(a, w, lane) : B::template rows<true, false>(a, w, lane);
    } else {
        const int r_lo = a.rlo + w * B::SW - K, r_hi = r_lo + 63;
        const bool cp = (!a.has[0] && r_lo <= 0 && r_hi >= 0) || (!a.has[1] && r_lo <= X - 1 && r_hi >= X - 1);
        if (band == 2)
            cp ? B::template cols<false, true>(a, w, lane) : B::template cols<false, false>(a, w, lane);
        else
            cp ? B::template cols<true, true>(a, w, lane) : B::template cols<true, false>(a, w, lane);
    }
}

// The bands beside the interior sweep (on the comm stream); four
// independent waves per workgroup.  With one wave per segment (~800 at
// 8192^2, K = 12) the kernel needs more wave slots than the interior's one
// round leaves, and its waves only run in the interior's tail -- the exchange
// then sits between two passes.  With fewer waves than segments (the wave
// slots the interior reserves, smi_stencil_set_bands) every wave walks
// segments wv, wv + waves, ... in turn and the bands finish beside the
// interior, so the exchange overlaps it.
template <int K>
__global__ __launch_bounds__(256) void bandk_kernel(BandKArgs a) {
    const int waves = gridDim.x * 4;
    const int wv0 = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (int)(threadIdx.x >> 6));
    for (int wv = wv0; wv < a.first[4]; wv += waves)  // wave-uniform
        bandk_wave<K>(a, wv, threadIdx.x & 63);
}

// ---------------------------------------------------------------------------
// The lean band kernel (K = 13..20, round 4): the same cells, the same
// arithmetic and the same stores as BandW, shaped to run BESIDE the deep
// interior sweep instead of in its tail.  sweepd_kernel<20> holds 2 waves per
// SIMD at 219 VGPRs (448 of the SIMD's 512), so a wave of <= 64 VGPRs still
// fits next to them; BandW<20> needs 249 (every input loaded up front, a
// K-level ring) and only gets slots as interior waves retire, which puts the
// bands -- and the exchange behind them -- on the pass boundary.  Beside the
// interior the band kernel's VALU work slows the interior down, so it is
// also cut: a lane owns TWO cells (columns 2l, 2l+1 of a 128-column window in
// the row walks, rows 2l, 2l+1 in the column walks), the neighbour across
// the pair comes from the lane itself, and a wave stores 128 - 2KE cells
// (KE = K rounded up to even: pair-aligned windows) instead of 64 - 2K:
// 88 instead of 24 at K = 20, ~2.5x less VALU per band cell.
//
// A streaming walk holds two values per level and cell: too many for 64
// VGPRs.  So each wave walks its segment in KS = ceil(K/5) stages of at most
// 5 levels: the first from the streamed inputs, its level-L0 values of
// positions [L0, N-L0) parked in LDS (lane-private columns), each later stage
// reading the previous one's parked values and overwriting them in place.
// Level l at walk position p always reads level l-1 at p-1, p, p+1, so a
// stage is the same recurrence on a shorter input -- bit-identical.
// Each workgroup reserves more than half a CU's LDS (kBandLeanLds), so at
// most one workgroup -- one wave per SIMD -- sits on a CU: the interior's two
// waves per SIMD always fit beside it.  The grid is at most one workgroup per
// CU, its waves looping over the band segments.
template <int K>
struct BandL {
    using B = BandW<K>;
    static constexpr int KC = B::KC, NR = B::NR, NC = B::NC, G4 = B::G4;
    static constexpr int KE = K + (K & 1);   // pair-aligned cone margin
    static constexpr int SW = 128 - 2 * KE;  // cells stored per wave (segment length)
    static constexpr int LMAX = 5;
    static constexpr int KS = (K + LMAX - 1) / LMAX;
    static constexpr int lv(int s) { return K / KS + (s < K % KS ? 1 : 0); }
    static constexpr int L0 = lv(0);
    // parked positions (x 2 cells) per lane: a row walk's stage outputs, or
    // a column walk's staged inputs (its 3KC columns, float4 groups from
    // -KC / Y - 2KC) -- whichever is more
    static constexpr int NPOS = (NR - 2 * L0 > 3 * KC) ? NR - 2 * L0 : 3 * KC;
    // LDS stride of one position, in float2: 64 lanes + 1, so that the
    // transposing writes of the column walks' staging spread over the banks
    static constexpr int PST = 65;
    static constexpr int LA = 3;                                // global inputs loaded ahead
    static constexpr int LAS = 2;                               // parked values read ahead

    // One level step of a lane's two cells (reference order 0.25 *
    // (((S + W) + E) + N) each).  ROWWALK: cells = columns (a | b), W / E of
    // a = b of lane-1 / own b, of b = own a / a of lane+1; else cells = rows,
    // N / S of a = b of lane-1 / own b, of b = own a / a of lane+1.
    // The two cells' adds are scalar where an operand crosses lanes (DPP,
    // fused into the add) and packed (v_pk_add_f32) where both operands are
    // a lane's own register pair; the x 0.25 is one v_pk_mul_f32: 6 VALU per
    // lane-level instead of 8, the same IEEE operations in the same order.
    template <bool ROWWALK>
    __device__ __forceinline__ static float2 cell2(float2 older, float2 c, float2 newer) {
        const f32x2 q = {0.25f, 0.25f};
        if constexpr (ROWWALK) {
            // ((S + W) + E) per cell, then + N on the pair
            float a = __fadd_rn(__fadd_rn(newer.x, shr1_any(c.y)), c.y);
            float b = __fadd_rn(__fadd_rn(newer.y, c.x), shl1_any(c.x));
            asm("" : "+v"(a), "+v"(b));  // no re-pairing of the scalar adds (moves)
            const f32x2 o = (f32x2{a, b} + f32x2{older.x, older.y}) * q;
            return make_float2(o.x, o.y);
        } else {
            // (S + W) per cell, + E on the pair, + N per cell
            float a = __fadd_rn(c.y, older.x);
            float b = __fadd_rn(shl1_any(c.x), older.y);
            asm("" : "+v"(a), "+v"(b));
            const f32x2 p = f32x2{a, b} + f32x2{newer.x, newer.y};
            float u = __fadd_rn(p.x, shr1_any(c.y));
            float v = __fadd_rn(p.y, c.x);
            asm("" : "+v"(u), "+v"(v));
            const f32x2 o = f32x2{u, v} * q;
            return make_float2(o.x, o.y);
        }
    }

    // Levels 1..LV over N inputs: ld(t) yields input t (issuing its own
    // loads ahead), out(q, v) takes the level-LV values of input t = q + 2LV.
    // cp: per cell, the copy rule (a global edge across the walk).
    template <bool ROWWALK, bool CP, int N, int LV, typename Ld, typename Out>
    __device__ __forceinline__ static void walk(bool cpa, bool cpb, Ld &&ld, Out &&out) {
        float2 W[LV][3];
        static_for<N>([&](auto T) {
            constexpr int t = T;
            W[0][t % 3] = ld(T);
            float2 v = make_float2(0.0f, 0.0f);
            static_for<LV>([&](auto L) {
                constexpr int l = L + 1;
                if constexpr (t >= 2 * l) {
                    const float2 c = W[l - 1][(t + 2) % 3];
                    v = cell2<ROWWALK>(W[l - 1][(t + 1) % 3], c, W[l - 1][t % 3]);
                    if constexpr (CP) {
                        v.x = cpa ? c.x : v.x;
                        v.y = cpb ? c.y : v.y;
                    }
                    if constexpr (l < LV) W[l][t % 3] = v;
                    // (a region per level: the scheduler would otherwise
                    // start every level's shuffles at once and spill)
                    __builtin_amdgcn_sched_barrier(0);
                }
            });
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (t >= 2 * LV) out(std::integral_constant<int, t - 2 * LV>{}, v);
        });
    }

    // Stages S.. over the N parked positions of the previous stage (in place:
    // stage output u is written after input u + 2LV was read); the last
    // stage hands its values to out.
    template <bool ROWWALK, bool CP, int S, int N, typename Out>
    __device__ __forceinline__ static void stages(bool cpa, bool cpb, float2 *park, int lane, Out &&out) {
        constexpr int LV = lv(S);
        // the previous stage's values go through LDS: without this barrier
        // the compiler forwards every parked value to its reload and keeps
        // them all in registers (and spills)
        asm volatile("" ::: "memory");
        float2 y[N];
        static_for<LAS>([&](auto U) { y[U] = park[U * PST + lane]; });
        auto ld = [&](auto U) {
            constexpr int u = U;
            if constexpr (u + LAS < N) y[u + LAS] = park[(u + LAS) * PST + lane];
            return y[u];
        };
        if constexpr (S + 1 == KS) {
            walk<ROWWALK, CP, N, LV>(cpa, cpb, ld, out);
        } else {
            walk<ROWWALK, CP, N, LV>(cpa, cpb, ld, [&](auto U, float2 v) { park[U * PST + lane] = v; });
            stages<ROWWALK, CP, S + 1, N - 2 * LV>(cpa, cpb, park, lane, out);
        }
    }

    // top (BOT = false) or bottom band: lane = columns c, c + 1, rows r0 + t
    template <bool BOT, bool CP>
    __device__ __forceinline__ static void rows(const BandKArgs &a, int w, int lane, float2 *park) {
        const int X = a.rows, Y = a.cols;
        const int c = w * SW - KE + 2 * lane;  // even: a pair never straddles a region
        const int r0 = BOT ? X - 2 * K : -K;
        const int th = BOT ? 2 * K : 0;
        const int tt = BOT ? 0 : K;
        const BandSrc src(a, K);
        // lanes past a global edge read any pair of the tile (their cells
        // only feed cells the copy rule overrides)
        const int cl = min(max(c, a.has[2] ? -KC : 0), a.has[3] ? Y + KC - 2 : Y - 2);
        const float *ph = src.at(r0 + th, cl);
        const float *pt = src.at(r0 + tt, cl);
        const int sh = (int)(src.at(r0 + th + 1, cl) - ph);
        const int st = (int)(src.at(r0 + tt + 1, cl) - pt);
        auto gload = [&](auto T) -> float2 {
            constexpr int t = T;
            constexpr bool halo = BOT ? t >= 2 * K : t < K;
            return *reinterpret_cast<const float2 *>(halo ? ph + (t - th) * sh : pt + (t - tt) * st);
        };
        const bool store = lane >= KE / 2 && lane < 64 - KE / 2 && c < Y;
        const bool cpa = !a.has[2] && c == 0;
        const bool cpb = !a.has[3] && c + 1 == Y - 1;
        float2 x[NR];
        static_for<LA>([&](auto T) { x[T] = gload(T); });
        walk<true, CP, NR, L0>(
            cpa, cpb,
            [&](auto T) {
                constexpr int t = T;
                if constexpr (t + LA < NR) x[t + LA] = gload(std::integral_constant<int, t + LA>{});
                return x[t];
            },
            [&](auto U, float2 v) { park[U * PST + lane] = v; });
        const int KCr = a.kc;
        stages<true, CP, 1, NR - 2 * L0>(cpa, cpb, park, lane, [&](auto Q, float2 v) {
            constexpr int q = Q;  // output row r0 + K + q
            if (!store) return;
            const int r = r0 + K + q;
            *reinterpret_cast<float2 *>(a.out + (size_t)r * Y + c) = v;
            if (!a.pack) return;
            // KCr and Y - KCr are multiples of 4: the pair lies on one side
            if (c < KCr) {
                *reinterpret_cast<float2 *>(a.h.send_left + (size_t)r * KCr + c) = v;
                *reinterpret_cast<float2 *>(a.h.send_corner[BOT ? 2 : 0] + q * KCr + c) = v;
            }
            if (c >= Y - KCr) {
                *reinterpret_cast<float2 *>(a.h.send_right + (size_t)r * KCr + c - (Y - KCr)) = v;
                *reinterpret_cast<float2 *>(a.h.send_corner[BOT ? 3 : 1] + q * KCr + c - (Y - KCr)) = v;
            }
        });
    }

    // left (RIGHT = false) or right band: lane = rows r, r + 1, columns c0 + t.
    // The walk is transposed (a lane owns two rows), but its global memory
    // traffic is not: the wave's 128 rows x 3KC input columns are loaded
    // row-contiguously (float4 groups, consecutive lanes along a row) and
    // written transposed into its LDS park, the walk reads its inputs from
    // there, and the KC output columns leave through the park the same way.
    // Lanes reading / writing 64 different rows per instruction made the
    // interior sweep beside this kernel ~7 % slower per pass than the row walks
    // with the same arithmetic (rehearsal cases brows / bcols, DESIGN.md
    // section 6).
    template <bool RIGHT, bool CP>
    __device__ __forceinline__ static void cols(const BandKArgs &a, int w, int lane, float2 *park) {
        const int X = a.rows, Y = a.cols;
        const int R = a.rlo + w * SW - KE;  // the wave's first row; lane l walks rows R + 2l, R + 2l + 1
        const int r = R + 2 * lane;
        const int g0 = RIGHT ? Y - 2 * KC : -KC;
        const BandSrc src(a, K);
        float *pf = reinterpret_cast<float *>(park);
        // staging: element e in [0, 3KC) of row R + rho -> park[e][rho / 2] . (rho % 2)
        constexpr int NG = 3 * KC / 4;  // float4 groups per row
        constexpr int NI = (128 * NG + 63) / 64, IB = 6;  // instructions, in batches of IB loads in flight
#pragma unroll 1
        for (int i0 = 0; i0 < NI; i0 += IB) static_for<IB>([&](auto I) {
            const int idx = (i0 + (int)I) * 64 + lane;
            if (idx < 128 * NG) {
                const int rho = idx / NG, j = idx - rho * NG;
                const float4 q = *reinterpret_cast<const float4 *>(src.at(R + rho, g0 + 4 * j));
                float *d = pf + ((4 * j) * PST + (rho >> 1)) * 2 + (rho & 1);
                d[0] = q.x;
                d[2 * PST] = q.y;
                d[4 * PST] = q.z;
                d[6 * PST] = q.w;
            }
        });
        asm volatile("" ::: "memory");  // (the walk reads the staging back)
        constexpr int E0 = KC - K;      // walk input t is staged element E0 + t
        const bool cpa = (!a.has[0] && r == 0) || (!a.has[1] && r == X - 1);
        const bool cpb = (!a.has[0] && r + 1 == 0) || (!a.has[1] && r + 1 == X - 1);
        float2 y[LAS + 1];
        static_for<LAS>([&](auto U) { y[U] = park[(E0 + U) * PST + lane]; });
        walk<false, CP, NC, L0>(
            cpa, cpb,
            [&](auto T) {
                constexpr int t = T;
                if constexpr (t + LAS < NC) y[(t + LAS) % (LAS + 1)] = park[(E0 + t + LAS) * PST + lane];
                return y[t % (LAS + 1)];
            },
            [&](auto U, float2 v) { park[U * PST + lane] = v; });
        // the last stage's KC outputs into park[0 .. KC), then out row-contiguously
        stages<false, CP, 1, NC - 2 * L0>(cpa, cpb, park, lane, [&](auto Q, float2 v) { park[Q * PST + lane] = v; });
        asm volatile("" ::: "memory");
        const int c0 = RIGHT ? Y - KC : 0;
        float *send = RIGHT ? a.h.send_right : a.h.send_left;
        constexpr int NO = KC / 4;  // float4 groups of a row's outputs
        constexpr int NJ = (128 * NO + 63) / 64;
#pragma unroll 1
        for (int i0 = 0; i0 < NJ; i0 += IB) static_for<IB>([&](auto I) {
            const int idx = (i0 + (int)I) * 64 + lane;
            if (idx < 128 * NO) {
                const int rho = idx / NO, j = idx - rho * NO;
                const int rr = R + rho;
                if (rho >= KE && rho < 128 - KE && rr < a.rhi) {
                    const float *sv = pf + ((4 * j) * PST + (rho >> 1)) * 2 + (rho & 1);
                    const float4 v = make_float4(sv[0], sv[2 * PST], sv[4 * PST], sv[6 * PST]);
                    *reinterpret_cast<float4 *>(a.out + (size_t)rr * Y + c0 + 4 * j) = v;
                    if (a.pack) {
                        *reinterpret_cast<float4 *>(send + (size_t)rr * KC + 4 * j) = v;
                        // corner blocks of rows this band owns (only when the top /
                        // bottom side is a global edge, i.e. never sent)
                        if (rr < K) *reinterpret_cast<float4 *>(a.h.send_corner[RIGHT ? 1 : 0] + rr * KC + 4 * j) = v;
                        if (rr >= X - K)
                            *reinterpret_cast<float4 *>(a.h.send_corner[RIGHT ? 3 : 2] + (rr - (X - K)) * KC + 4 * j) = v;
                    }
                }
            }
        });
    }
};

template <int K>
__device__ __forceinline__ void bandl_wave(const BandKArgs &a, int wv, int lane, float2 *park) {
    using L = BandL<K>;
    const int band = (wv >= a.first[1]) + (wv >= a.first[2]) + (wv >= a.first[3]);
    const int w = wv - (band == 0 ? 0 : band == 1 ? a.first[1] : band == 2 ? a.first[2] : a.first[3]);
    const int X = a.rows, Y = a.cols;
    if (band < 2) {
        // does this wave hold column 0 or Y-1 of a global left / right edge?
        const int c_lo = w * L::SW - L::KE, c_hi = c_lo + 127;
        const bool cp = (!a.has[2] && c_lo <= 0 && c_hi >= 0) || (!a.has[3] && c_lo <= Y - 1 && c_hi >= Y - 1);
        if (band == 0)
            cp ? L::template rows<false, true>(a, w, lane, park) : L::template rows<false, false>(a, w, lane, park);
        else
            cp ? L::template rows<true, true>(a, w, lane, park) : L::template rows<true, false>(a, w, lane, park);
    } else {
        const int r_lo = a.rlo + w * L::SW - L::KE, r_hi = r_lo + 127;
        const bool cp = (!a.has[0] && r_lo <= 0 && r_hi >= 0) || (!a.has[1] && r_lo <= X - 1 && r_hi >= X - 1);
        if (band == 2)
            cp ? L::template cols<false, true>(a, w, lane, park) : L::template cols<false, false>(a, w, lane, park);
        else
            cp ? L::template cols<true, true>(a, w, lane, park) : L::template cols<true, false>(a, w, lane, park);
    }
}

// 8 waves per EU caps the kernel at 64 VGPRs (512 / 8)
template <int K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void bandl_kernel(BandKArgs a) {
    const int waves = gridDim.x * 4;
    const int wv0 = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (int)(threadIdx.x >> 6));
    // band waves first: beside the interior's two waves per SIMD the bands
    // (and the exchange behind them) finish early in the pass instead of
    // living on the interior's leftover issue slots until its end
    if (a.prio) __builtin_amdgcn_s_setprio(3);
    extern __shared__ float2 bandl_lds[];
    float2 *park = bandl_lds + (threadIdx.x >> 6) * (BandL<K>::NPOS * BandL<K>::PST);
    for (int wv = wv0; wv < a.first[4]; wv += waves)  // wave-uniform
        bandl_wave<K>(a, wv, threadIdx.x & 63, park);
}

// LDS each lean workgroup reserves: more than half of the CU's 160 KiB (its
// four waves park 4 x NPOS x PST float2 in it: 121.9 KiB at K = 20)
constexpr int kBandLeanLds = 122 * 1024;
static_assert(4 * BandL<SWEEPD_MAX>::NPOS * BandL<SWEEPD_MAX>::PST * 8 <= kBandLeanLds,
              "lean band kernel: LDS park too small");
static_assert(kBandLeanLds > 80 * 1024 && kBandLeanLds <= 160 * 1024, "one lean workgroup per CU");

template <int K>
int bandl_launch_impl(const BandKArgs &a, int blocks, hipStream_t s, hipEvent_t start, hipEvent_t stop) {
    // (once per process, thread-safe: the reservation exceeds the 64 KiB a
    // launch may request without it)
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void *>(&bandl_kernel<K>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, kBandLeanLds);
    SMI_HIP_CHECK(attr);
    if (start || stop)
        hipExtLaunchKernelGGL((bandl_kernel<K>), dim3(blocks), dim3(256), kBandLeanLds, s, start, stop, 0, a);
    else
        hipLaunchKernelGGL((bandl_kernel<K>), dim3(blocks), dim3(256), kBandLeanLds, s, a);
    SMI_HIP_CHECK(hipGetLastError());
    return SMI_SUCCESS;
}

template <int K>
int bandk_launch_impl(const BandKArgs &a, int waves, hipStream_t s, hipEvent_t start, hipEvent_t stop) {
    if (start || stop)  // events carried by the dispatch itself (no marker packets around it)
        hipExtLaunchKernelGGL((bandk_kernel<K>), dim3((waves + 3) / 4), dim3(256), 0, s, start, stop, 0, a);
    else
        hipLaunchKernelGGL((bandk_kernel<K>), dim3((waves + 3) / 4), dim3(256), 0, s, a);
    SMI_HIP_CHECK(hipGetLastError());
    return SMI_SUCCESS;
}

}  // namespace smi

#define SMI_BANDK_INSTANCE(K)                                                                            \
    namespace smi {                                                                                      \
    int bandk_launch_k##K(const BandKArgs &a, int waves, hipStream_t s, hipEvent_t start,                \
                          hipEvent_t stop) {                                                             \
        return bandk_launch_impl<K>(a, waves, s, start, stop);                                           \
    }                                                                                                    \
    }

#define SMI_BANDL_INSTANCE(K)                                                                            \
    namespace smi {                                                                                      \
    int bandl_launch_k##K(const BandKArgs &a, int blocks, hipStream_t s, hipEvent_t start,               \
                          hipEvent_t stop) {                                                             \
        return bandl_launch_impl<K>(a, blocks, s, start, stop);                                          \
    }                                                                                                    \
    }
