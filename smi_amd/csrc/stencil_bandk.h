// stencil_bandk.h -- the halo-facing bands of a multi-rank K-step pass as
// short register walks (instantiated per K beside sweepk_kernel<K> in
// stencilk_k<K>.hip).
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
// Shape.  The kernel runs beside the interior sweep on the comm stream, so
// what it costs the interior is the wave slots it holds times how long it
// holds them.  Round 2's ring kernel dealt the bands to 512 LDS workgroups
// (2048 waves, K barrier-separated levels each): it took ~30 us alone and up
// to 80 us beside the interior, and took every slot the interior needed -- an
// interior rank ran at 0.74-0.81 of a lone tile (profiles/r02/rehearsal/).
// Here one wave walks a short run of rows down a column window, every input
// row advancing K register-resident levels (the sweep's 3-slot rings).  Beside
// the interior, which keeps HBM saturated, every load round trip takes
// microseconds: a walk that loads its rows a batch ahead spent ~140 us per
// pass in 16 dependent round trips (profiles/r03/).  So a wave first issues
// LDS-DMA loads of ALL its input rows (1 KiB each, no VGPRs held) -- one
// round trip -- and then walks them from LDS:
//   top / bottom band: one 256-column window per wave (KC-column aprons),
//     input rows [-K, 2K) -> output rows [0, K)   (3K rows walked)
//   left / right band: four 64-column sub-windows per wave, each walking its
//     own block of hb rows (hb + 2K rows walked), storing the KC band columns
//     (the DPP neighbour shifts run across the whole wave: a sub-window's edge
//     lanes receive the next sub-window's values, and those lanes are apron)
// About 200 waves of 60-odd rows each at 8192^2, K = 12.
#pragma once

#include "stencilk.h"

namespace smi {

// extended-tile address of the 4 cells (r, c..c+3), c a multiple of 4, r in
// [-K, X+K), c in [-KC, Y+KC): tile, side halo, or corner block.  Rows /
// columns beyond a global edge (no neighbour there) are clamped onto the
// tile: those cells only ever feed cells the copy rule overrides.
__device__ __forceinline__ const float4 *band_addr(const BandKArgs &a, int K, int r, int c) {
    const int X = a.rows, Y = a.cols, KC = a.kc;
    r = min(max(r, a.has[0] ? -K : 0), a.has[1] ? X + K - 1 : X - 1);
    c = min(max(c, a.has[2] ? -KC : 0), a.has[3] ? Y + KC - 4 : Y - 4);
    const bool rin = r >= 0 && r < X, cin = c >= 0 && c < Y;
    const int rt = min(max(r, 0), X - 1), ct = min(max(c, 0), Y - 4);
    const int hr = r < 0 ? r + K : r - X;  // halo row (valid when !rin)
    const int hc = c < 0 ? c + KC : c - Y; // halo column (valid when !cin)
    const float *tile = a.in + (size_t)rt * Y + ct;
    const float *vert = (r < 0 ? a.h.top : a.h.bot) + (size_t)max(hr, 0) * Y + ct;
    const float *horz = (c < 0 ? a.h.left : a.h.right) + (size_t)rt * KC + max(hc, 0);
    const float *cb = r < 0 ? (c < 0 ? a.h.corner[0] : a.h.corner[1]) : (c < 0 ? a.h.corner[2] : a.h.corner[3]);
    const float *corn = cb + max(hr, 0) * KC + max(hc, 0);
    const float *p = (rin && cin) ? tile : rin ? horz : cin ? vert : corn;
    return reinterpret_cast<const float4 *>(p);
}

template <int K>
struct BandK {
    static constexpr int LL = (K + 3) / 4;  // apron lanes per window side (4 LL = KC >= K columns)
    static constexpr int PRO = 2 * K + 1;   // prologue rows (the last one stores the first output row)

    const BandKArgs &a;  // the kernel argument (a copy would live in scratch)
    __device__ BandK(const BandKArgs &args) : a(args) {}
    int rb;           // input row of t = 0 (this lane's sub-window: o0 - K)
    int o1;           // end of this lane's output rows
    int c;            // first column of this lane's 4 cells
    bool st;          // this lane stores (band columns, live sub-window)
    bool copyL, copyR, gT, gB;
    float4 W[K][3];   // level 0..K-1, slot = input row index mod 3

    float4 *rows_lds;    // this wave's input rows in LDS: row t at rows_lds[t * 64 + lane]
    unsigned rows_m0;    // their LDS byte address (wave-uniform)

    __device__ __forceinline__ float4 ld(int t) const { return rows_lds[t * 64 + (threadIdx.x & 63)]; }

    // LDS-DMA of input row t: lane i's 16 bytes (from wherever band_addr
    // finds them: tile, halo or corner block) land at rows_m0 + 1024 t + 16 i
    // (cdna_hip_programming.md, LDS-DMA recipe: M0 set and restored in the
    // same statement)
    __device__ __forceinline__ void dma(int t) const {
        const float4 *src = band_addr(a, K, rb + t, c);
        const unsigned dst = __builtin_amdgcn_readfirstlane(rows_m0 + 1024u * (unsigned)t);
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(src), "s"(dst)
                     : "memory");
    }

    // level step at row i with the global-edge copy rule per cell
    __device__ __forceinline__ float4 step(int i, const float4 &n, const float4 &m, const float4 &s) const {
        const float w = shr1_any(m.w);
        const float e = shl1_any(m.x);
        float4 o;
        o.x = jacobi(s.x, w, m.y, n.x);
        o.y = jacobi(s.y, m.x, m.z, n.y);
        o.z = jacobi(s.z, m.y, m.w, n.z);
        o.w = jacobi(s.w, m.z, e, n.w);
        const bool rcopy = (i == 0 && gT) || (i == a.rows - 1 && gB);
        o.x = (rcopy || copyL) ? m.x : o.x;
        o.y = rcopy ? m.y : o.y;
        o.z = rcopy ? m.z : o.z;
        o.w = (rcopy || copyR) ? m.w : o.w;
        return o;
    }

    // level l at input t from the level l-1 rows of inputs t-2 (N), t-1, t (S)
    template <int PH>
    __device__ __forceinline__ float4 level(int l, int t, const float4 (&P)[3]) const {
        return step(rb + t - l, P[(PH + 1) % 3], P[(PH + 2) % 3], P[PH]);
    }

    __device__ __forceinline__ void store(int t, const float4 &v) const {
        const int j = rb + K + (t - 2 * K);  // output row o0 + t - 2K
        if (!st || j >= o1) return;
        const int X = a.rows, Y = a.cols, KC = a.kc;
        *reinterpret_cast<float4 *>(a.out + (size_t)j * Y + c) = v;
        if (!a.pack) return;
        // tee the next exchange's sends: columns [0, KC) / [Y-KC, Y) packed
        // [row][KC], and the K x KC corner blocks
        const bool L = c < KC, R = c >= Y - KC;
        const int q = L ? c : c - (Y - KC);
        if (L || R) {
            *reinterpret_cast<float4 *>((L ? a.h.send_left : a.h.send_right) + (size_t)j * KC + q) = v;
            if (j < K) *reinterpret_cast<float4 *>((L ? a.h.send_corner[0] : a.h.send_corner[1]) + j * KC + q) = v;
            if (j >= X - K)
                *reinterpret_cast<float4 *>((L ? a.h.send_corner[2] : a.h.send_corner[3]) + (j - (X - K)) * KC + q) = v;
        }
    }

    template <int PH>
    __device__ __forceinline__ void advance(int t, const float4 &x) {
        W[0][PH] = x;
        float4 v;
        static_for<K>([&](auto L) {
            constexpr int l = L + 1;
            v = level<PH>(l, t, W[l - 1]);
            if constexpr (l < K) W[l][PH] = v;
        });
        store(t, v);
    }

    __device__ __forceinline__ void run(int n_in) {
        // every input row in flight at once, one wait (hipcc does not count
        // the asm loads: the wait is explicit)
        for (int t = 0; t < n_in; ++t) dma(t);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // prologue: input rows 0 .. 2K (n_in >= 3K > 2K), level l from input 2l on
        static_for<PRO>([&](auto T) {
            constexpr int t = T;
            W[0][t % 3] = ld(t);
            float4 v;
            static_for<K>([&](auto L) {
                constexpr int l = L + 1;
                if constexpr (t >= 2 * l) {
                    v = level<t % 3>(l, t, W[l - 1]);
                    if constexpr (l < K) W[l][t % 3] = v;
                }
            });
            if constexpr (t == 2 * K) store(t, v);
        });
        // steady state: batches of 3 rows, LDS reads one batch ahead (n_in
        // is wave-uniform; reads past the end hit spare rows, never used)
        float4 A[3], B[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) A[u] = ld(PRO + u);
        for (int t = PRO; t < n_in; t += 6) {
#pragma unroll
            for (int u = 0; u < 3; ++u) B[u] = ld(t + 3 + u);
            static_for<3>([&](auto V) {
                if (t + V < n_in) advance<(PRO + V) % 3>(t + V, A[V]);
            });
            if (t + 3 >= n_in) break;
#pragma unroll
            for (int u = 0; u < 3; ++u) A[u] = ld(t + 6 + u);
            static_for<3>([&](auto V) {
                if (t + 3 + V < n_in) advance<(PRO + 3 + V) % 3>(t + 3 + V, B[V]);
            });
        }
    }
};

// rows per wave: top/bottom 3K, left/right hb + 2K with hb <= 2K (launch_bandk
// clamps it), + 6 spare rows for the reads one batch past the end
template <int K>
constexpr int bandk_lds_rows() { return 4 * K + 6; }

template <int K>
__global__ __launch_bounds__(64) void bandk_kernel(BandKArgs a) {
    using B = BandK<K>;
    constexpr int LL = B::LL;
    __shared__ float4 rows_lds[bandk_lds_rows<K>() * 64];
    const int wv = blockIdx.x;
    const int band = (wv >= a.first[1]) + (wv >= a.first[2]) + (wv >= a.first[3]);
    const int lw = wv - (band == 0 ? 0 : band == 1 ? a.first[1] : band == 2 ? a.first[2] : a.first[3]);
    const int lane = threadIdx.x;
    const int X = a.rows, Y = a.cols;
    B w(a);
    w.rows_lds = rows_lds;
    w.rows_m0 = __builtin_amdgcn_readfirstlane(
        (unsigned)(uintptr_t)(__attribute__((address_space(3))) float4 *)(rows_lds));
    int o0, n_in;
    if (band < 2) {
        // top / bottom: window lw stores columns [lw sw, (lw + 1) sw)
        w.c = lw * a.sw - 4 * LL + 4 * lane;
        o0 = band == 0 ? 0 : X - K;
        w.o1 = o0 + K;
        n_in = 3 * K;
        w.st = lane >= LL && lane < 64 - LL && w.c < Y;
    } else {
        // left / right: sub-window (lw, lane / 16) of 16 lanes, hb rows
        const int li = lane & 15, sub = lw * 4 + (lane >> 4);
        w.c = (band == 2 ? -4 * LL : Y + 4 * LL - 64) + 4 * li;
        o0 = a.rlo + sub * a.hb;
        w.o1 = min(o0 + a.hb, a.rhi);
        n_in = a.hb + 2 * K;
        w.st = li >= LL && li < 16 - LL && sub < a.nsub && (band == 2 ? w.c < a.kc : w.c >= Y - a.kc);
    }
    w.rb = o0 - K;
    w.gT = !a.has[0];
    w.gB = !a.has[1];
    w.copyL = !a.has[2] && w.c == 0;
    w.copyR = !a.has[3] && w.c + 4 == Y;
    w.run(n_in);
}

template <int K>
int bandk_launch_impl(const BandKArgs &a, int waves, hipStream_t s) {
    hipLaunchKernelGGL((bandk_kernel<K>), dim3(waves), dim3(64), 0, s, a);
    SMI_HIP_CHECK(hipGetLastError());
    return SMI_SUCCESS;
}

}  // namespace smi

#define SMI_BANDK_INSTANCE(K)                                                                            \
    namespace smi {                                                                                      \
    int bandk_launch_k##K(const BandKArgs &a, int waves, hipStream_t s) {                                \
        return bandk_launch_impl<K>(a, waves, s);                                                        \
    }                                                                                                    \
    }
