// stencilk.hip -- K Jacobi steps per pass over HBM (deep temporal blocking).
//
// Same per-cell arithmetic as every other stencil kernel here
// (stencil_smi.cl:153-156, global-edge cells copied per :143-151), applied K
// times inside one streaming pass.  Each wave owns a 256-column window of the
// input and walks it down the rows; every incoming input row advances a
// pipeline of K levels (level l lags l rows behind the input, each keeping a
// two-row window in registers), and only level K is stored.  The window is
// 256 input columns wide but outputs only the central 256-2K: each level
// loses one valid column on each side, so adjacent windows overlap by 2K
// columns instead of fetching strip-edge extras (no cross-lane broadcasts,
// 1.6 % redundant columns at K=4).  HBM traffic per pass is that of a single
// step, so the algorithmic 8 B/cell/step are moved up to K times faster.
//
// The kernel computes an arbitrary output rectangle [row_lo,row_hi) x
// [col_lo,col_hi) of the tile from input rows/columns within K of it, so the
// same kernel is the single-tile sweep (whole tile) and, in multi-rank runs,
// the interior sweep that stays K cells clear of every halo-facing side.
#include "stencil_common.h"

namespace smi {

template <int K, int U, bool NT>
__global__ __launch_bounds__(256) void sweepk_kernel(const float *__restrict__ in, float *__restrict__ out,
                                                     SweepKArgs a, int nstrips, int nrb, int ht) {
    static_assert(K % 4 == 0 && K >= 4 && K <= 16, "K must be a multiple of 4 (float4 lanes)");
    constexpr int SW = 256 - 2 * K;  // output columns per window
    constexpr int LL = K / 4;        // lanes on each side that never store
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int lane = threadIdx.x & 63;
    const int task = __builtin_amdgcn_readfirstlane(lb * 4 + (int)(threadIdx.x >> 6));
    const int rb = task / nstrips;
    const int strip = task - rb * nstrips;
    if (rb >= nrb) return;  // wave-uniform

    const int rows = a.rows, cols = a.cols;
    const int o0 = a.row_lo + rb * ht;
    const int o1 = min(o0 + ht, a.row_hi);
    const int cs = a.col_lo + strip * SW;
    const int cb = cs - K + 4 * lane;                 // this lane's first column
    const int cl = min(max(cb, 0), cols - 4);         // clamped load column
    const bool st = lane >= LL && lane < 64 - LL && cb < a.col_hi;
    const bool copyL = a.gL && cb == 0;
    const bool copyR = a.gR && cb + 4 == cols;
    const bool gT = a.gT, gB = a.gB;

    auto ld = [&](int r) -> float4 {
        const size_t i = (size_t)min(max(r, 0), rows - 1) * cols + cl;
        return *reinterpret_cast<const float4 *>(in + i);
    };
    // level value at row i from (N, C, S) of the level below
    auto step = [&](int i, const float4 &n, const float4 &c, const float4 &s) -> float4 {
        const bool rcopy = (i == 0 && gT) || (i == rows - 1 && gB);
        const float w = wave_shr1(c.w);
        const float e = wave_shl1(c.x);
        float4 o;
        o.x = jacobi(s.x, w, c.y, n.x);
        o.y = jacobi(s.y, c.x, c.z, n.y);
        o.z = jacobi(s.z, c.y, c.w, n.z);
        o.w = jacobi(s.w, c.z, e, n.w);
        o.x = (rcopy || copyL) ? c.x : o.x;
        o.y = rcopy ? c.y : o.y;
        o.z = rcopy ? c.z : o.z;
        o.w = (rcopy || copyR) ? c.w : o.w;
        return o;
    };

    // P[l][0], P[l][1]: level-l rows (r-l-2, r-l-1) when input row r arrives
    float4 P[K][2];
#pragma unroll
    for (int l = 0; l < K; ++l) P[l][0] = P[l][1] = make_float4(0.f, 0.f, 0.f, 0.f);

    // Push input row r through the K levels.  The first 2K rows only prime
    // the pipeline (their level-K rows lie above o0 and are not stored).
    auto advance = [&](int r, const float4 &x) {
        float4 s = x;
#pragma unroll
        for (int l = 1; l <= K; ++l) {
            const float4 v = step(r - l, P[l - 1][0], P[l - 1][1], s);
            P[l - 1][0] = P[l - 1][1];
            P[l - 1][1] = s;
            s = v;
        }
        const int j = r - K;
        if (j >= o0 && st) {
            float *op = out + (size_t)j * cols + cb;
            store4<NT>(op, s);
        }
    };

    const int r_begin = o0 - K, r_end = o1 + K;  // input rows [r_begin, r_end)
    float4 A[U];
#pragma unroll
    for (int u = 0; u < U; ++u) A[u] = ld(min(r_begin + u, r_end - 1));
    for (int r = r_begin; r < r_end; r += U) {
        float4 B[U];
        const bool more = r + U < r_end;  // uniform
        if (more) {
#pragma unroll
            for (int u = 0; u < U; ++u) B[u] = ld(min(r + U + u, r_end - 1));
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (r + u < r_end) advance(r + u, A[u]);
        if (more) {
#pragma unroll
            for (int u = 0; u < U; ++u) A[u] = B[u];
        }
    }
}

template <int K, int U>
static void launch_k(const SweepKArgs &a, int nstrips, int nrb, int ht, int blocks, bool nt, hipStream_t s) {
    if (nt)
        hipLaunchKernelGGL((sweepk_kernel<K, U, true>), dim3(blocks), dim3(256), 0, s, a.in, a.out, a, nstrips,
                           nrb, ht);
    else
        hipLaunchKernelGGL((sweepk_kernel<K, U, false>), dim3(blocks), dim3(256), 0, s, a.in, a.out, a, nstrips,
                           nrb, ht);
}

template <int K>
static int launch_k_u(const SweepKArgs &a, int nstrips, int nrb, int ht, int blocks, int u, bool nt,
                      hipStream_t s) {
    switch (u) {
    case 2: launch_k<K, 2>(a, nstrips, nrb, ht, blocks, nt, s); break;
    case 4: launch_k<K, 4>(a, nstrips, nrb, ht, blocks, nt, s); break;
    default: launch_k<K, 8>(a, nstrips, nrb, ht, blocks, nt, s); break;
    }
    return SMI_SUCCESS;
}

int launch_sweepk(int K, const SweepKArgs &a, hipStream_t s) {
    if (a.row_hi <= a.row_lo || a.col_hi <= a.col_lo) return SMI_SUCCESS;
    SMI_ARG_CHECK(a.cols % 4 == 0 && a.col_lo % 4 == 0 && a.col_hi % 4 == 0, "sweepk: columns not float4 aligned");
    SMI_ARG_CHECK(a.row_lo >= 0 && a.row_hi <= a.rows && a.col_lo >= 0 && a.col_hi <= a.cols,
                  "sweepk: output rectangle outside the tile");
    const int ht = std::max(1, g_tune.htk);
    const int sw = 256 - 2 * K;
    const int nstrips = (a.col_hi - a.col_lo + sw - 1) / sw;
    const int nrb = (a.row_hi - a.row_lo + ht - 1) / ht;
    const long tasks = (long)nstrips * nrb;
    const int blocks = (int)((tasks + 3) / 4);
    int tok = -1;
    if (prof_enabled()) SMI_TRY(prof_begin(SMI_PROF_STENCIL_SWEEP, s, &tok));
    switch (K) {
    case 4: launch_k_u<4>(a, nstrips, nrb, ht, blocks, g_tune.uk, g_tune.nt, s); break;
    case 8: launch_k_u<8>(a, nstrips, nrb, ht, blocks, g_tune.uk, g_tune.nt, s); break;
    default: set_error("sweepk: steps per pass must be 4 or 8"); return SMI_ERR_INVALID_ARG;
    }
    SMI_HIP_CHECK(hipGetLastError());
    if (tok >= 0) SMI_TRY(prof_end(tok, s));
    return SMI_SUCCESS;
}

}  // namespace smi
