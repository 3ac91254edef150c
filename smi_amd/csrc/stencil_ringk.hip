// stencil_ringk.hip -- the halo-facing ring of a K-step pass (3 <= K <= 12),
// and the global edge-column bands of any K-step pass.
//
// In a multi-rank run with K Jacobi steps per pass, every tile cell within K
// of a side that has a neighbour depends on that neighbour's cells (up to K
// rows/columns deep, plus a K x K block from each diagonal neighbour for the
// corners).  The ring kernel computes exactly those cells: the ring is cut
// into small output blocks; each workgroup loads its block plus a K-cell
// apron from the "extended tile" (tile cells, depth-K halos, corner blocks)
// into LDS, runs the K levels in LDS (the valid region shrinks by one cell
// per level), stores the block, and packs the new left/right columns and
// corner blocks for the next exchange.  The per-cell arithmetic and the
// global-edge copy rule are the sweep's (stencil_smi.cl:143-156); cells of
// the apron that lie outside the global grid are never used by a stored cell.
#include <cstdlib>

#include "stencil_common.h"

namespace smi {

// extended-tile cell (p, q), p in [-K, X+K), q in [-K, Y+K): the address it
// is read from, or nullptr where no data exists (outside the global grid:
// only ever read by unused cells).  Branch-free (selects only), so a thread's
// loads of all its cells issue back to back.
__device__ __forceinline__ const float *ext_ptr(const RingKArgs &a, int p, int q) {
    const int X = a.rows, Y = a.cols, K = a.k;
    const bool pin = p >= 0 && p < X, qin = q >= 0 && q < Y;
    const int pc = min(max(p, 0), X - 1), qc = min(max(q, 0), Y - 1);
    const int hr = p < 0 ? max(p + K, 0) : min(p - X, K - 1);  // halo row (top / bottom)
    const int hc = q < 0 ? max(q + K, 0) : min(q - Y, K - 1);  // halo column (left / right)
    const float *tile = a.in + (size_t)pc * Y + qc;
    const float *vert = (p < 0 ? a.h.top : a.h.bot) + (size_t)hr * Y + qc;
    const float *horz = (q < 0 ? a.h.left : a.h.right) + (size_t)pc * K + hc;
    const int ci = (p < 0 ? 0 : 2) + (q < 0 ? 0 : 1);  // tl, tr, bl, br
    const float *corn = a.h.corner[ci] + hr * K + hc;
    const bool has_v = p < 0 ? a.has[0] : a.has[1];
    const bool has_h = q < 0 ? a.has[2] : a.has[3];
    const float *src = (pin && qin) ? tile : qin ? (has_v ? vert : nullptr)
                       : pin ? (has_h ? horz : nullptr) : (a.has_diag[ci] ? corn : nullptr);
    return src;
}

// Output blocks: top/bottom bands in K x RB_W blocks, left/right bands in
// RB_H x K blocks (block b -> band via the prefix table in RingKArgs).  K is
// a runtime value (the depth of the current phase); LDS is sized for
// RING_KMAX.
//
// The block's H x W region (output block + K apron) is dealt to the threads
// once: thread t owns cells t, t + 256, ... (at most RING_CELLS) and keeps
// each cell's depth (distance to the region's edge: the cell is valid at
// levels 1..depth; 0 for a global-edge cell, which is copied) in a register,
// so the K level sweeps are divide- and branch-free.  (Round 1 recomputed the coordinates with a division per cell per
// level: 35 us per pass at 8192^2, K = 12, which an interior rank could not
// hide behind its 0.11 ms interior sweep -- tools/rehearsal.py measured 0.78
// of a lone tile's rate.)
constexpr int RING_REGION = 3 * RING_KMAX * ((RB_W > RB_H ? RB_W : RB_H) + 2 * RING_KMAX);

template <int NT>
__global__ __launch_bounds__(NT) void ringk_kernel(RingKArgs a) {
    constexpr int RING_CELLS = (RING_REGION + NT - 1) / NT;
    // horizontal blocks: 3K x (RB_W + 2K); vertical blocks: (RB_H + 2K) x 3K;
    // PAD floats before and after each buffer keep the neighbour reads of the
    // region's border cells inside the allocation (their results are unused)
    constexpr int LDS_N = 3 * RING_KMAX * ((RB_W > RB_H ? RB_W : RB_H) + 2 * RING_KMAX);
    constexpr int PAD = (RB_W > RB_H ? RB_W : RB_H) + 2 * RING_KMAX + 4;
    __shared__ float lds[2][LDS_N + 2 * PAD];
    const int K = a.k;
    const int b = blockIdx.x;
    int band = 0;
    while (band < 3 && b >= a.first_block[band + 1]) ++band;
    const int lb = b - a.first_block[band];
    const int r0 = a.r0[band], r1 = a.r1[band], c0 = a.c0[band], c1 = a.c1[band];
    const bool horiz = band < 2;  // top/bottom band: K rows x wide
    const int bh = horiz ? K : RB_H, bw = horiz ? RB_W : a.bandw;
    const int nbc = (c1 - c0 + bw - 1) / bw;
    const int oR0 = r0 + (lb / nbc) * bh, oC0 = c0 + (lb % nbc) * bw;
    const int oR1 = min(oR0 + bh, r1), oC1 = min(oC0 + bw, c1);
    const int H = oR1 - oR0 + 2 * K, W = oC1 - oC0 + 2 * K;
    const int pb = oR0 - K, qb = oC0 - K;  // extended coordinates of lds (0,0)
    const int X = a.rows, Y = a.cols;
    const bool gT = !a.has[0], gB = !a.has[1], gL = !a.has[2], gR = !a.has[3];
    const int n = H * W;
    float *L0 = lds[0] + PAD, *L1 = lds[1] + PAD;

    int dep[RING_CELLS];   // levels the cell is computed at (1..dep); 0 for a copied cell
#pragma unroll
    for (int j = 0; j < RING_CELLS; ++j) {
        const int i = threadIdx.x + NT * j;
        dep[j] = 0;
        if (i < n) {
            const int y = i / W, x = i - y * W;
            const int p = pb + y, q = qb + x;
            const bool copy = (p == 0 && gT) || (p == X - 1 && gB) || (q == 0 && gL) || (q == Y - 1 && gR);
            dep[j] = copy ? 0 : min(min(y, H - 1 - y), min(x, W - 1 - x));
            const float *src = (a.exp_mode & 2) ? nullptr : ext_ptr(a, p, q);
            const float v = *(src ? src : a.in);  // unconditional load (a.in: any valid address)
            L0[i] = src ? v : 0.f;
        }
    }
    __syncthreads();
    // Branch-free level sweeps: every cell of the region is rewritten each
    // level -- the new value where it is valid (depth >= l), its old value
    // elsewhere (copied cells keep theirs; cells shallower than l are never
    // read by a valid one) -- so all LDS reads of a level issue together.
#pragma unroll 1
    for (int l = 1; l <= ((a.exp_mode & 1) ? 0 : K); ++l) {
        const float *src = (l & 1) ? L0 : L1;
        float *dst = (l & 1) ? L1 : L0;
        float v[RING_CELLS];
#pragma unroll
        for (int j = 0; j < RING_CELLS; ++j) {
            const int o = min((int)threadIdx.x + NT * j, n - 1);
            const float nv = jacobi(src[o + W], src[o - 1], src[o + 1], src[o - W]);
            v[j] = dep[j] >= l ? nv : src[o];
        }
#pragma unroll
        for (int j = 0; j < RING_CELLS; ++j) {
            const int o = threadIdx.x + NT * j;
            if (o < n) dst[o] = v[j];
        }
        __syncthreads();
    }
    const float *res = (K & 1) ? L1 : L0;
#pragma unroll
    for (int j = 0; j < RING_CELLS; ++j) {
        const int o = threadIdx.x + NT * j;
        if (o >= n || (a.exp_mode & 4)) continue;
        const int y = o / W, x = o - y * W;
        if (y < K || y >= H - K || x < K || x >= W - K) continue;  // apron cell: not an output
        const int p = pb + y, q = qb + x;
        const float v = res[o];
        a.out[(size_t)p * Y + q] = v;
        if (!a.pack) continue;
        if (q < K) a.h.send_left[(size_t)p * K + q] = v;
        if (q >= Y - K) a.h.send_right[(size_t)p * K + (q - (Y - K))] = v;
        if (p < K || p >= X - K) {
            const int pi = p < K ? p : p - (X - K);
            if (q < K) a.h.send_corner[p < K ? 0 : 2][pi * K + q] = v;
            if (q >= Y - K) a.h.send_corner[p < K ? 1 : 3][pi * K + (q - (Y - K))] = v;
        }
    }
}

// Initial depth-K sends from the current tile: columns 0..K-1 and Y-K..Y-1
// packed [row][k], and the four K x K corner blocks.
__global__ __launch_bounds__(256) void packk_kernel(const float *in, int X, int Y, int K, HaloK h) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= X * K) return;
    const int p = t / K, k = t - p * K;
    const float *row = in + (size_t)p * Y;
    const float vl = row[k], vr = row[Y - K + k];
    h.send_left[t] = vl;
    h.send_right[t] = vr;
    if (p < K) {
        h.send_corner[0][p * K + k] = vl;
        h.send_corner[1][p * K + k] = vr;
    }
    if (p >= X - K) {
        h.send_corner[2][(p - (X - K)) * K + k] = vl;
        h.send_corner[3][(p - (X - K)) * K + k] = vr;
    }
}

int launch_ringk(RingKArgs a, hipStream_t s) {
    const int X = a.rows, Y = a.cols, K = a.k;
    // left/right bands are K rounded up to whole float4 columns wide, so the
    // interior sweep's column range stays 16-byte aligned
    const int W = 4 * ((K + 3) / 4);
    a.bandw = W;
    SMI_ARG_CHECK(K >= 1 && K <= RING_KMAX, "ring: K must be 1..12");
    SMI_ARG_CHECK(X >= 2 * K && Y >= 2 * W, "ring: tile smaller than 2K x 2W");
    // bands: top rows [0,K), bottom rows [X-K,X) (full width); left/right
    // columns [0,W) / [Y-W,Y) over the rows the top/bottom bands leave.
    // band[k]: side k facing a halo, or a global edge column the interior
    // sweep leaves to this kernel (its copy rule, stencil_smi.cl:143-151)
    const int rlo = a.band[0] ? K : 0, rhi = a.band[1] ? X - K : X;
    const int band_r0[4] = {0, X - K, rlo, rlo}, band_r1[4] = {K, X, rhi, rhi};
    const int band_c0[4] = {0, 0, 0, Y - W}, band_c1[4] = {Y, Y, W, Y};
    int nb = 0;
    for (int k = 0; k < 4; ++k) {
        a.r0[k] = band_r0[k];
        a.r1[k] = band_r1[k];
        a.c0[k] = band_c0[k];
        a.c1[k] = band_c1[k];
        a.first_block[k] = nb;
        if (!a.band[k] || a.r1[k] <= a.r0[k]) continue;
        const bool horiz = k < 2;
        const int bh = horiz ? K : RB_H, bw = horiz ? RB_W : W;
        nb += ((a.r1[k] - a.r0[k] + bh - 1) / bh) * ((a.c1[k] - a.c0[k] + bw - 1) / bw);
    }
    a.first_block[4] = nb;
    if (nb == 0) return SMI_SUCCESS;
    a.exp_mode = 0;
#ifdef SMI_LOOPBACK_REHEARSAL
    if (const char *e = getenv("SMI_RING_EXP")) a.exp_mode = atoi(e);
#endif
    int tok = -1;
    if (prof_enabled()) SMI_TRY(prof_begin(SMI_PROF_STENCIL_EDGE, s, &tok));
    int nt = 256;
#ifdef SMI_LOOPBACK_REHEARSAL
    if (const char *e = getenv("SMI_RING_THREADS")) nt = atoi(e);
#endif
    if (nt == 64)
        hipLaunchKernelGGL(ringk_kernel<64>, dim3(nb), dim3(64), 0, s, a);
    else if (nt == 128)
        hipLaunchKernelGGL(ringk_kernel<128>, dim3(nb), dim3(128), 0, s, a);
    else
        hipLaunchKernelGGL(ringk_kernel<256>, dim3(nb), dim3(256), 0, s, a);
    SMI_HIP_CHECK(hipGetLastError());
    if (tok >= 0) SMI_TRY(prof_end(tok, s));
    return SMI_SUCCESS;
}

int launch_packk(const float *in, int rows, int cols, int K, const HaloK &h, hipStream_t s) {
    const int n = rows * K;
    hipLaunchKernelGGL(packk_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, rows, cols, K, h);
    SMI_HIP_CHECK(hipGetLastError());
    return SMI_SUCCESS;
}

#ifdef SMI_LOOPBACK_REHEARSAL
// Rehearsal build only: the 8-way loopback exchange as ONE copy kernel (an
// RCCL send/recv group is one kernel launch too), so tools/rehearsal.py can
// price the exchange without the in-process transport's per-message events.
struct CopySegs {
    const float4 *src[8];
    float4 *dst[8];
    int n4[8];
};
__global__ __launch_bounds__(256) void multicopy_kernel(CopySegs c, int nseg, int blocks_per_seg) {
    const int seg = blockIdx.x / blocks_per_seg;
    if (seg >= nseg) return;
    const int b = blockIdx.x - seg * blocks_per_seg;
    for (int i = b * 256 + threadIdx.x; i < c.n4[seg]; i += blocks_per_seg * 256) c.dst[seg][i] = c.src[seg][i];
}
int launch_multicopy(const float *const *src, float *const *dst, const size_t *bytes, int nseg, hipStream_t s) {
    CopySegs c{};
    for (int i = 0; i < nseg && i < 8; ++i) {
        c.src[i] = reinterpret_cast<const float4 *>(src[i]);
        c.dst[i] = reinterpret_cast<float4 *>(dst[i]);
        c.n4[i] = (int)(bytes[i] / 16);
    }
    const int bps = 8;
    hipLaunchKernelGGL(multicopy_kernel, dim3(bps * nseg), dim3(256), 0, s, c, nseg, bps);
    SMI_HIP_CHECK(hipGetLastError());
    return SMI_SUCCESS;
}
#endif

}  // namespace smi
