// stencil_bands.hip -- the halo-facing bands of a multi-rank K-step pass as
// register sweeps (the ring kernel's job, stencil_ringk.hip, done by
// sweepk_kernel<K>).
//
// Same cells, same arithmetic (stencil_smi.cl:143-156 through the K-step
// sweep), same halo inputs: the band cells within K of a halo-facing side
// need depth-K halos and K x K corner blocks.  The LDS ring kernel computes
// them in 512 small workgroups whose K barrier-separated levels take ~30 us
// and whose waves cannot share a SIMD with the interior sweep's (248 VGPRs
// each), so an interior rank ran at ~0.78 of a lone tile.  Here the bands'
// inputs are gathered into two small images, each band is a rectangle of an
// image, and sweepk_kernel<K> sweeps those rectangles with few tall row
// blocks (~100 waves); the interior sweep is sized to leave them their slots
// (BAND_RESERVE_WAVES), so the two run side by side.
//
// Status: an experiment, off by default (SMI_RING_MODE=1 selects it).  It is
// bit-identical to the LDS ring (the multi-rank parity suite passes in both
// modes) but slower on an interior rank: run beside the interior sweep, which
// saturates HBM, its six small dependent kernels are latency-bound (about
// 350 us per pass end to end against 30 us for the LDS ring).
//
// H image (6K rows x wi columns, wi = la + Y + ra, la/ra = KC where a
// left/right neighbour exists, else 0): rows [0, 3K) = extended rows
// [-K, 2K), rows [3K, 6K) = extended rows [X-2K, X+K); image column j holds
// extended column j - la.  Output rows [K, 5K): the top band is image rows
// [K, 2K), the bottom band [4K, 5K); rows [2K, 4K) mix the two parts and are
// discarded (their cones never reach a kept row).  Global column edges are the
// image's own edges (la / ra = 0 there), so the sweep's edge rule applies.
// V image (X rows x 6KC columns): columns [0, 3KC) = extended columns
// [-KC, 2KC), [3KC, 6KC) = [Y-2KC, Y+KC); output columns [KC, 5KC) and the
// rows the left/right bands cover; global row edges are the image's.
#include <algorithm>

#include "stencil_common.h"

namespace smi {

static int kc_of(int K) { return 4 * ((K + 3) / 4); }

bool bands_eligible(int rows, int cols, int K) {
    // the H image's two parts must not reach the tile's opposite global edge
    // row, nor the V image's parts its opposite edge column
    return K >= SWEEPK_MIN && K <= SWEEPK_MAX && rows > 2 * K && cols > 2 * kc_of(K) && cols % 4 == 0;
}

size_t band_images_elems(int rows, int cols, int K) {
    const int KC = kc_of(K);
    const size_t h = (size_t)6 * K * (cols + 2 * KC), v = (size_t)rows * 6 * KC;
    return 2 * h + 2 * v + 16;
}

BandImages band_images_at(float *base, int rows, int cols, int K) {
    const int KC = kc_of(K);
    const size_t h = (size_t)6 * K * (cols + 2 * KC), v = (size_t)rows * 6 * KC;
    BandImages im;
    // 16-byte aligned sub-buffers (every size above is a multiple of 4 floats)
    im.h_in = base;
    im.h_out = im.h_in + h;
    im.v_in = im.h_out + h;
    im.v_out = im.v_in + v;
    return im;
}

// extended-tile cell (p, q) -> its address, nullptr where no data exists
// (the same selection as the ring kernel's; cells beyond a halo's depth are
// clamped onto it -- they never reach a kept cell)
__device__ __forceinline__ const float *band_src(const RingKArgs &a, int p, int q) {
    const int X = a.rows, Y = a.cols, K = a.k;
    const bool pin = p >= 0 && p < X, qin = q >= 0 && q < Y;
    const int pc = min(max(p, 0), X - 1), qc = min(max(q, 0), Y - 1);
    const int hr = p < 0 ? max(p + K, 0) : min(p - X, K - 1);
    const int hc = q < 0 ? max(q + K, 0) : min(q - Y, K - 1);
    const int ci = (p < 0 ? 0 : 2) + (q < 0 ? 0 : 1);
    if (pin && qin) return a.in + (size_t)pc * Y + qc;
    if (qin) return (p < 0 ? a.has[0] : a.has[1]) ? (p < 0 ? a.h.top : a.h.bot) + (size_t)hr * Y + qc : nullptr;
    if (pin) return (q < 0 ? a.has[2] : a.has[3]) ? (q < 0 ? a.h.left : a.h.right) + (size_t)pc * K + hc : nullptr;
    return a.has_diag[ci] ? a.h.corner[ci] + hr * K + hc : nullptr;
}

// float4 group (4 cells) of an extended row p from column q on (q, Y, the
// images' apron and part widths are multiples of 4): one aligned 16-byte load
// when the group lies inside [0, Y) (tile or top/bottom halo row), else per
// element (left/right halos, corners)
__device__ __forceinline__ float4 band_group(const RingKArgs &a, int p, int q) {
    if (q >= 0 && q + 4 <= a.cols) {
        const float *src = band_src(a, p, q);
        return src ? *reinterpret_cast<const float4 *>(src) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float e[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float *src = band_src(a, p, q + k);
        e[k] = src ? *src : 0.f;
    }
    return make_float4(e[0], e[1], e[2], e[3]);
}

// Gather, 32-bit index math only.  H image: blockIdx.y walks image rows
// (uniform per workgroup), threads the row's float4 groups.  V image: each
// row is 6KC/4 groups; a thread keeps one group column and walks rows.
__global__ __launch_bounds__(256) void band_gather_h_kernel(RingKArgs a, BandImages im, int wi, int la) {
    const int X = a.rows, K = a.k;
    const int groups = wi >> 2;
    for (int r = blockIdx.y; r < 6 * K; r += gridDim.y) {
        const int p = r < 3 * K ? r - K : X - 2 * K + (r - 3 * K);
        for (int g = blockIdx.x * 256 + threadIdx.x; g < groups; g += gridDim.x * 256)
            *reinterpret_cast<float4 *>(im.h_in + (size_t)r * wi + 4 * g) = band_group(a, p, 4 * g - la);
    }
}
__global__ __launch_bounds__(256) void band_gather_v_kernel(RingKArgs a, BandImages im) {
    const int X = a.rows, Y = a.cols, K = a.k, KC = 4 * ((K + 3) / 4);
    const int gpr = (6 * KC) >> 2;                  // groups per image row
    const int rows_per_it = 256 / gpr;              // rows a workgroup covers per iteration
    const int t = threadIdx.x, dr = t / gpr, g = t - dr * gpr;
    if (dr >= rows_per_it) return;
    const int j = 4 * g;
    const int q = j < 3 * KC ? j - KC : Y - 2 * KC + (j - 3 * KC);
    for (int r = blockIdx.x * rows_per_it + dr; r < X; r += gridDim.x * rows_per_it)
        *reinterpret_cast<float4 *>(im.v_in + (size_t)r * 6 * KC + j) = band_group(a, r, q);
}

// the next exchange's packed sends for band cell (p, q) = v
__device__ __forceinline__ void band_pack(const RingKArgs &a, int p, int q, float v) {
    const int X = a.rows, Y = a.cols, K = a.k;
    if (q < K) a.h.send_left[(size_t)p * K + q] = v;
    if (q >= Y - K) a.h.send_right[(size_t)p * K + (q - (Y - K))] = v;
    if (p < K || p >= X - K) {
        const int pi = p < K ? p : p - (X - K);
        if (q < K) a.h.send_corner[p < K ? 0 : 2][pi * K + q] = v;
        if (q >= Y - K) a.h.send_corner[p < K ? 1 : 3][pi * K + (q - (Y - K))] = v;
    }
}

// Scatter: band cells back into the tile (float4 groups) plus the packed
// sends for the groups within K of a left/right edge.  Top/bottom bands:
// blockIdx.y walks the 2K band rows; left/right bands: like the V gather.
__global__ __launch_bounds__(256) void band_scatter_h_kernel(RingKArgs a, BandImages im, int wi, int la) {
    const int X = a.rows, Y = a.cols, K = a.k;
    const int groups = Y >> 2;
    for (int r = blockIdx.y; r < 2 * K; r += gridDim.y) {
        const bool top = r < K;
        if (!(top ? a.band[0] : a.band[1])) continue;  // uniform
        const int p = top ? r : X - 2 * K + r;
        const int ir = top ? K + r : 3 * K + r;  // image row: top band rows [K,2K), bottom [4K,5K)
        for (int g = blockIdx.x * 256 + threadIdx.x; g < groups; g += gridDim.x * 256) {
            const int q = 4 * g;
            const float4 v = *reinterpret_cast<const float4 *>(im.h_out + (size_t)ir * wi + la + q);
            *reinterpret_cast<float4 *>(a.out + (size_t)p * Y + q) = v;
            if (a.pack && (q < K || q + 4 > Y - K)) {
                band_pack(a, p, q, v.x);
                band_pack(a, p, q + 1, v.y);
                band_pack(a, p, q + 2, v.z);
                band_pack(a, p, q + 3, v.w);
            }
        }
    }
}
__global__ __launch_bounds__(256) void band_scatter_v_kernel(RingKArgs a, BandImages im, int rlo, int rhi) {
    const int Y = a.cols, K = a.k, KC = 4 * ((K + 3) / 4);
    const int gps = KC >> 2;                        // groups per band row and side
    const int gpr = 2 * gps;
    const int rows_per_it = 256 / gpr;
    const int t = threadIdx.x, dr = t / gpr, g = t - dr * gpr;
    if (dr >= rows_per_it) return;
    const bool left = g < gps;
    if (!(left ? a.band[2] : a.band[3])) return;
    const int c = 4 * (left ? g : g - gps);
    const int q = left ? c : Y - KC + c;
    const int j = left ? KC + c : 4 * KC + c;       // image column
    for (int p = rlo + blockIdx.x * rows_per_it + dr; p < rhi; p += gridDim.x * rows_per_it) {
        const float4 v = *reinterpret_cast<const float4 *>(im.v_out + (size_t)p * 6 * KC + j);
        *reinterpret_cast<float4 *>(a.out + (size_t)p * Y + q) = v;
        if (a.pack) {
            band_pack(a, p, q, v.x);
            band_pack(a, p, q + 1, v.y);
            band_pack(a, p, q + 2, v.z);
            band_pack(a, p, q + 3, v.w);
        }
    }
}

int launch_ring_bands(const RingKArgs &a, const BandImages &im, hipStream_t s) {
    const int X = a.rows, Y = a.cols, K = a.k, KC = kc_of(K);
    SMI_ARG_CHECK(bands_eligible(X, Y, K), "ring bands: tile too small for the band sweep");
    if (!(a.band[0] || a.band[1] || a.band[2] || a.band[3])) return SMI_SUCCESS;
    const int la = a.has[2] ? KC : 0, ra = a.has[3] ? KC : 0, wi = la + Y + ra;
    const int rlo = a.band[0] ? K : 0, rhi = a.band[1] ? X - K : X;
    int tok = -1;
    if (prof_enabled()) SMI_TRY(prof_begin(SMI_PROF_STENCIL_EDGE, s, &tok));
    // small grids that loop (about 100 waves each): the interior sweep leaves
    // the comm stream BAND_RESERVE_WAVES slots, not a full round
    hipLaunchKernelGGL(band_gather_h_kernel, dim3(std::min(3, (wi / 4 + 255) / 256), 8), dim3(256), 0, s, a, im, wi,
                       la);
    hipLaunchKernelGGL(band_gather_v_kernel, dim3(32), dim3(256), 0, s, a, im);
    SMI_HIP_CHECK(hipGetLastError());
    if (a.band[0] || a.band[1]) {
        SweepKArgs h{};
        h.in = im.h_in;
        h.out = im.h_out;
        h.rows = 6 * K;
        h.cols = wi;
        h.row_lo = K;
        h.row_hi = 5 * K;
        h.col_lo = la;
        h.col_hi = la + Y;
        h.gT = h.gB = 0;
        h.gL = !a.has[2];
        h.gR = !a.has[3];
        SMI_TRY(launch_sweepk_ex(K, h, 4 * K, 0, false, s));  // one row block per strip
    }
    if (a.band[2] || a.band[3]) {
        SweepKArgs v{};
        v.in = im.v_in;
        v.out = im.v_out;
        v.rows = X;
        v.cols = 6 * KC;
        v.row_lo = rlo;
        v.row_hi = rhi;
        v.col_lo = KC;
        v.col_hi = 5 * KC;
        v.gT = !a.has[0];
        v.gB = !a.has[1];
        v.gL = v.gR = 0;
        const int ht = std::max(2 * K, (rhi - rlo + 95) / 96);  // ~96 waves
        SMI_TRY(launch_sweepk_ex(K, v, ht, 0, false, s));
    }
    if (a.band[0] || a.band[1])
        hipLaunchKernelGGL(band_scatter_h_kernel, dim3(std::min(4, (Y / 4 + 255) / 256), 8), dim3(256), 0, s, a, im, wi,
                           la);
    if (a.band[2] || a.band[3])
        hipLaunchKernelGGL(band_scatter_v_kernel, dim3(32), dim3(256), 0, s, a, im, rlo, rhi);
    SMI_HIP_CHECK(hipGetLastError());
    if (tok >= 0) SMI_TRY(prof_end(tok, s));
    return SMI_SUCCESS;
}

}  // namespace smi
