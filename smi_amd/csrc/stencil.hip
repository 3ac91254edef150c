// stencil.hip -- the stencil_smi hot path on gfx950.
//
// Reference pipeline replaced (ryutakashino/SMI, examples/kernels/stencil_smi.cl):
//   Read    :20-115   streams the tile + 1-cell halo ring from 4 DDR banks
//   Stencil :117-165  out = 0.25*(S+W+E+N), global-edge cells copied
//   Write   :167-234  stores the result, tees edge rows/cols to the neighbours
//   Convert{Send,Receive}* :236-386  per-element SMI_Push/SMI_Pop halo bridges
// MI355X design: one sweep kernel streams each 256-column strip of the tile
// down its rows with 16-byte loads (one float4 per lane, one wave per strip),
// keeps the north/centre/south rows in registers, gets the west/east
// neighbours across lanes with DPP wave shifts, and fetches only the two
// strip-edge cells per row separately.  Each cell is read once from HBM and
// written once (8 B/cell/step algorithmic).  In multi-rank runs an edge
// kernel computes the tile's halo-facing rows/columns first (fusing the
// column pack that Write's send_left/send_right tee did), the halo
// exchange runs on a dedicated stream through the transport (RCCL over xGMI),
// and the interior sweep overlaps it.
#include <algorithm>

#include "stencil_common.h"

namespace smi {

// One wave = one strip of 256 columns x `ht` rows; 4 waves per block take 4
// consecutive (row-block, strip) tasks, strip fastest.  U rows are fetched
// per batch and the next batch is in flight while the current one computes.
// All control values are wave-uniform (readfirstlane) and every load is
// unconditional with a clamped address, so the loop body has no divergent
// control flow around its loads and the compiler emits counted vmcnt waits.
template <int U, bool NT>
__global__ __launch_bounds__(256) void sweep_kernel(const float *__restrict__ in,
                                                    float *__restrict__ out, SweepArgs a,
                                                    int nstrips, int nrb, int ht) {
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int lane = threadIdx.x & 63;
    const int task = __builtin_amdgcn_readfirstlane(lb * 4 + (int)(threadIdx.x >> 6));
    const int rb = task / nstrips;
    const int strip = task - rb * nstrips;
    if (rb >= nrb) return;  // wave-uniform

    const int rows = a.rows, cols = a.cols;
    const int r0 = rb * ht;
    const int r1 = min(r0 + ht, rows);
    const int cs = strip * 256;
    const int nl = min(64, (cols - cs) >> 2);  // active lanes of this strip
    const bool act = lane < nl;
    const int c0 = cs + 4 * min(lane, nl - 1);  // clamped: inactive lanes re-read lane nl-1
    const bool first_strip = strip == 0;
    const bool last_strip = cs + 256 >= cols;
    const int mT = a.mode[0], mB = a.mode[1], mL = a.mode[2], mR = a.mode[3];
    const bool own_first_col = first_strip && lane == 0;
    const bool own_last_col = last_strip && lane == nl - 1;
    const bool skipL = own_first_col && mL == SMI_SIDE_SKIP;
    const bool skipR = own_last_col && mR == SMI_SIDE_SKIP;
    const bool copyL = own_first_col && mL == SMI_SIDE_COPY;
    const bool copyR = own_last_col && mR == SMI_SIDE_COPY;
    const bool plain_store = act && !skipL && !skipR;
    const bool part_store = act && (skipL || skipR);
    // uniform base pointers for the out-of-tile rows / strip-edge columns
    const float *top = mT == SMI_SIDE_HALO ? a.halo[0] : in;
    const float *bot = mB == SMI_SIDE_HALO ? a.halo[1] : in + (size_t)(rows - 1) * cols;
    const bool west_halo = first_strip && mL == SMI_SIDE_HALO;
    const bool east_halo = last_strip && mR == SMI_SIDE_HALO;
    // west edge of row r: in[r*cols + cs-1]  |  halo_left[r]  |  (unused) in[r*cols]
    const float *wbase = first_strip ? (west_halo ? a.halo[2] : in) : in + cs - 1;
    const int wstride = west_halo ? 1 : cols;
    const float *ebase = last_strip ? (east_halo ? a.halo[3] : in) : in + cs + 256;
    const int estride = east_halo ? 1 : cols;

    auto rowp = [&](int r) -> const float * {
        return r < 0 ? top : (r >= rows ? bot : in + (size_t)r * cols);
    };
    auto ld4 = [&](int r) -> float4 { return *reinterpret_cast<const float4 *>(rowp(r) + c0); };
    auto ldw = [&](int r) -> float { return wbase[(size_t)r * wstride]; };
    auto lde = [&](int r) -> float { return ebase[(size_t)r * estride]; };

    auto do_row = [&](int r, float4 n, float4 c, float4 s, float ew, float ee) {
        const bool row_skip = (r == 0 && mT == SMI_SIDE_SKIP) || (r == rows - 1 && mB == SMI_SIDE_SKIP);
        const bool row_copy = (r == 0 && mT == SMI_SIDE_COPY) || (r == rows - 1 && mB == SMI_SIDE_COPY);
        float w = wave_shr1(c.w);
        float e = wave_shl1(c.x);
        w = lane == 0 ? ew : w;
        e = lane == nl - 1 ? ee : e;
        float4 o;
        o.x = jacobi(s.x, w, c.y, n.x);
        o.y = jacobi(s.y, c.x, c.z, n.y);
        o.z = jacobi(s.z, c.y, c.w, n.z);
        o.w = jacobi(s.w, c.z, e, n.w);
        o.x = (copyL || row_copy) ? c.x : o.x;
        o.y = row_copy ? c.y : o.y;
        o.z = row_copy ? c.z : o.z;
        o.w = (copyR || row_copy) ? c.w : o.w;
        if (row_skip) return;  // wave-uniform
        float *op = out + (size_t)r * cols + c0;
        if (plain_store) store4<NT>(op, o);
        if (part_store) {
            if (!skipL) op[0] = o.x;
            op[1] = o.y;
            op[2] = o.z;
            if (!skipR) op[3] = o.w;
        }
        if (own_first_col && !skipL && a.send_left) a.send_left[r] = o.x;
        if (own_last_col && !skipR && a.send_right) a.send_right[r] = o.w;
    };

    float4 n = ld4(r0 - 1);
    float4 c = ld4(r0);
    float4 sA[U];
    float wA[U], eA[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int r = min(r0 + u, r1 - 1);
        sA[u] = ld4(r + 1);
        wA[u] = ldw(r);
        eA[u] = lde(r);
    }
    for (int r = r0; r < r1; r += U) {
        float4 sB[U];
        float wB[U], eB[U];
        const bool more = r + U < r1;  // uniform
        if (more) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int rr = min(r + U + u, r1 - 1);
                sB[u] = ld4(rr + 1);
                wB[u] = ldw(rr);
                eB[u] = lde(rr);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (r + u < r1) {
                do_row(r + u, n, c, sA[u], wA[u], eA[u]);
                n = c;
                c = sA[u];
            }
        }
        if (more) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                sA[u] = sB[u];
                wA[u] = wB[u];
                eA[u] = eB[u];
            }
        }
    }
}

// Cells of the tile's halo-facing sides (those with side_mask bit set),
// computed with the true side modes (COPY / HALO); also packs the new
// first / last column for the left / right neighbours.  One thread per cell:
// [0, cols) row 0, [cols, 2cols) row rows-1, then col 0, then col cols-1.
__global__ __launch_bounds__(256) void edge_kernel(SweepArgs a, int side_mask) {
    const int rows = a.rows, cols = a.cols;
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    int r, c, side;
    if (t < cols) { r = 0; c = t; side = 0; }
    else if ((t -= cols) < cols) { r = rows - 1; c = t; side = 1; }
    else if ((t -= cols) < rows) { r = t; c = 0; side = 2; }
    else if ((t -= rows) < rows) { r = t; c = cols - 1; side = 3; }
    else return;
    if (!(side_mask & (1 << side))) return;
    const float *in = a.in;
    const size_t idx = (size_t)r * cols + c;
    const bool copy = (r == 0 && a.mode[0] == SMI_SIDE_COPY) ||
                      (r == rows - 1 && a.mode[1] == SMI_SIDE_COPY) ||
                      (c == 0 && a.mode[2] == SMI_SIDE_COPY) ||
                      (c == cols - 1 && a.mode[3] == SMI_SIDE_COPY);
    float v;
    if (copy) {
        v = in[idx];
    } else {
        // select the address, then load once: no load of an unused halo
        // pointer or of an out-of-tile offset can be speculated
        const float *np = r > 0 ? in + idx - cols : a.halo[0] + c;
        const float *sp = r < rows - 1 ? in + idx + cols : a.halo[1] + c;
        const float *wp = c > 0 ? in + idx - 1 : a.halo[2] + r;
        const float *ep = c < cols - 1 ? in + idx + 1 : a.halo[3] + r;
        v = jacobi(*sp, *wp, *ep, *np);
    }
    a.out[idx] = v;
    if (c == 0 && a.send_left) a.send_left[r] = v;
    if (c == cols - 1 && a.send_right) a.send_right[r] = v;
}

// Pack the first / last column of a tile (the initial halos that the
// reference's artificial timestep t=0 sends, stencil_smi.cl:26-29,183-224).
__global__ __launch_bounds__(256) void pack_cols_kernel(const float *in, int rows, int cols,
                                                        float *left, float *right) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    if (left) left[r] = in[(size_t)r * cols];
    if (right) right[r] = in[(size_t)r * cols + cols - 1];
}

// ---------------------------------------------------------------- host --
Tuning g_tune;

int check_tile(const float *in, const float *out, int rows, int cols) {
    SMI_ARG_CHECK(in && out, "NULL tile buffer");
    SMI_ARG_CHECK(in != out, "in and out must differ");
    SMI_ARG_CHECK(rows >= 1 && cols >= 4 && cols % 4 == 0, "tile must be >=1 x >=4 with y_local % 4 == 0");
    SMI_ARG_CHECK(aligned16(in) && aligned16(out), "tile buffers must be 16-byte aligned");
    return SMI_SUCCESS;
}

template <int U>
static void launch_sweep_u(const SweepArgs &a, int nstrips, int nrb, int ht, int blocks, bool nt,
                           hipStream_t s) {
    if (nt)
        hipLaunchKernelGGL((sweep_kernel<U, true>), dim3(blocks), dim3(256), 0, s, a.in, a.out, a,
                           nstrips, nrb, ht);
    else
        hipLaunchKernelGGL((sweep_kernel<U, false>), dim3(blocks), dim3(256), 0, s, a.in, a.out, a,
                           nstrips, nrb, ht);
}

int launch_sweep(const SweepArgs &a, hipStream_t s) {
    const int ht = std::max(1, g_tune.ht);
    const int nstrips = (a.cols + 255) / 256;
    const int nrb = (a.rows + ht - 1) / ht;
    const long tasks = (long)nstrips * nrb;
    const int blocks = (int)((tasks + 3) / 4);
    int tok = -1;
    if (prof_enabled()) SMI_TRY(prof_begin(SMI_PROF_STENCIL_SWEEP, s, &tok, 1, (double)a.rows * a.cols));
    switch (g_tune.u) {
    case 1: launch_sweep_u<1>(a, nstrips, nrb, ht, blocks, g_tune.nt, s); break;
    case 2: launch_sweep_u<2>(a, nstrips, nrb, ht, blocks, g_tune.nt, s); break;
    case 8: launch_sweep_u<8>(a, nstrips, nrb, ht, blocks, g_tune.nt, s); break;
    case 16: launch_sweep_u<16>(a, nstrips, nrb, ht, blocks, g_tune.nt, s); break;
    default: launch_sweep_u<4>(a, nstrips, nrb, ht, blocks, g_tune.nt, s); break;
    }
    SMI_HIP_CHECK(hipGetLastError());
    if (tok >= 0) SMI_TRY(prof_end(tok, s));
    return SMI_SUCCESS;
}

int launch_edge(const SweepArgs &a, int side_mask, hipStream_t s) {
    const long cells = 2L * a.cols + 2L * a.rows;
    const int blocks = (int)((cells + 255) / 256);
    int tok = -1;
    if (prof_enabled()) SMI_TRY(prof_begin(SMI_PROF_STENCIL_EDGE, s, &tok));
    hipLaunchKernelGGL(edge_kernel, dim3(blocks), dim3(256), 0, s, a, side_mask);
    SMI_HIP_CHECK(hipGetLastError());
    if (tok >= 0) SMI_TRY(prof_end(tok, s));
    return SMI_SUCCESS;
}

int launch_pack_cols(const float *in, int rows, int cols, float *left, float *right, hipStream_t s) {
    hipLaunchKernelGGL(pack_cols_kernel, dim3((rows + 255) / 256), dim3(256), 0, s, in, rows, cols, left, right);
    SMI_HIP_CHECK(hipGetLastError());
    return SMI_SUCCESS;
}

}  // namespace smi

using namespace smi;

extern "C" {

int smi_stencil_set_tuning(int rows_per_wave, int rows_in_flight, int nontemporal_stores, int overlap) {
    if (rows_per_wave > 0) g_tune.ht = rows_per_wave;
    if (rows_in_flight > 0) {
        SMI_ARG_CHECK(rows_in_flight == 1 || rows_in_flight == 2 || rows_in_flight == 4 ||
                          rows_in_flight == 8 || rows_in_flight == 16,
                      "rows_in_flight must be 1, 2, 4, 8 or 16");
        g_tune.u = rows_in_flight;
    }
    if (nontemporal_stores >= 0) g_tune.nt = nontemporal_stores != 0;
    if (overlap >= 0) g_tune.overlap = overlap != 0;
    return SMI_SUCCESS;
}

int smi_stencil_get_tuning(int *rows_per_wave, int *rows_in_flight, int *nontemporal_stores, int *overlap) {
    if (rows_per_wave) *rows_per_wave = g_tune.ht;
    if (rows_in_flight) *rows_in_flight = g_tune.u;
    if (nontemporal_stores) *nontemporal_stores = g_tune.nt;
    if (overlap) *overlap = g_tune.overlap;
    return SMI_SUCCESS;
}

int smi_stencil_step(const float *in, float *out, int x_local, int y_local, const int mode[4],
                     const float *const halo[4], float *send_left, float *send_right,
                     SMI_Stream stream) {
    SMI_TRY(check_tile(in, out, x_local, y_local));
    SMI_ARG_CHECK(mode, "NULL mode array");
    SweepArgs a{};
    a.in = in;
    a.out = out;
    a.rows = x_local;
    a.cols = y_local;
    for (int k = 0; k < 4; ++k) {
        SMI_ARG_CHECK(mode[k] >= SMI_SIDE_COPY && mode[k] <= SMI_SIDE_SKIP, "bad side mode");
        a.mode[k] = mode[k];
        a.halo[k] = halo ? halo[k] : nullptr;
        if (mode[k] == SMI_SIDE_HALO) SMI_ARG_CHECK(a.halo[k] != nullptr, "HALO side without halo vector");
    }
    a.send_left = send_left;
    a.send_right = send_right;
    return launch_sweep(a, (hipStream_t)stream);
}

}  // extern "C"
