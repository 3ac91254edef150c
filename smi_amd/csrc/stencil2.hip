// stencil2.hip -- two Jacobi steps per pass over HBM (temporal blocking).
//
// Same per-cell arithmetic as the single-step sweep (stencil_smi.cl:153-156,
// edges copied per :143-151), evaluated twice inside one pass: each wave
// streams its 256-column strip down the rows, forms the intermediate step
// (L1) one row ahead in registers -- including one extra column on each side
// of the strip, computed from two extra input columns fetched by broadcast
// loads -- and stores only the second step (L2).  HBM traffic per pass is the
// same as one single step, so the algorithmic 8 B/cell/step are moved at up to
// twice the single-step rate.  Multi-rank tiles keep a 2-cell ring on every
// side that has a neighbour; the ring kernel computes that ring from depth-2
// halos (two rows / two columns per neighbour and one corner cell per
// diagonal neighbour), exchanged once per pair of steps.
#include "stencil_common.h"

namespace smi {

// Diagnostic builds (-DSMI_BOUNDS_CHECK, tools/debug_fused.py) check every
// global index of the two-step kernels, record violations in a flag word and
// clamp the access instead of faulting.  Release builds compile this away.
#ifdef SMI_BOUNDS_CHECK
__device__ unsigned int g_smi_oob;
#define SMI_IDX(idx, size, code)                                   \
    do {                                                           \
        if ((size_t)(idx) >= (size_t)(size)) {                     \
            atomicOr(&g_smi_oob, (unsigned)(code));                \
            (idx) = 0;                                             \
        }                                                          \
    } while (0)
#else
#define SMI_IDX(idx, size, code) \
    do {                         \
    } while (0)
#endif

__device__ __forceinline__ float lane_val(float v, int lane) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}

struct Row2 {
    float4 v;  // this lane's 4 cells
    float2 w;  // input columns cs-2, cs-1 (strip west extras, wave-uniform)
    float2 e;  // input columns cs+4nl, cs+4nl+1 (strip east extras)
};

template <int U, bool NT>
__global__ __launch_bounds__(256) void sweep2_kernel(const float *__restrict__ in, float *__restrict__ out,
                                                     Sweep2Args a, int nstrips, int nrb, int ht, int row_lo,
                                                     int row_hi) {
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int lane = threadIdx.x & 63;
    const int task = __builtin_amdgcn_readfirstlane(lb * 4 + (int)(threadIdx.x >> 6));
    const int rb = task / nstrips;
    const int strip = task - rb * nstrips;
    if (rb >= nrb) return;  // wave-uniform

    const int rows = a.rows, cols = a.cols;
    const int o0 = row_lo + rb * ht;
    const int o1 = min(o0 + ht, row_hi);
    const int cs = strip * 256;
    const int nl = min(64, (cols - cs) >> 2);
    const bool act = lane < nl;
    const int c0 = cs + 4 * min(lane, nl - 1);
    const bool first_strip = strip == 0;
    const bool last_strip = cs + 256 >= cols;
    const bool gT = !a.skip[0], gB = !a.skip[1], gL = !a.skip[2], gR = !a.skip[3];
    const bool own_first = first_strip && lane == 0;
    const bool own_last = last_strip && lane == nl - 1;
    const bool copyL = own_first && gL, copyR = own_last && gR;
    const bool skipL = own_first && !gL, skipR = own_last && !gR;  // cols 0,1 / cols-2,cols-1
    const bool plain_store = act && !skipL && !skipR;
    const bool part_store = act && (skipL || skipR);
    // outside the tile the extras are never used: point them at column 0
    const int wcol = first_strip ? 0 : cs - 2;
    const int ecol = last_strip ? 0 : cs + 256;

    auto ld = [&](int r, Row2 &R) {
        size_t base = (size_t)min(max(r, 0), rows - 1) * cols;
        size_t iv = base + c0, iw = base + wcol, ie = base + ecol;
        SMI_IDX(iv, (size_t)rows * cols - 3, 0x1);
        SMI_IDX(iw, (size_t)rows * cols - 1, 0x2);
        SMI_IDX(ie, (size_t)rows * cols - 1, 0x4);
        R.v = *reinterpret_cast<const float4 *>(in + iv);
        R.w = *reinterpret_cast<const float2 *>(in + iw);
        R.e = *reinterpret_cast<const float2 *>(in + ie);
    };
    // intermediate step at row i (+ its values at columns cs-1 and cs+4nl)
    auto level1 = [&](int i, const Row2 &n, const Row2 &c, const Row2 &s, float4 &L, float &lw, float &le) {
        const bool rcopy = (i == 0 && gT) || (i == rows - 1 && gB);
        float w = wave_shr1(c.v.w);
        float e = wave_shl1(c.v.x);
        w = lane == 0 ? c.w.y : w;
        e = lane == nl - 1 ? c.e.x : e;
        L.x = jacobi(s.v.x, w, c.v.y, n.v.x);
        L.y = jacobi(s.v.y, c.v.x, c.v.z, n.v.y);
        L.z = jacobi(s.v.z, c.v.y, c.v.w, n.v.z);
        L.w = jacobi(s.v.w, c.v.z, e, n.v.w);
        L.x = (rcopy || copyL) ? c.v.x : L.x;
        L.y = rcopy ? c.v.y : L.y;
        L.z = rcopy ? c.v.z : L.z;
        L.w = (rcopy || copyR) ? c.v.w : L.w;
        const float c_first = lane_val(c.v.x, 0);       // input (i, cs)
        const float c_last = lane_val(c.v.w, nl - 1);   // input (i, cs+4nl-1)
        lw = rcopy ? c.w.y : jacobi(s.w.y, c.w.x, c_first, n.w.y);
        le = rcopy ? c.e.x : jacobi(s.e.x, c_last, c.e.y, n.e.x);
    };
    auto level2 = [&](int j, const float4 &N, const float4 &C, float Cw, float Ce, const float4 &S) {
        const bool rcopy = (j == 0 && gT) || (j == rows - 1 && gB);
        float w = wave_shr1(C.w);
        float e = wave_shl1(C.x);
        w = lane == 0 ? Cw : w;
        e = lane == nl - 1 ? Ce : e;
        float4 o;
        o.x = jacobi(S.x, w, C.y, N.x);
        o.y = jacobi(S.y, C.x, C.z, N.y);
        o.z = jacobi(S.z, C.y, C.w, N.z);
        o.w = jacobi(S.w, C.z, e, N.w);
        o.x = (rcopy || copyL) ? C.x : o.x;
        o.y = rcopy ? C.y : o.y;
        o.z = rcopy ? C.z : o.z;
        o.w = (rcopy || copyR) ? C.w : o.w;
        size_t io = (size_t)j * cols + c0;
        SMI_IDX(io, (size_t)rows * cols - 3, 0x8);
        float *op = out + io;
        if (plain_store) store4<NT>(op, o);
        if (part_store) {
            if (!skipL) {
                op[0] = o.x;
                op[1] = o.y;
            }
            if (!skipR) {
                op[2] = o.z;
                op[3] = o.w;
            }
        }
    };

    Row2 i0, i1, i2, i3;
    ld(o0 - 2, i0);
    ld(o0 - 1, i1);
    ld(o0, i2);
    ld(o0 + 1, i3);
    float4 Ln, Lc;
    float lwn, len, lwc, lec;
    level1(o0 - 1, i0, i1, i2, Ln, lwn, len);
    level1(o0, i1, i2, i3, Lc, lwc, lec);
    Row2 in_n = i2, in_c = i3;  // input rows j, j+1

    Row2 A[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ld(min(o0 + u, o1 - 1) + 2, A[u]);
    for (int j = o0; j < o1; j += U) {
        Row2 B[U];
        const bool more = j + U < o1;  // uniform
        if (more) {
#pragma unroll
            for (int u = 0; u < U; ++u) ld(min(j + U + u, o1 - 1) + 2, B[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (j + u < o1) {
                float4 Ls;
                float lws, les;
                level1(j + u + 1, in_n, in_c, A[u], Ls, lws, les);
                level2(j + u, Ln, Lc, lwc, lec, Ls);
                in_n = in_c;
                in_c = A[u];
                Ln = Lc;
                Lc = Ls;
                lwc = lws;
                lec = les;
            }
        }
        if (more) {
#pragma unroll
            for (int u = 0; u < U; ++u) A[u] = B[u];
        }
    }
    (void)lwn;
    (void)len;
}

// ---- ring of 2 cells on the halo-facing sides, from depth-2 halos --------
struct Ring2Ctx {
    const float *in;
    int X, Y;
    bool gT, gB, gL, gR;
    Halo2 h;

    // Input cell of the extended domain.  Every pointer of h is valid (the
    // launcher substitutes allocated buffers for absent sides) and every
    // index is clamped into its buffer, so the loads are safe even where the
    // compiler executes them speculatively (it did: an unclamped negative
    // offset from an unused NULL halo pointer faulted on gfx950).
    __device__ float at(int p, int q) const {
        const int pc = min(max(p, 0), X - 1), qc = min(max(q, 0), Y - 1);
        size_t i;
        if (p >= 0 && p < X && q >= 0 && q < Y) {
            i = (size_t)p * Y + q;
            SMI_IDX(i, (size_t)X * Y, 0x10);
            return in[i];
        }
        if (p < 0 && q >= 0 && q < Y) {
            i = (size_t)min(p + 2, 1) * Y + qc;
            SMI_IDX(i, 2 * (size_t)Y, 0x20);
            return h.top2[i];
        }
        if (p >= X && q >= 0 && q < Y) {
            i = (size_t)min(p - X, 1) * Y + qc;
            SMI_IDX(i, 2 * (size_t)Y, 0x40);
            return h.bot2[i];
        }
        if (p < 0 || p >= X) return h.corner[(p < 0 ? 0 : 2) + (q < 0 ? 0 : 1)];
        if (q < 0) {
            i = (size_t)min(max(q + 2, 0), 1) * X + pc;
            SMI_IDX(i, 2 * (size_t)X, 0x80);
            return h.left2[i];
        }
        i = (size_t)min(max(q - Y, 0), 1) * X + pc;
        SMI_IDX(i, 2 * (size_t)X, 0x100);
        return h.right2[i];
    }
    __device__ bool edge(int p, int q) const {
        return (p == 0 && gT) || (p == X - 1 && gB) || (q == 0 && gL) || (q == Y - 1 && gR);
    }
    __device__ float l1(int p, int q) const {
        if (edge(p, q)) return at(p, q);
        return jacobi(at(p + 1, q), at(p, q - 1), at(p, q + 1), at(p - 1, q));
    }
    __device__ float l2(int r, int c) const {
        if (edge(r, c)) return at(r, c);
        return jacobi(l1(r + 1, c), l1(r, c - 1), l1(r, c + 1), l1(r - 1, c));
    }
};

// One thread per ring cell: bands top (rows 0,1), bottom (rows X-2,X-1),
// left (cols 0,1), right (cols Y-2,Y-1); bands whose side is a global edge
// are skipped.  Also packs the new columns / corners for the neighbours.
__global__ __launch_bounds__(256) void ring2_kernel(Sweep2Args a, Halo2 h) {
    const int X = a.rows, Y = a.cols;
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    int r, c, band;
    if (t < 2 * Y) { band = 0; r = t / Y; c = t % Y; }
    else if ((t -= 2 * Y) < 2 * Y) { band = 1; r = X - 2 + t / Y; c = t % Y; }
    else if ((t -= 2 * Y) < 2 * X) { band = 2; c = t / X; r = t % X; }
    else if ((t -= 2 * X) < 2 * X) { band = 3; c = Y - 2 + t / X; r = t % X; }
    else return;
    if (!a.skip[band] || r < 0 || r >= X || c < 0 || c >= Y) return;
    Ring2Ctx ctx{a.in, X, Y, !a.skip[0], !a.skip[1], !a.skip[2], !a.skip[3], h};
    const float v = ctx.l2(r, c);
    size_t io = (size_t)r * Y + c;
    SMI_IDX(io, (size_t)X * Y, 0x200);
    a.out[io] = v;
    if (h.send_left2 && c < 2) {
        size_t i = (size_t)c * X + r;
        SMI_IDX(i, 2 * (size_t)X, 0x400);
        h.send_left2[i] = v;
    }
    if (h.send_right2 && c >= Y - 2) {
        size_t i = (size_t)(c - (Y - 2)) * X + r;
        SMI_IDX(i, 2 * (size_t)X, 0x800);
        h.send_right2[i] = v;
    }
    if (h.send_corner) {
        if (r == 0 && c == 0) h.send_corner[0] = v;
        if (r == 0 && c == Y - 1) h.send_corner[1] = v;
        if (r == X - 1 && c == 0) h.send_corner[2] = v;
        if (r == X - 1 && c == Y - 1) h.send_corner[3] = v;
    }
}

// Initial depth-2 halos: pack columns 0,1 / Y-2,Y-1 and the corner cells.
__global__ __launch_bounds__(256) void pack2_kernel(const float *in, int X, int Y, Halo2 h) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= X) return;
    const float *row = in + (size_t)r * Y;
    if (h.send_left2) {
        h.send_left2[r] = row[0];
        h.send_left2[(size_t)X + r] = row[Y > 1 ? 1 : 0];
    }
    if (h.send_right2) {
        h.send_right2[r] = row[Y >= 2 ? Y - 2 : 0];
        h.send_right2[(size_t)X + r] = row[Y - 1];
    }
    if (h.send_corner) {
        if (r == 0) {
            h.send_corner[0] = row[0];
            h.send_corner[1] = row[Y - 1];
        }
        if (r == X - 1) {
            h.send_corner[2] = row[0];
            h.send_corner[3] = row[Y - 1];
        }
    }
}

template <int U>
static void launch_sweep2_u(const Sweep2Args &a, int nstrips, int nrb, int ht, int blocks, int lo, int hi,
                            bool nt, hipStream_t s) {
    if (nt)
        hipLaunchKernelGGL((sweep2_kernel<U, true>), dim3(blocks), dim3(256), 0, s, a.in, a.out, a, nstrips,
                           nrb, ht, lo, hi);
    else
        hipLaunchKernelGGL((sweep2_kernel<U, false>), dim3(blocks), dim3(256), 0, s, a.in, a.out, a, nstrips,
                           nrb, ht, lo, hi);
}

int launch_sweep2(const Sweep2Args &a, hipStream_t s) {
    const int lo = a.skip[0] ? 2 : 0;
    const int hi = a.rows - (a.skip[1] ? 2 : 0);
    if (hi <= lo) return SMI_SUCCESS;  // tile is all ring
    const int ht = std::max(1, g_tune.ht2);
    const int nstrips = (a.cols + 255) / 256;
    const int nrb = (hi - lo + ht - 1) / ht;
    const long tasks = (long)nstrips * nrb;
    const int blocks = (int)((tasks + 3) / 4);
    int tok = -1;
    if (prof_enabled()) SMI_TRY(prof_begin(SMI_PROF_STENCIL_SWEEP, s, &tok, 2, 2.0 * (hi - lo) * a.cols));
    switch (g_tune.u2) {
    case 1: launch_sweep2_u<1>(a, nstrips, nrb, ht, blocks, lo, hi, g_tune.nt, s); break;
    case 2: launch_sweep2_u<2>(a, nstrips, nrb, ht, blocks, lo, hi, g_tune.nt, s); break;
    case 8: launch_sweep2_u<8>(a, nstrips, nrb, ht, blocks, lo, hi, g_tune.nt, s); break;
    default: launch_sweep2_u<4>(a, nstrips, nrb, ht, blocks, lo, hi, g_tune.nt, s); break;
    }
    SMI_HIP_CHECK(hipGetLastError());
    if (tok >= 0) SMI_TRY(prof_end(tok, s));
    return SMI_SUCCESS;
}

int launch_ring2(const Sweep2Args &a, const Halo2 &h, hipStream_t s) {
    const long cells = 4L * a.cols + 4L * a.rows;
    const int blocks = (int)((cells + 255) / 256);
    int tok = -1;
    if (prof_enabled()) SMI_TRY(prof_begin(SMI_PROF_STENCIL_EDGE, s, &tok));
    hipLaunchKernelGGL(ring2_kernel, dim3(blocks), dim3(256), 0, s, a, h);
    SMI_HIP_CHECK(hipGetLastError());
    if (tok >= 0) SMI_TRY(prof_end(tok, s));
    return SMI_SUCCESS;
}

int launch_pack2(const float *in, int rows, int cols, const Halo2 &h, hipStream_t s) {
    hipLaunchKernelGGL(pack2_kernel, dim3((rows + 255) / 256), dim3(256), 0, s, in, rows, cols, h);
    SMI_HIP_CHECK(hipGetLastError());
    return SMI_SUCCESS;
}

}  // namespace smi

#ifdef SMI_BOUNDS_CHECK
// Diagnostic builds only (not part of include/smi): read and clear the flags.
extern "C" int smi_debug_oob(unsigned int *flags) {
    SMI_HIP_CHECK(hipDeviceSynchronize());
    SMI_HIP_CHECK(hipMemcpyFromSymbol(flags, HIP_SYMBOL(smi::g_smi_oob), sizeof(unsigned int)));
    unsigned int zero = 0;
    SMI_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(smi::g_smi_oob), &zero, sizeof(unsigned int)));
    return SMI_SUCCESS;
}
#endif
