// stencil_common.h -- shared pieces of the stencil kernels and driver.
#pragma once

#include <algorithm>

#include "smi_internal.h"

namespace smi {

struct SweepArgs {
    const float *in;
    float *out;
    int rows, cols;
    int mode[4];            // SMI_SIDE_* per side: top, bottom, left, right
    const float *halo[4];   // halo vectors for SMI_SIDE_HALO sides
    float *send_left;       // packed new first column (nullable)
    float *send_right;      // packed new last column (nullable)
};

// 0.25 * (((S + W) + E) + N), fp32, round-to-nearest, never contracted
// (stencil_smi.cl:153-156; 0.25*x is exact, so the double literal there
// gives the same bits as this fp32 multiply).
__device__ __forceinline__ float jacobi(float s, float w, float e, float n) {
    float sum = __fadd_rn(s, w);
    sum = __fadd_rn(sum, e);
    sum = __fadd_rn(sum, n);
    return __fmul_rn(0.25f, sum);
}

// lane i <- lane i-1 (DPP wave_shr:1); lane 0 gets 0
__device__ __forceinline__ float wave_shr1(float v) {
    return __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138, 0xf, 0xf, false));
}
// lane i <- lane i+1 (DPP wave_shl:1); lane 63 gets 0
__device__ __forceinline__ float wave_shl1(float v) {
    return __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, false));
}

// Blocks b, b+8, b+16 ... share an XCD (round-robin dispatch); give each XCD
// a contiguous range of logical blocks so that vertically and horizontally
// adjacent strips -- whose edge rows/cells each reads -- share one L2.
// Bijective for any nb (cdna_hip_programming.md, "XCD swizzle").
__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int q = nb >> 3, r = nb & 7, x = b & 7;
    const int base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    return base + (b >> 3);
}

template <bool NT>
__device__ __forceinline__ void store4(float *p, float4 v) {
    if constexpr (NT) {
        __builtin_nontemporal_store(v.x, p + 0);
        __builtin_nontemporal_store(v.y, p + 1);
        __builtin_nontemporal_store(v.z, p + 2);
        __builtin_nontemporal_store(v.w, p + 3);
    } else {
        *reinterpret_cast<float4 *>(p) = v;
    }
}

struct Tuning {
    int ht = 12;        // rows per wave (single-step sweep)
    int u = 16;         // rows in flight per batch
    int nt = 1;         // non-temporal stores
    int overlap = 1;    // overlap halo exchange with the interior sweep
    int fuse = 20;      // Jacobi steps per pass over HBM (1..20; K > 12: rotating-ring sweep, single tiles)
    int ht2 = 8;        // rows per wave (two-step sweep)
    int u2 = 8;         // rows in flight per batch (two-step sweep)
    int htk = 0;        // rows per wave (K-step sweep, K >= 4); 0 = one round of resident waves
    // K-step interior in multi-rank runs: rounds of resident waves, and
    // wave slots left free for the band kernel and the exchange
    // (smi_stencil_set_bands).  One round, none reserved: the interior-rank
    // rehearsal runs at 0.87 of a lone tile with the band kernel in the
    // interior's tail, 0.81-0.85 with two rounds (profiles/r03/).
    int rounds_multi = 1;
    int band_reserve = 0;
    int uk = 3;        // rows loaded ahead (K-step sweep: one 3-row register batch, fixed at build time)
    // deep sweep (stencild.hip): extra work of an edge-column strip's and of
    // an upward-walking bottom block's waves, in 16ths of a plain block's
    // (their blocks are shortened by it); waves of the launch (0 = one round
    // of resident waves)
    int deep_ce16 = 10;  // tools/deep_tune.py: K = 20 at 8192^2, 0.141 ms (4/2: 0.156)
    int deep_rev16 = 6;
    int deep_waves = 0;
    // multi-rank bands for K >= SWEEPD_MIN: 1 = the lean kernel that runs
    // beside the interior sweep (bandl_kernel, <= 64 VGPRs, one workgroup per
    // CU), 0 = one wave per segment (bandk_kernel)
    int band_lean = 1;
    int host_join = 1;  // smi_stencil_set_join
};
extern Tuning g_tune;

inline bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }
int check_tile(const float *in, const float *out, int rows, int cols);

// single step (stencil.hip)
int launch_sweep(const SweepArgs &a, hipStream_t s);
int launch_edge(const SweepArgs &a, int side_mask, hipStream_t s);
int launch_pack_cols(const float *in, int rows, int cols, float *left, float *right, hipStream_t s);

// two steps per pass (stencil2.hip).  skip[k] = 1: the 2-wide ring on side k
// has a neighbour and is computed by the ring kernel; 0: global edge (copy).
struct Sweep2Args {
    const float *in;
    float *out;
    int rows, cols;
    int skip[4];
};
// depth-2 halos: top2 = rows -2,-1 (2 x cols); bot2 = rows X, X+1; left2 =
// cols -2,-1 ([2][rows]); right2 = cols Y, Y+1; corner = (-1,-1), (-1,Y),
// (X,-1), (X,Y).  send2 = packed cols 0,1 | cols Y-2,Y-1 ([2][rows] each) and
// the 4 corner cells (0,0), (0,Y-1), (X-1,0), (X-1,Y-1).
struct Halo2 {
    const float *top2, *bot2, *left2, *right2, *corner;
    float *send_left2, *send_right2, *send_corner;
};
int launch_sweep2(const Sweep2Args &a, hipStream_t s);
int launch_ring2(const Sweep2Args &a, const Halo2 &h, hipStream_t s);
int launch_pack2(const float *in, int rows, int cols, const Halo2 &h, hipStream_t s);

// K steps per pass (stencilk.hip, 3 <= K <= 12): output rectangle
// [row_lo,row_hi) x [col_lo,col_hi) of the tile, computed from input cells
// within K of it (all inside the tile); g* = 1 where the side is a global
// edge of the grid (its outermost row/column is copied every step).
struct SweepKArgs {
    const float *in;
    float *out;
    int rows, cols;
    int row_lo, row_hi, col_lo, col_hi;
    int gT, gB, gL, gR;
};
constexpr int SWEEPK_MIN = 3, SWEEPK_MAX = 12;
// Lanes per 64-lane window side that never store (the window apron is 4x
// as many columns, >= K): 4 for K >= 9 (224 stored columns, line-aligned
// stores), else the minimal ceil(K / 4).
__host__ __device__ constexpr int sweepk_apron_lanes(int K) { return K >= 9 ? 4 : (K + 3) / 4; }
int launch_sweepk(int K, const SweepKArgs &a, hipStream_t s);
int launch_sweepk_ex(int K, const SweepKArgs &a, int ht, int reserve, bool prof, hipStream_t s,
                     hipEvent_t stop = nullptr);
int sweepk_window_cols(int K);  // output columns per 256-column window

// Deep K-step sweep (stencild.h / stencild.hip, SWEEPD_MIN <= K <= SWEEPD_MAX):
// same arguments and output as the K-step sweep (a whole single tile, or a
// multi-rank interior beside the band kernel), for passes of more than
// SWEEPK_MAX steps.  The launch geometry: strips of 256 - 2 KC
// output columns; interior strips cut into nrb row blocks, the strips
// holding a global-edge column (their waves run the per-lane column copy)
// into nrb_ce shorter blocks, and in every strip the bottom block of a tile
// with a global bottom edge (it walks upwards: one extra DPP move per W/E
// pair) shortened to weight wlast/16 of a block -- so that every wave of the
// single round finishes at about the same time.
constexpr int SWEEPD_MIN = 13, SWEEPD_MAX = 20;
struct SweepDGeom {
    int nstrips;   // all strips
    int n_int;     // interior strips (no global-edge column): [int0, int0 + n_int)
    int int0;
    int nrb;       // row blocks per interior strip
    int ce[4];     // strip indices of the edge-column strips (-1: none)
    int nrb_ce;    // row blocks per edge-column strip
    int wlast;     // weight of a bottom block (gB) in 16ths of a block
    int tasks;     // waves of the launch
};
// Rows [o0, o1) of block rb of nb in a strip: blocks of weight 16 except a
// bottom block of weight wlast (integer arithmetic: both neighbours of a
// boundary compute it identically).
__host__ __device__ inline void sweepd_block_rows(const SweepKArgs &a, int rb, int nb, int wlast, int *o0, int *o1) {
    const long out_rows = a.row_hi - a.row_lo;
    const long den = (long)(nb - 1) * 16 + (a.gB ? wlast : 16);
    *o0 = a.row_lo + (int)(out_rows * rb * 16 / den);
    *o1 = rb == nb - 1 ? a.row_hi : a.row_lo + (int)(out_rows * (rb + 1) * 16 / den);
}
bool sweepd_fits(int K, const SweepKArgs &a);
int sweepd_window_cols(int K);
int sweepd_geometry(int K, const SweepKArgs &a, int reserve, SweepDGeom *g);
int launch_sweepd(int K, const SweepKArgs &a, int reserve, hipStream_t s, hipEvent_t start, hipEvent_t stop);

// Depth-K halos (stencil_bandk.h / stencil_bandk.hip).  KC = 4 ceil(K/4):
// the column depth, whole float4 groups.  Receive side: top = rows -K..-1 and
// bot = rows X..X+K-1 (K x Y, row-major), left = cols -KC..-1 and right =
// cols Y..Y+KC-1 (X x KC, [row][k]), corner[tl,tr,bl,br] = K x KC blocks of
// the diagonal neighbours.  Send side: send_left/right = this tile's cols
// 0..KC-1 / Y-KC..Y-1 ([row][k]), send_corner = its own four K x KC corner
// blocks.  The top/bottom rows are sent straight from the tile.  Every
// pointer is a valid allocation, also for sides without a neighbour.
struct HaloK {
    const float *top, *bot, *left, *right;
    const float *corner[4];
    float *send_left, *send_right;
    float *send_corner[4];
};
__host__ __device__ constexpr int kc_of(int K) { return 4 * ((K + 3) / 4); }
struct BandKArgs {
    const float *in;
    float *out;
    int rows, cols;
    int kc;            // column depth of the side bands / halos / packs: kc_of(K)
    int has[4];        // neighbour on side top, bottom, left, right
    int pack;          // tee the next exchange's packed columns / corner blocks
    HaloK h;
    // filled by launch_bandk
    int first[5];      // first wave of band top, bottom, left, right; first[4] = all waves
    int sw;            // cells stored per wave (64 - 2K; lean kernel 128 - 2 KE)
    int rlo, rhi;      // rows of the left/right bands
    int prio;          // lean kernel: 1 = raised wave priority (s_setprio 3), 0 = normal
};
int plan_bands(int K, BandKArgs *a, bool lean);  // fills kc, first[], sw, rlo, rhi
// the bands of a pass: one wave per segment, or max_waves (> 0) waves;
// stop (nullable): an event the launch's dispatch records at completion
int launch_bandk(int K, BandKArgs a, int max_waves, hipStream_t s, hipEvent_t stop = nullptr);
int launch_packk(const float *in, int rows, int cols, int K, const HaloK &h, hipStream_t s);

}  // namespace smi
