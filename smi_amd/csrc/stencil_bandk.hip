// stencil_bandk.hip -- host side of the halo-facing bands of a K-step pass
// (kernels: stencil_bandk.h, one instantiation per K in bandk_k<K>.hip) and
// the initial depth-K pack.
#include <cstdlib>

#include "stencil_common.h"

namespace smi {

#define SMI_BANDK_DECL(K) \
    int bandk_launch_k##K(const BandKArgs &a, int waves, hipStream_t s, hipEvent_t start, hipEvent_t stop);
SMI_BANDK_DECL(3)
SMI_BANDK_DECL(4)
SMI_BANDK_DECL(5)
SMI_BANDK_DECL(6)
SMI_BANDK_DECL(7)
SMI_BANDK_DECL(8)
SMI_BANDK_DECL(9)
SMI_BANDK_DECL(10)
SMI_BANDK_DECL(11)
SMI_BANDK_DECL(12)
SMI_BANDK_DECL(13)
SMI_BANDK_DECL(14)
SMI_BANDK_DECL(15)
SMI_BANDK_DECL(16)
SMI_BANDK_DECL(17)
SMI_BANDK_DECL(18)
SMI_BANDK_DECL(19)
SMI_BANDK_DECL(20)

#define SMI_BANDL_DECL(K) \
    int bandl_launch_k##K(const BandKArgs &a, int blocks, hipStream_t s, hipEvent_t start, hipEvent_t stop);
SMI_BANDL_DECL(13)
SMI_BANDL_DECL(14)
SMI_BANDL_DECL(15)
SMI_BANDL_DECL(16)
SMI_BANDL_DECL(17)
SMI_BANDL_DECL(18)
SMI_BANDL_DECL(19)
SMI_BANDL_DECL(20)

static int compute_units() {
    static int cached[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    if (!cached[dev]) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
        cached[dev] = cus;
    }
    return cached[dev];
}

static int launch_bandl(int K, const BandKArgs &a, int blocks, hipStream_t s, hipEvent_t start, hipEvent_t stop) {
    switch (K) {
    case 13: return bandl_launch_k13(a, blocks, s, start, stop);
    case 14: return bandl_launch_k14(a, blocks, s, start, stop);
    case 15: return bandl_launch_k15(a, blocks, s, start, stop);
    case 16: return bandl_launch_k16(a, blocks, s, start, stop);
    case 17: return bandl_launch_k17(a, blocks, s, start, stop);
    case 18: return bandl_launch_k18(a, blocks, s, start, stop);
    case 19: return bandl_launch_k19(a, blocks, s, start, stop);
    default: return bandl_launch_k20(a, blocks, s, start, stop);
    }
}

int plan_bands(int K, BandKArgs *ap, bool lean) {
    BandKArgs &a = *ap;
    const int X = a.rows, Y = a.cols;
    a.kc = kc_of(K);
    SMI_ARG_CHECK(K >= SWEEPK_MIN && K <= SWEEPD_MAX, "bandk: K must be 3..20");
    SMI_ARG_CHECK(X >= 2 * K && Y >= 2 * a.kc && Y % 4 == 0, "bandk: tile smaller than 2K x 2KC");
    // one wave per 64 - 2K cells along a band (stencil_bandk.h)
    // lean kernel: two cells per lane, pair-aligned windows (BandL::SW)
    a.sw = lean ? 128 - 2 * (K + (K & 1)) : 64 - 2 * K;
    a.rlo = a.has[0] ? K : 0;
    a.rhi = a.has[1] ? X - K : X;
    const int nrow = (Y + a.sw - 1) / a.sw;
    const int ncol = a.rhi > a.rlo ? (a.rhi - a.rlo + a.sw - 1) / a.sw : 0;
    const int waves_of[4] = {a.has[0] ? nrow : 0, a.has[1] ? nrow : 0, a.has[2] ? ncol : 0, a.has[3] ? ncol : 0};
    int n = 0;
    for (int k = 0; k < 4; ++k) {
        a.first[k] = n;
        n += waves_of[k];
    }
    a.first[4] = n;
    a.prio = 1;
#ifdef SMI_LOOPBACK_REHEARSAL
    if (const char *v = getenv("SMI_REH_BAND_PRIO")) a.prio = atoi(v) != 0;  // priority A/B
    // timing experiments (results are wrong): no band work at all, or only
    // the row walks (top / bottom bands) or only the transposed column walks
    if (getenv("SMI_REH_NOBANDS")) a.first[1] = a.first[2] = a.first[3] = a.first[4] = 0;
    if (const char *m = getenv("SMI_REH_BANDS")) {
        if (m[0] == 'r') {
            a.first[3] = a.first[4] = a.first[2];
        } else if (m[0] == 'c') {
            const int nl = a.first[3] - a.first[2], nr = a.first[4] - a.first[3];
            a.first[1] = a.first[2] = 0;
            a.first[3] = nl;
            a.first[4] = nl + nr;
        }
    }
#endif
    return SMI_SUCCESS;
}

int launch_bandk(int K, BandKArgs a, int max_waves, hipStream_t s, hipEvent_t stop) {
    const bool lean = K >= SWEEPD_MIN && g_tune.band_lean;
    SMI_TRY(plan_bands(K, &a, lean));
    const int segs = a.first[4];
    if (segs == 0) {
        if (stop) SMI_HIP_CHECK(hipEventRecord(stop, s));
        return SMI_SUCCESS;
    }
    // one wave per segment, or at most max_waves (> 0) waves looping over them
    const int n = max_waves > 0 ? std::min(segs, std::max(4, max_waves)) : segs;
    // timed by the dispatch itself (as the K-step sweep, stencilk.hip); the
    // caller's ordering event is then recorded right after the launch
    hipEvent_t start = nullptr, kstop = stop, after = nullptr;
    int tok = -1;
    if (prof_enabled()) {
        SMI_TRY(prof_launch(SMI_PROF_STENCIL_EDGE, &tok, K, 0.0, &start, &kstop));
        after = stop;
    }
    int rc = SMI_SUCCESS;
    if (lean) {
        // the lean kernel beside the interior: one workgroup (4 waves) per CU
        // at most, fewer when max_waves asks for fewer
        const int cus = compute_units();
        SMI_ARG_CHECK(cus > 0, "bandl: compute-unit query failed");
        int blocks = std::min(cus, (segs + 3) / 4);
        if (max_waves > 0) blocks = std::min(blocks, std::max(1, max_waves / 4));
        SMI_TRY(launch_bandl(K, a, blocks, s, start, kstop));
        if (after) SMI_HIP_CHECK(hipEventRecord(after, s));
        return SMI_SUCCESS;
    }
    switch (K) {
    case 3: rc = bandk_launch_k3(a, n, s, start, kstop); break;
    case 4: rc = bandk_launch_k4(a, n, s, start, kstop); break;
    case 5: rc = bandk_launch_k5(a, n, s, start, kstop); break;
    case 6: rc = bandk_launch_k6(a, n, s, start, kstop); break;
    case 7: rc = bandk_launch_k7(a, n, s, start, kstop); break;
    case 8: rc = bandk_launch_k8(a, n, s, start, kstop); break;
    case 9: rc = bandk_launch_k9(a, n, s, start, kstop); break;
    case 10: rc = bandk_launch_k10(a, n, s, start, kstop); break;
    case 11: rc = bandk_launch_k11(a, n, s, start, kstop); break;
    case 12: rc = bandk_launch_k12(a, n, s, start, kstop); break;
    case 13: rc = bandk_launch_k13(a, n, s, start, kstop); break;
    case 14: rc = bandk_launch_k14(a, n, s, start, kstop); break;
    case 15: rc = bandk_launch_k15(a, n, s, start, kstop); break;
    case 16: rc = bandk_launch_k16(a, n, s, start, kstop); break;
    case 17: rc = bandk_launch_k17(a, n, s, start, kstop); break;
    case 18: rc = bandk_launch_k18(a, n, s, start, kstop); break;
    case 19: rc = bandk_launch_k19(a, n, s, start, kstop); break;
    default: rc = bandk_launch_k20(a, n, s, start, kstop); break;
    }
    SMI_TRY(rc);
    if (after) SMI_HIP_CHECK(hipEventRecord(after, s));
    (void)tok;
    return SMI_SUCCESS;
}

// Initial depth-K sends from the current tile: columns 0..KC-1 and
// Y-KC..Y-1 packed [row][k], and the four K x KC corner blocks.
__global__ __launch_bounds__(256) void packk_kernel(const float *in, int X, int Y, int K, int KC, HaloK h) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= X * KC) return;
    const int p = t / KC, k = t - p * KC;
    const float *row = in + (size_t)p * Y;
    const float vl = row[k], vr = row[Y - KC + k];
    h.send_left[t] = vl;
    h.send_right[t] = vr;
    if (p < K) {
        h.send_corner[0][p * KC + k] = vl;
        h.send_corner[1][p * KC + k] = vr;
    }
    if (p >= X - K) {
        h.send_corner[2][(p - (X - K)) * KC + k] = vl;
        h.send_corner[3][(p - (X - K)) * KC + k] = vr;
    }
}

int launch_packk(const float *in, int rows, int cols, int K, const HaloK &h, hipStream_t s) {
    const int KC = kc_of(K);
    SMI_ARG_CHECK(cols >= 2 * KC && rows >= K, "packk: tile smaller than 2KC columns");
    const int n = rows * KC;
    hipLaunchKernelGGL(packk_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, rows, cols, K, KC, h);
    SMI_HIP_CHECK(hipGetLastError());
    return SMI_SUCCESS;
}


}  // namespace smi
