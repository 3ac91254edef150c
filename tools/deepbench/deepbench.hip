// deepbench.hip -- timing + bit-check harness for the deep K-step sweep
// (smi_amd/csrc/stencild.h); experiments only, not part of libsmi_amd.
//
//   deepbench <N> [launches] [warm-up launches] [ht]
//
// Runs the sweep over the whole N x N tile (global edges inside), checks it
// bit for bit against K launches of a plain one-step kernel, then times
// back-to-back ping-pong passes with HIP events between launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "stencild.h"

#ifndef KSTEPS
#define KSTEPS 20
#endif
#ifndef VARIANT_NAME
#define VARIANT_NAME "deep"
#endif

namespace smi {
void set_error(const std::string &) {}
}

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(2);                                                                     \
        }                                                                                \
    } while (0)

__global__ void ref_step(const float *in, float *out, int n) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    const int r = blockIdx.y;
    if (c >= n) return;
    const size_t i = (size_t)r * n + c;
    if (r == 0 || r == n - 1 || c == 0 || c == n - 1) {
        out[i] = in[i];
        return;
    }
    out[i] = smi::jacobi(in[i + n], in[i - 1], in[i + 1], in[i - n]);
}

int main(int argc, char **argv) {
    constexpr int K = KSTEPS;
    const int n = argc > 1 ? atoi(argv[1]) : 8192;
    const int launches = argc > 2 ? atoi(argv[2]) : 100;
    const int warm = argc > 3 ? atoi(argv[3]) : 100;
    const int ht_arg = argc > 4 ? atoi(argv[4]) : 0;
    const size_t cells = (size_t)n * n;
    std::vector<float> h(cells);
    unsigned s = 12345;
    for (auto &v : h) {
        s = s * 1664525u + 1013904223u;
        v = (s >> 8) * (1.0f / 16777216.0f);
    }
    float *a, *b, *r0, *r1;
    CK(hipMalloc(&a, cells * 4));
    CK(hipMalloc(&b, cells * 4));
    CK(hipMalloc(&r0, cells * 4));
    CK(hipMalloc(&r1, cells * 4));
    CK(hipMemcpy(a, h.data(), cells * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(r0, a, cells * 4, hipMemcpyDeviceToDevice));
    CK(hipMemset(b, 0, cells * 4));
    for (int k = 0; k < K; ++k) {
        hipLaunchKernelGGL(ref_step, dim3((n + 255) / 256, n), dim3(256), 0, 0, r0, r1, n);
        std::swap(r0, r1);
    }
    CK(hipDeviceSynchronize());

    using S = smi::SweepD<K>;
    smi::SweepKArgs args{a, b, n, n, 0, n, 0, n, 1, 1, 1, 1};
    const int sw = 256 - 2 * S::KC;
    int per_cu = 0, cus = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, smi::sweepd_kernel<K>, 256, 0));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipFuncAttributes fa;
    CK(hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(smi::sweepd_kernel<K>)));
    const int waves = per_cu * cus * 4;
    // the library's geometry (stencild.hip sweepd_geometry), defaults ce16=4, rev16=2
    const int ce16 = getenv("CE16") ? atoi(getenv("CE16")) + 16 : 20;
    const int rev16 = getenv("REV16") ? atoi(getenv("REV16")) : 2;
    smi::SweepDGeom g{};
    const int KC = S::KC;
    g.nstrips = (n + sw - 1) / sw;
    g.ce[0] = g.ce[1] = g.ce[2] = g.ce[3] = -1;
    int nce = 0;
    g.int0 = -1;
    for (int st = 0; st < g.nstrips; ++st) {
        const int cs = st * sw;
        if (cs - KC <= 0 || cs - KC + 256 >= n) g.ce[nce++] = st;
        else { if (g.int0 < 0) g.int0 = st; ++g.n_int; }
    }
    g.wlast = std::max(4, std::min(16, 256 / (16 + rev16)));
    int nrb = ht_arg > 0 ? (n + ht_arg - 1) / ht_arg : (int)((long)waves * 16 / ((long)g.n_int * 16 + (long)nce * ce16));
    g.nrb = nrb;
    g.nrb_ce = std::max(nrb, nrb * ce16 / 16);
    g.tasks = g.n_int * g.nrb + nce * g.nrb_ce;
    const int nstrips = g.nstrips, ht = n / nrb;
    const int blocks = (g.tasks + 3) / 4;
    bool flip = false;
    auto launch = [&]() {
        smi::SweepKArgs la = args;
        if (flip) {
            la.in = args.out;
            la.out = const_cast<float *>(args.in);
        }
        flip = !flip;
        hipLaunchKernelGGL((smi::sweepd_kernel<K>), dim3(blocks), dim3(256), 0, 0, la, g);
    };
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> got(cells), want(cells);
    CK(hipMemcpy(got.data(), b, cells * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(want.data(), r0, cells * 4, hipMemcpyDeviceToHost));
    long bad = 0, bad_int = 0;
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) {
            const size_t i = (size_t)r * n + c;
            if (memcmp(&got[i], &want[i], 4) != 0) {
                if (bad++ < 3) fprintf(stderr, "mismatch (%d,%d): %a vs %a\n", r, c, got[i], want[i]);
                if (r > K && r < n - 1 - K && c > K && c < n - 1 - K) {
                    if (bad_int++ < 8)
                        fprintf(stderr, "interior mismatch (%d,%d) row-in-block %d col-in-strip %d: %a vs %a\n", r, c,
                                r % ht, c % sw, got[i], want[i]);
                }
            }
        }
    for (int i = 0; i < warm; ++i) launch();
    std::vector<hipEvent_t> ev(launches + 1);
    for (auto &evt : ev) CK(hipEventCreate(&evt));
    CK(hipEventRecord(ev[0], 0));
    for (int i = 0; i < launches; ++i) {
        launch();
        CK(hipEventRecord(ev[i + 1], 0));
    }
    CK(hipDeviceSynchronize());
    std::vector<float> ms(launches);
    for (int i = 0; i < launches; ++i) CK(hipEventElapsedTime(&ms[i], ev[i], ev[i + 1]));
    float total = 0;
    for (float m : ms) total += m;
    std::sort(ms.begin(), ms.end());
    const double mean = total / launches, med = ms[launches / 2];
    const double cellsteps = (double)n * n * K;
    printf("{\"variant\": \"%s\", \"K\": %d, \"LL\": %d, \"D\": %d, \"B\": %d, \"vgprs\": %d, \"n\": %d, \"ht\": %d, "
           "\"nrb\": %d, \"nstrips\": %d, \"waves\": %d, \"resident\": %d, \"mismatches\": %ld, \"mismatches_interior\": %ld, "
           "\"ms_mean\": %.5f, \"ms_med\": %.5f, \"ms_min\": %.5f, \"GCells\": %.1f, \"compulsory_frac\": %.4f}\n",
           VARIANT_NAME, K, S::LL, S::D, S::B, fa.numRegs, n, ht, nrb, nstrips, g.tasks, waves, bad, bad_int,
           mean, med, ms[0], cellsteps / med / 1e6, 8.0 * n * n / (med * 1e-3) / 8e12);
    return bad ? 1 : 0;
}
