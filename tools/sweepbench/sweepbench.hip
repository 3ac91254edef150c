// sweepbench.hip -- standalone timing + bit-check harness for the K-step
// sweep kernel (experiments only; not part of libsmi_amd).
//
//   sweepbench <N> <ht> [launches] [warm-up launches]     ht <= 0: one round of resident waves
//
// Builds (tools/sweepbench/build.sh) the sweep over the whole tile (global
// edges inside), checks it bit for bit against K launches of a plain one-step
// kernel, then times `launches` back-to-back passes with HIP events around
// each.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

// SB_KERNEL: the header holding SweepK / sweepk_kernel<K> (default: the
// library's); experiments copy it to tools/sweepbench/ and edit the copy.
#ifndef SB_KERNEL
#define SB_KERNEL "stencilk.h"
#endif
#include SB_KERNEL

#ifndef KSTEPS
#define KSTEPS 12
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
    const int K = KSTEPS;
    const int n = argc > 1 ? atoi(argv[1]) : 8192;
    const int ht_arg = argc > 2 ? atoi(argv[2]) : -1;
    const int launches = argc > 3 ? atoi(argv[3]) : 200;
    const int warm = argc > 4 ? atoi(argv[4]) : 300;
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

    smi::SweepKArgs args{a, b, n, n, 0, n, 0, n, 1, 1, 1, 1};
    constexpr int KC = smi::SweepK<K, 3>::KC;
    const int sw = 256 - 2 * KC;
    int per_cu = 0, cus = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, smi::sweepk_kernel<K>, 256, 0));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int waves = per_cu * cus * 4;
    const int out_rows = args.row_hi - args.row_lo;
    const int nstrips = (args.col_hi - args.col_lo + sw - 1) / sw;
    int ht = ht_arg;
    if (ht <= 0) {
        const int per_strip = std::max(1, waves / nstrips);
        ht = std::max(2 * K, (out_rows + per_strip - 1) / per_strip);
    }
    int nrb = (out_rows + ht - 1) / ht;
#ifdef SB_EVEN_NRB
    nrb += nrb & 1;  // alternating walks: first block down, last block up
#endif
#ifdef SB_EVEN_NRB_DOWN
    if (nrb > 1) nrb -= nrb & 1;  // even, and never more waves than one round
#endif
    const int blocks = (int)(((long)nstrips * nrb + 3) / 4);
    // timing ping-pongs between the two buffers like a real run (reading the
    // same input every launch would let the 256 MB MALL hold part of it)
    bool flip = false;
    auto launch = [&]() {
        smi::SweepKArgs la = args;
        if (flip) {
            la.in = args.out;
            la.out = const_cast<float *>(args.in);
        }
        flip = !flip;
        hipLaunchKernelGGL((smi::sweepk_kernel<K>), dim3(blocks), dim3(256), 0, 0, la, nstrips, nrb);
    };
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> got(cells), want(cells);
    CK(hipMemcpy(got.data(), b, cells * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(want.data(), r0, cells * 4, hipMemcpyDeviceToHost));
    long bad = 0;
    for (int r = args.row_lo; r < args.row_hi; ++r)
        for (int c = args.col_lo; c < args.col_hi; ++c) {
            const size_t i = (size_t)r * n + c;
            if (memcmp(&got[i], &want[i], 4) != 0 && bad++ < 5)
                fprintf(stderr, "mismatch (%d,%d): %a vs %a\n", r, c, got[i], want[i]);
        }
    // warm the clock, then time
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
    const double cellsteps = (double)out_rows * (args.col_hi - args.col_lo) * K;
    const char *var = VARIANT_NAME;
    printf("{\"variant\": \"%s\", \"K\": %d, \"n\": %d, \"ht\": %d, \"nrb\": %d, \"nstrips\": %d, \"waves\": %d, "
           "\"resident\": %d, \"mismatches\": %ld, \"ms_mean\": %.5f, \"ms_med\": %.5f, \"GCells\": %.1f}\n",
           var, K, n, ht, nrb, nstrips, nstrips * nrb, waves, bad, mean, med, cellsteps / med / 1e6);
    return bad ? 1 : 0;
}
