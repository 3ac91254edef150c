// xbench.hip -- timing + bit-check harness for the shared-boundary sweep
// (smi_amd/csrc/stencilx.h) next to the rotating-ring sweep it replaces
// (stencild.h); experiments only, not part of libsmi_amd.
//
//   xbench <N> [launches] [warm-up launches]
//   env: XB_NB (blocks per interior strip, even), XB_DCONE (extra rows a cone
//        start costs, sets the cone-start weight), XB_CE16 (edge-column strip
//        extra work, 16ths), XB_KERNEL (x | d | both)
//
// Runs each kernel over the whole N x N tile (global edges inside), checks it
// bit for bit against K launches of a plain one-step kernel, then times
// back-to-back ping-pong passes with HIP events between launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "stencilx.h"

#ifndef KSTEPS
#define KSTEPS 20
#endif
#ifndef VARIANT_NAME
#define VARIANT_NAME "x"
#endif

namespace smi {
void set_error(const std::string &) {}
}

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(2);                                                                         \
        }                                                                                    \
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

static int env(const char *k, int d) { return getenv(k) ? atoi(getenv(k)) : d; }

struct Strips {
    int nstrips = 0, n_int = 0, int0 = -1, nce = 0, ce[4] = {-1, -1, -1, -1};
};
static Strips strips(int n, int K) {
    const int KC = 4 * ((K + 3) / 4), SW = 256 - 2 * KC;
    Strips s;
    s.nstrips = (n + SW - 1) / SW;
    for (int st = 0; st < s.nstrips; ++st) {
        const int cs = st * SW;
        if (cs - KC <= 0 || cs - KC + 256 >= n) s.ce[s.nce++] = st;
        else {
            if (s.int0 < 0) s.int0 = st;
            ++s.n_int;
        }
    }
    return s;
}

template <typename F>
static void timeit(const char *name, int K, int n, int launches, int warm, F launch, const float *got_dev,
                   const float *want_dev, const char *extra) {
    const size_t cells = (size_t)n * n;
    launch(false);
    CK(hipDeviceSynchronize());
    std::vector<float> got(cells), want(cells);
    CK(hipMemcpy(got.data(), got_dev, cells * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(want.data(), want_dev, cells * 4, hipMemcpyDeviceToHost));
    long bad = 0;
    for (size_t i = 0; i < cells; ++i)
        if (memcmp(&got[i], &want[i], 4) != 0) {
            if (bad++ < 5) fprintf(stderr, "%s mismatch (%zu,%zu): %a vs %a\n", name, i / n, i % n, got[i], want[i]);
        }
    bool flip = true;
    for (int i = 0; i < warm; ++i) {
        launch(flip);
        flip = !flip;
    }
    std::vector<hipEvent_t> ev(launches + 1);
    for (auto &evt : ev) CK(hipEventCreate(&evt));
    CK(hipEventRecord(ev[0], 0));
    for (int i = 0; i < launches; ++i) {
        launch(flip);
        flip = !flip;
        CK(hipEventRecord(ev[i + 1], 0));
    }
    CK(hipDeviceSynchronize());
    std::vector<float> ms(launches);
    for (int i = 0; i < launches; ++i) CK(hipEventElapsedTime(&ms[i], ev[i], ev[i + 1]));
    std::sort(ms.begin(), ms.end());
    const double med = ms[launches / 2];
    printf("{\"variant\": \"%s\", \"kernel\": \"%s\", \"K\": %d, \"n\": %d, %s, \"mismatches\": %ld, \"ms_med\": %.5f, "
           "\"ms_min\": %.5f, \"GCells\": %.1f}\n",
           VARIANT_NAME, name, K, n, extra, bad, med, ms[0], (double)n * n * K / med / 1e6);
    fflush(stdout);
    for (auto &evt : ev) CK(hipEventDestroy(evt));
}

int main(int argc, char **argv) {
    constexpr int K = KSTEPS;
    const int n = argc > 1 ? atoi(argv[1]) : 8192;
    const int launches = argc > 2 ? atoi(argv[2]) : 100;
    const int warm = argc > 3 ? atoi(argv[3]) : 100;
    const std::string which = getenv("XB_KERNEL") ? getenv("XB_KERNEL") : "both";
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
    for (int k = 0; k < K; ++k) {
        hipLaunchKernelGGL(ref_step, dim3((n + 255) / 256, n), dim3(256), 0, 0, r0, r1, n);
        std::swap(r0, r1);
    }
    CK(hipDeviceSynchronize());
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const Strips st = strips(n, K);
    smi::SweepKArgs args{a, b, n, n, 0, n, 0, n, 1, 1, 1, 1};
    char extra[512];

#ifndef XB_NO_X
    if (which == "x" || which == "both") {
        int per_cu = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, smi::sweepx_kernel<K>, 256, 0));
        hipFuncAttributes fa;
        CK(hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(smi::sweepx_kernel<K>)));
        const int waves = env("XB_WAVES", per_cu * cus * 4);
        const int ce16 = 16 + env("XB_CE16", 10);
        int nb = env("XB_NB", 0);
        if (nb <= 0) nb = (int)((long)waves * 16 / ((long)st.n_int * 16 + (long)st.nce * ce16)) & ~1;
        smi::SweepXGeom g{};
        g.nstrips = st.nstrips;
        g.n_int = st.n_int;
        g.int0 = st.int0;
        for (int k = 0; k < 4; ++k) g.ce[k] = st.ce[k];
        g.nb = nb;
        g.nb_ce = std::max(nb, (nb * ce16 / 16) & ~1);
        const int bavg = n / nb, dcone = env("XB_DCONE", 30);
        g.wcone = std::max(4, std::min(16, 16 * bavg / (bavg + dcone)));
        g.tasks = g.n_int * g.nb + st.nce * g.nb_ce;
        const int blocks = (g.tasks + 3) / 4;
        snprintf(extra, sizeof extra,
                 "\"vgprs\": %d, \"lds\": %zu, \"per_cu\": %d, \"nb\": %d, \"nb_ce\": %d, \"wcone\": %d, \"tasks\": %d, "
                 "\"resident\": %d",
                 fa.numRegs, fa.sharedSizeBytes, per_cu, g.nb, g.nb_ce, g.wcone, g.tasks, waves);
#ifdef SMI_X_WAVETIMES
        unsigned long long *wt = nullptr;
        CK(hipMalloc(&wt, (size_t)3 * 8 * g.tasks));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(smi::g_wavetimes), &wt, sizeof(wt)));
#endif
        timeit("sweepx", K, n, launches, warm,
               [&](bool flip) {
                   smi::SweepKArgs la = args;
                   if (flip) {
                       la.in = args.out;
                       la.out = const_cast<float *>(args.in);
                   }
                   hipLaunchKernelGGL((smi::sweepx_kernel<K>), dim3(blocks), dim3(256), 0, 0, la, g);
               },
               b, r0, extra);
#ifdef SMI_X_WAVETIMES
        {
            // the last launch's waves: per SIMD (xcc, se, sh, cu, simd), the
            // older / younger wave's start and end relative to the launch start
            std::vector<unsigned long long> h(3 * (size_t)g.tasks);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), wt, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull, t1 = 0;
            for (int i = 0; i < g.tasks; ++i) t0 = std::min(t0, h[3 * i + 1]), t1 = std::max(t1, h[3 * i + 2]);
            FILE *f = fopen("wavetimes.csv", "w");
            fprintf(f, "wave,xcc,hw_id,wave_slot,simd,cu,sh,se,start,end\n");
            for (int i = 0; i < g.tasks; ++i) {
                const unsigned hw = (unsigned)h[3 * i], xcc = (unsigned)(h[3 * i] >> 32);
                fprintf(f, "%d,%u,%u,%u,%u,%u,%u,%u,%llu,%llu\n", i, xcc, hw, hw & 15, (hw >> 4) & 3, (hw >> 8) & 15,
                        (hw >> 12) & 1, (hw >> 13) & 7, h[3 * i + 1] - t0, h[3 * i + 2] - t0);
            }
            fclose(f);
            printf("{\"wavetimes\": \"wavetimes.csv\", \"launch_cycles\": %llu}\n", t1 - t0);
        }
#endif
        CK(hipMemset(b, 0, cells * 4));
        CK(hipMemcpy(a, h.data(), cells * 4, hipMemcpyHostToDevice));
    }
#endif
#ifndef XB_NO_D
    if (which.find('d') != std::string::npos || which == "both") {
        int per_cu = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, smi::sweepd_kernel<K>, 256, 0));
        hipFuncAttributes fa;
        CK(hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(smi::sweepd_kernel<K>)));
        const int waves = per_cu * cus * 4;
        // the library's geometry (stencild.hip sweepd_geometry), defaults 10/16, 6/16
        const int ce16 = 16 + 10, rev16 = 6;
        smi::SweepDGeom g{};
        g.nstrips = st.nstrips;
        g.n_int = st.n_int;
        g.int0 = st.int0;
        for (int k = 0; k < 4; ++k) g.ce[k] = st.ce[k];
        g.wlast = std::max(4, std::min(16, 256 / (16 + rev16)));
        g.nrb = (int)((long)waves * 16 / ((long)st.n_int * 16 + (long)st.nce * ce16));
        g.nrb_ce = std::max(g.nrb, g.nrb * ce16 / 16);
        g.tasks = g.n_int * g.nrb + st.nce * g.nrb_ce;
        const int blocks = (g.tasks + 3) / 4;
        snprintf(extra, sizeof extra, "\"vgprs\": %d, \"per_cu\": %d, \"nrb\": %d, \"tasks\": %d, \"resident\": %d",
                 fa.numRegs, per_cu, g.nrb, g.tasks, waves);
        timeit("sweepd", K, n, launches, warm,
               [&](bool flip) {
                   smi::SweepKArgs la = args;
                   if (flip) {
                       la.in = args.out;
                       la.out = const_cast<float *>(args.in);
                   }
                   hipLaunchKernelGGL((smi::sweepd_kernel<K>), dim3(blocks), dim3(256), 0, 0, la, g);
               },
               b, r0, extra);
    }
#endif
#ifdef SMI_X_UNEQUAL
    if (which.find('u') != std::string::npos) {
        // the d geometry with nrb, nrb_ce even; pair tasks split fo/256 : rest
        int per_cu = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, smi::sweepu_kernel<K>, 256, 0));
        hipFuncAttributes fa;
        CK(hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(smi::sweepu_kernel<K>)));
        const int waves = per_cu * cus * 4;
        const int ce16 = 16 + 10, rev16 = 6;
        const int fo = env("XB_FO", 167);
        smi::SweepDGeom g{};
        g.nstrips = st.nstrips;
        g.n_int = st.n_int;
        g.int0 = st.int0;
        for (int k = 0; k < 4; ++k) g.ce[k] = st.ce[k];
        g.wlast = std::max(4, std::min(16, 256 / (16 + rev16)));
        g.nrb = (int)((long)waves * 16 / ((long)st.n_int * 16 + (long)st.nce * ce16)) & ~1;
        g.nrb_ce = std::max(g.nrb, g.nrb * ce16 / 16) & ~1;
        g.tasks = g.n_int * g.nrb + st.nce * g.nrb_ce;
        const int P = (((g.tasks / 2 + 3) / 4) + 7) & ~7;  // b and b + P on one XCD
        // every half at least K + 1 rows (the shortest: the young half of a pair)
        const int bmin = n / g.nrb_ce;
        if (bmin * (256 - std::max(fo, 256 - fo)) / 256 < K + 1) {
            fprintf(stderr, "sweepu: halves too short\n");
            return 1;
        }
        snprintf(extra, sizeof extra,
                 "\"vgprs\": %d, \"per_cu\": %d, \"nrb\": %d, \"nrb_ce\": %d, \"tasks\": %d, \"resident\": %d, "
                 "\"P\": %d, \"fo\": %d",
                 fa.numRegs, per_cu, g.nrb, g.nrb_ce, g.tasks, waves, P, fo);
#ifdef SMI_X_WAVETIMES
        unsigned long long *wt = nullptr;
        CK(hipMalloc(&wt, (size_t)5 * 8 * g.tasks));
        CK(hipMemset(wt, 0, (size_t)5 * 8 * g.tasks));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(smi::g_wavetimes), &wt, sizeof(wt)));
#endif
        timeit("sweepu", K, n, launches, warm,
               [&](bool flip) {
                   smi::SweepKArgs la = args;
                   if (flip) {
                       la.in = args.out;
                       la.out = const_cast<float *>(args.in);
                   }
                   hipLaunchKernelGGL((smi::sweepu_kernel<K>), dim3(2 * P), dim3(256), 0, 0, la, g, P, fo);
               },
               b, r0, extra);
#ifdef SMI_X_WAVETIMES
        {
            std::vector<unsigned long long> h(5 * (size_t)g.tasks);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), wt, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull;
            unsigned long long rt0 = ~0ull;
            for (int i = 0; i < g.tasks; ++i)
                if (h[5 * i + 4]) t0 = std::min(t0, h[5 * i + 1]), rt0 = std::min(rt0, h[5 * i + 3]);
            FILE *f = fopen("wavetimes_u.csv", "w");
            fprintf(f, "wave,xcc,hw_id,wave_slot,simd,cu,sh,se,start,end,rstart,rend\n");
            for (int i = 0; i < g.tasks; ++i) {
                if (!h[5 * i + 4]) continue;
                const unsigned hw = (unsigned)h[5 * i], xcc = (unsigned)(h[5 * i] >> 32);
                fprintf(f, "%d,%u,%u,%u,%u,%u,%u,%u,%llu,%llu,%llu,%llu\n", i, xcc, hw, hw & 15, (hw >> 4) & 3,
                        (hw >> 8) & 15, (hw >> 12) & 1, (hw >> 13) & 7, h[5 * i + 1] - t0, h[5 * i + 2] - t0,
                        h[5 * i + 3] - rt0, h[5 * i + 4] - rt0);
            }
            fclose(f);
        }
#endif
    }
#endif
    return 0;
}
