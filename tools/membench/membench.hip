// membench.hip -- HBM rate of the sweeps' access pattern without the
// stencil: every wave walks a column strip down a block of rows, reading a
// C x 16-byte-per-lane chunk of each row and writing it to the other buffer
// (what a sweep wave moves per input row), D rows of loads in flight.
// Compares the pattern's rate with a linear float4 copy of the same bytes.
//   membench [rows=8192] [cols=8192]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                         \
        }                                                                                    \
    } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_nt(float4 *p, const float4 &v) {
    __builtin_nontemporal_store(v4f{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f *>(p));
}

__global__ void copy_kernel(const float4 *__restrict__ in, float4 *__restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        st_nt(out + i, in[i]);
}

// wave w: strip w % nstrips (band-major: consecutive waves = neighbouring
// strips of one band) or w / nbands (strip-major), rows of band b
__device__ __forceinline__ int xcd_remap(int b, int nb) {  // as smi_amd/csrc/stencil_common.h
    const int q = nb >> 3, r = nb & 7, x = b & 7;
    const int base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    return base + (b >> 3);
}

template <int C, int D>
__global__ __launch_bounds__(256) void walk_kernel(const float4 *__restrict__ in, float4 *__restrict__ out, int rows,
                                                   int cols4, int nstrips, int nbands, int strip_major, int remap) {
    const int blk = remap ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int w = __builtin_amdgcn_readfirstlane((int)(blk * 4 + (threadIdx.x >> 6)));
    const int lane = threadIdx.x & 63;
    if (w >= nstrips * nbands) return;
    const int s = strip_major ? w / nbands : w % nstrips;
    const int b = strip_major ? w % nbands : w / nstrips;
    const int r0 = (int)((long)rows * b / nbands), r1 = (int)((long)rows * (b + 1) / nbands);
    const int c0 = s * 64 * C + lane;  // float4 column of this lane's first chunk element
    float4 ring[D][C];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int r = min(r0 + d, rows - 1);
            ring[d][c] = c0 + 64 * c < cols4 ? in[(size_t)r * cols4 + c0 + 64 * c] : make_float4(0, 0, 0, 0);
        }
    for (int r = r0; r < r1; r += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            if (r + d < r1) {
#pragma unroll
                for (int c = 0; c < C; ++c)
                    if (c0 + 64 * c < cols4) st_nt(out + (size_t)(r + d) * cols4 + c0 + 64 * c, ring[d][c]);
            }
            const int rn = min(r + d + D, rows - 1);
#pragma unroll
            for (int c = 0; c < C; ++c)
                ring[d][c] = c0 + 64 * c < cols4 ? in[(size_t)rn * cols4 + c0 + 64 * c] : make_float4(0, 0, 0, 0);
        }
    }
}

// the sweeps' window geometry: a wave reads 256 columns (one float4 per
// lane) starting AP columns left of its strip and stores the middle SW
// columns of each row (lanes AP/4 .. (AP+SW)/4 - 1), strips SW apart.
template <int D, int NT>
__global__ __launch_bounds__(256) void sweepgeo_kernel(const float *__restrict__ in, float *__restrict__ out, int rows,
                                                       int cols, int sw, int ap, int nstrips, int nbands, int remap,
                                                       int alt, int rapron) {
    const int blk = remap ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int w = __builtin_amdgcn_readfirstlane((int)(blk * 4 + (threadIdx.x >> 6)));
    const int lane = threadIdx.x & 63;
    if (w >= nstrips * nbands) return;
    const int s = w % nstrips, b = w / nstrips;  // band-major
    const int o0 = (int)((long)rows * b / nbands), o1 = (int)((long)rows * (b + 1) / nbands);
    // the walk reads rapron rows before and after its band (the sweeps' row
    // cones) and stores its band's rows; alt: odd bands walk upwards
    const bool up = alt && (b & 1);
    const int n = (o1 - o0) + 2 * rapron;
    const int rb = up ? o1 - 1 + rapron : o0 - rapron;
    auto row_of = [&](int t) { return min(max(up ? rb - t : rb + t, 0), rows - 1); };
    const int cb = s * sw - ap + 4 * lane;
    const int cl = min(max(cb, 0), cols - 4);
    const bool st = 4 * lane >= ap && 4 * lane < ap + sw && cb >= 0 && cb < cols;
    float4 ring[D];
#pragma unroll
    for (int d = 0; d < D; ++d) ring[d] = *reinterpret_cast<const float4 *>(in + (size_t)row_of(d) * cols + cl);
    for (int t = 0; t < n; t += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int ro = up ? rb - (t + d) : rb + (t + d);  // store the row just read (one row per read)
            if (t + d < n && st && ro >= o0 && ro < o1) {
                float4 *p = reinterpret_cast<float4 *>(out + (size_t)ro * cols + cb);
                if (NT) st_nt(p, ring[d]);
                else *p = ring[d];
            }
            ring[d] = *reinterpret_cast<const float4 *>(in + (size_t)row_of(t + d + D) * cols + cl);
        }
    }
}

template <typename F>
static float timeit(F f, int reps = 20) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 5; ++i) f();
    std::vector<float> ms;
    for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(a, 0));
        f();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float m;
        CK(hipEventElapsedTime(&m, a, b));
        ms.push_back(m);
    }
    std::sort(ms.begin(), ms.end());
    return ms[reps / 2];
}

template <int C, int D>
static void walk(const float4 *in, float4 *out, int rows, int cols, int waves, int strip_major, int remap) {
    const int cols4 = cols / 4, nstrips = (cols4 + 64 * C - 1) / (64 * C);
    const int nbands = std::max(1, waves / nstrips);
    const int nw = nstrips * nbands, blocks = (nw + 3) / 4;
    const float ms = timeit([&] {
        hipLaunchKernelGGL((walk_kernel<C, D>), dim3(blocks), dim3(256), 0, 0, in, out, rows, cols4, nstrips, nbands,
                           strip_major, remap);
    });
    const double bytes = 2.0 * rows * cols * 4;
    printf("{\"pattern\": \"walk\", \"chunk_bytes\": %d, \"D\": %d, \"waves\": %d, \"strips\": %d, \"bands\": %d, "
           "\"order\": \"%s\", \"xcd_remap\": %d, \"rows\": %d, \"ms\": %.5f, \"TBs\": %.3f}\n",
           C * 1024, D, nw, nstrips, nbands, strip_major ? "strip" : "band", remap, rows, ms, bytes / (ms * 1e-3) / 1e12);
    fflush(stdout);
}

template <int NT>
static void sweepgeo(const float4 *in, float4 *out, int rows, int cols, int sw, int ap, int waves, int remap,
                     int alt = 0, int rapron = 0) {
    const int nstrips = (cols + sw - 1) / sw, nbands = std::max(1, waves / nstrips);
    const int nw = nstrips * nbands, blocks = (nw + 3) / 4;
    const float ms = timeit([&] {
        hipLaunchKernelGGL((sweepgeo_kernel<3, NT>), dim3(blocks), dim3(256), 0, 0, (const float *)in, (float *)out, rows,
                           cols, sw, ap, nstrips, nbands, remap, alt, rapron);
    });
    const double bytes = 2.0 * rows * cols * 4;
    printf("{\"pattern\": \"sweep geometry\", \"store_cols\": %d, \"apron\": %d, \"nt\": %d, \"waves\": %d, "
           "\"xcd_remap\": %d, \"alt_up\": %d, \"row_apron\": %d, \"rows\": %d, \"ms\": %.5f, \"TBs_compulsory\": %.3f}\n",
           sw, ap, NT, nw, remap, alt, rapron, rows, ms, bytes / (ms * 1e-3) / 1e12);
    fflush(stdout);
}

int main(int argc, char **argv) {
    const int rows = argc > 1 ? atoi(argv[1]) : 8192, cols = argc > 2 ? atoi(argv[2]) : 8192;
    const size_t n4 = (size_t)rows * cols / 4;
    float4 *a, *b;
    CK(hipMalloc(&a, n4 * 16));
    CK(hipMalloc(&b, n4 * 16));
    CK(hipMemset(a, 0, n4 * 16));
    const float ms = timeit([&] { hipLaunchKernelGGL(copy_kernel, dim3(8192), dim3(256), 0, 0, a, b, n4); });
    printf("{\"pattern\": \"copy\", \"ms\": %.5f, \"TBs\": %.3f}\n", ms, 2.0 * n4 * 16 / (ms * 1e-3) / 1e12);
    sweepgeo<1>(a, b, rows, cols, 216, 20, 2048, 1);
    sweepgeo<1>(a, b, rows, cols, 216, 20, 2048, 1, 1, 0);
    sweepgeo<1>(a, b, rows, cols, 216, 20, 2048, 1, 0, 20);
    sweepgeo<1>(a, b, rows, cols, 216, 20, 2048, 1, 1, 20);
    sweepgeo<1>(a, b, rows, cols, 216, 20, 2048, 1, 0, 10);
    sweepgeo<1>(a, b, rows, cols, 216, 20, 4096, 1, 0, 20);
    return 0;
}
