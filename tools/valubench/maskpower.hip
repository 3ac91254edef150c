// maskpower.hip -- does an exec-masked lane cost power on MI355X?
//
// The K = 20 sweep is bound by the chip's power cap, and its
// apron lanes compute ~7 % of the lane-levels for columns no output needs.
// This runs the sweep's add mix (v_add_f32, v_add_f32 with a DPP row shift,
// v_pk_add_f32) for ~1 s per setting on every SIMD (2 waves each, as the
// sweep) with only `active` lanes of each wave enabled, and prints the time
// per iteration: if masked lanes save power, fewer active lanes run faster
// at the cap.  usage: maskpower [seconds per setting]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void mix(float *out, int iters, int active) {
    const int lane = threadIdx.x & 63;
    float a[8];
    f2 p[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 0.001f + i;
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = f2{a[i], a[i + 4]};
    const float b = 1.0001f;
    const f2 pb = {1.0001f, 1.0002f};
    if (lane < active) {
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int r = 0; r < 8; ++r) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float s = __builtin_bit_cast(
                        float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, a[i]), 0x138, 0xf, 0xf, true));
                    a[i] = __fadd_rn(__fadd_rn(a[i], s), b);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) p[i] = p[i] + pb;
            }
        }
    }
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += a[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc += p[i].x + p[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main(int argc, char **argv) {
    const double secs = argc > 1 ? atof(argv[1]) : 1.0;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess || cus <= 0) {
        fprintf(stderr, "no device\n");
        return 1;
    }
    float *out;
    if (hipMalloc(&out, (size_t)cus * 2 * 256 * sizeof(float)) != hipSuccess) return 1;
    const int blocks = cus * 2;  // 4 waves per block: 2 waves per SIMD
    const int iters = 20000;
    const int settings[] = {64, 60, 56, 48, 32, 64};
    for (int active : settings) {
        // one launch to size the repetitions, then ~secs of back-to-back launches
        auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(mix, dim3(blocks), dim3(256), 0, 0, out, iters, active);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        const double one = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        const int reps = (int)(secs / one) + 1;
        t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(mix, dim3(blocks), dim3(256), 0, 0, out, iters, active);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        // lane-adds per launch: active lanes x waves x iters x (8 x (16 + 8))
        const double adds = (double)active * blocks * 4 * iters * 8 * (16 + 8);
        const double end = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
        printf("active %2d lanes: %.4f ms per launch (%d launches), %.2f T lane-adds/s, epoch %.3f - %.3f\n", active,
               t / reps * 1e3, reps, adds / (t / reps) / 1e12, end - t, end);
        fflush(stdout);
    }
    return 0;
}
