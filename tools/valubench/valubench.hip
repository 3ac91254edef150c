// valubench.hip -- VALU issue-rate microbenchmark on MI355X: waves/SIMD x
// instruction mix (v_add_f32, v_pk_add_f32, v_add_f32_dpp), 8 independent
// chains per lane; reports wave-instructions per SIMD-cycle (clock64) and the
// shader clock (cycles / wall time).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(256) void valu(float *out, int iters, long long *cyc) {
    float a[8];
    f2 p[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = threadIdx.x * 0.001f + i;
        p[i] = f2{a[i], a[i] + 1.f};
    }
    const float b = 1.0001f;
    const f2 pb = {1.0001f, 1.0002f};
    long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if constexpr (MODE == 0) a[i] = __fadd_rn(a[i], b);
                if constexpr (MODE == 1) p[i] = p[i] + pb;
                if constexpr (MODE == 2) {
                    const float s = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, a[i]), 0x138, 0xf, 0xf, true));
                    a[i] = __fadd_rn(a[i], s);
                }
            }
        }
    }
    long long t1 = clock64();
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += a[i] + p[i].x + p[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main() {
    float *out;
    long long *cyc;
    hipMalloc(&out, 1 << 26);
    hipMalloc(&cyc, 8);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 2000;
    for (int mode = 0; mode < 3; ++mode) {
        for (int wps : {1, 2, 4, 8}) {  // waves per SIMD: blocks of 4 waves, wps blocks per CU
            const int blocks = cus * wps;
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            auto launch = [&]() {
                if (mode == 0) hipLaunchKernelGGL(valu<0>, dim3(blocks), dim3(256), 0, 0, out, iters, cyc);
                if (mode == 1) hipLaunchKernelGGL(valu<1>, dim3(blocks), dim3(256), 0, 0, out, iters, cyc);
                if (mode == 2) hipLaunchKernelGGL(valu<2>, dim3(blocks), dim3(256), 0, 0, out, iters, cyc);
            };
            launch();
            hipDeviceSynchronize();
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            long long c = 0;
            hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            const double instr_per_wave = (double)iters * 16 * 8 * (mode == 2 ? 2 : 1);
            const double waves_per_simd = wps;
            printf("{\"mode\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"wave0_cycles\": %lld, "
                   "\"clock_GHz_est\": %.3f, \"wave_instr_per_simd_cycle\": %.3f}\n",
                   mode == 0 ? "v_add_f32" : mode == 1 ? "v_pk_add_f32" : "mov_dpp+v_add_f32", wps, ms, c,
                   c / (ms * 1e6), instr_per_wave * waves_per_simd / c);
        }
    }
    return 0;
}
