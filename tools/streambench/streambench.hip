// streambench.hip -- cost of the two-stream pass schedule of a multi-rank
// stencil run, without the stencil: per pass a long streaming kernel (the
// interior stand-in: a 256 MiB copy) on the main stream and a short kernel
// (the band stand-in) on a second stream, joined by cross-stream event waits
// exactly as smi_stencil_run does.  Prints us per pass for each variant next
// to the main-stream kernels alone, as JSON lines.
//   streambench [passes]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                                 \
        }                                                                            \
    } while (0)

__global__ void copy_kernel(const float4 *__restrict__ in, float4 *__restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

// a few us of dependent VALU work per wave, no memory
__global__ void small_kernel(float *out, int iters) {
    float v = threadIdx.x;
    for (int i = 0; i < iters; ++i) v = v * 1.0000001f + 0.5f;
    if (v == -1.0f) out[threadIdx.x] = v;
}

// mode 13: the big kernel's waves wait on a device flag instead of a
// cross-stream wait packet; the band stand-in's last block releases it
__global__ void copy_wait_kernel(const float4 *__restrict__ in, float4 *__restrict__ out, size_t n,
                                 const unsigned *flag, unsigned target) {
    if (threadIdx.x == 0) {
        while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target)
            __builtin_amdgcn_s_sleep(2);
    }
    __syncthreads();
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

// mode 16 / 17: the flag is written by a one-thread kernel after the band
// stand-in on the comm stream (the band's own end-of-kernel release makes its
// stores visible); the big kernel's checking blocks (16: the first 64, 17: all)
// read it with a relaxed device-coherent load and pay the acquire (L2
// invalidate) only when they had to wait
__global__ void set_flag_kernel(unsigned *flag, unsigned value) {
    __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void copy_check_kernel(const float4 *__restrict__ in, float4 *__restrict__ out, size_t n,
                                  const unsigned *flag, unsigned target, unsigned checkers) {
    if (blockIdx.x < checkers) {
        if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) <
            target) {
            while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) <
                   target)
                __builtin_amdgcn_s_sleep(2);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
    }
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

// mode 18: a one-wave gate kernel before the big one on the main stream
// spins on the flag (relaxed, device-coherent); the big kernel is unchanged
__global__ void gate_kernel(const unsigned *flag, unsigned target) {
    while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) <
           target)
        __builtin_amdgcn_s_sleep(2);
}

__global__ void small_flag_kernel(float *out, int iters, unsigned *count, unsigned *flag, unsigned value) {
    float v = threadIdx.x;
    for (int i = 0; i < iters; ++i) v = v * 1.0000001f + 0.5f;
    if (v == -1.0f) out[threadIdx.x] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned done = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1;
        if (done == value * gridDim.x) __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

struct Ctx {
    float4 *a, *b;
    size_t n;
    float *sink;
    hipStream_t s, cs;
    hipEvent_t e_int, e_band;
    uint32_t *f_int, *f_band;  // hipMallocSignalMemory counters (mode 7)
    unsigned *dflag, *dcount;  // device flag + block counter (mode 13)
    static constexpr int kPool = 4096;
    hipEvent_t pool[kPool];
};
constexpr int kPool = Ctx::kPool;

static void big(Ctx &c, int p) {
    hipLaunchKernelGGL(copy_kernel, dim3(4096), dim3(256), 0, c.s, p & 1 ? c.b : c.a, p & 1 ? c.a : c.b, c.n);
}
static void small(Ctx &c, hipStream_t st) { hipLaunchKernelGGL(small_kernel, dim3(800), dim3(64), 0, st, c.sink, 2000); }
// a band stand-in that runs ~40 us: its completion must not gate the next big kernel
static void small_long(Ctx &c, hipStream_t st) {
    hipLaunchKernelGGL(small_kernel, dim3(16), dim3(64), 0, st, c.sink, 3000);
}
// the same launches with the completion event carried by the dispatch itself
static void big_ev(Ctx &c, int p, hipEvent_t stop, hipStream_t st = nullptr) {
    hipExtLaunchKernelGGL(copy_kernel, dim3(4096), dim3(256), 0, st ? st : c.s, nullptr, stop, 0, p & 1 ? c.b : c.a,
                          p & 1 ? c.a : c.b, c.n);
}
static void small_ev(Ctx &c, hipStream_t st, hipEvent_t stop) {
    hipExtLaunchKernelGGL(small_kernel, dim3(800), dim3(64), 0, st, nullptr, stop, 0, c.sink, 2000);
}

// mode 0: big kernels alone; 1: + small kernel on cs, no dependencies;
// 2: the stencil schedule (cs: [wait int(t-1)] small(t) rec band(t);
//    s: big(t) rec int(t) [wait band(t)])
// 3: as 2, the small kernel on the main stream before big (no second stream)
// 4-6: the completion events carried by the kernel dispatches
// (hipExtLaunchKernelGGL stop events), see run()
// 7: as 2 with stream memory operations (write / wait value) for the joins
// 8 / 9: as 2 with a ~40 us second-stream kernel, events re-recorded every
// pass (8) or fresh per pass (9): does a wait see the record current when it
// was enqueued, or a later one?
// 10 / 11: as 2 / 8 with the main kernel's completion event carried by its
// dispatch (hipExtLaunchKernelGGL) instead of a record packet
// 12: one stream, the big kernel launched with hipExtAnyOrderLaunch after the
// small one; 13: no wait packet on the main stream: the big kernel's blocks
// wait on a device flag the small kernel's last block releases (round 5)
// 14 / 15: the streams swap roles every pass so that the wait before each
// big kernel is armed while its predecessor still runs (round 5)
static double run(Ctx &c, int mode, int passes) {
    CK(hipDeviceSynchronize());
    if (mode == 13 || mode >= 16) {
        CK(hipMemset(c.dflag, 0, 4));
        CK(hipMemset(c.dcount, 0, 4));
        CK(hipDeviceSynchronize());
    }
    if (mode == 7) {  // counters restart at 0 (nothing pending on them now)
        CK(hipStreamWriteValue32(c.s, c.f_int, 0u, 0));
        CK(hipStreamWriteValue32(c.s, c.f_band, 0u, 0));
        CK(hipDeviceSynchronize());
    }
    auto t0 = std::chrono::steady_clock::now();
    for (int p = 0; p < passes; ++p) {
        if (mode == 0) {
            big(c, p);
        } else if (mode == 1) {
            small(c, c.cs);
            big(c, p);
        } else if (mode == 2) {
            small(c, c.cs);
            CK(hipEventRecord(c.e_band, c.cs));
            big(c, p);
            CK(hipEventRecord(c.e_int, c.s));
            CK(hipStreamWaitEvent(c.s, c.e_band, 0));
            CK(hipStreamWaitEvent(c.cs, c.e_int, 0));
        } else if (mode == 10 || mode == 11) {
            // 10: as 2, the main kernel's completion event carried by its
            // dispatch (no record packet on the main stream); 11: the same
            // with the long band stand-in
            if (mode == 10) small(c, c.cs); else small_long(c, c.cs);
            CK(hipEventRecord(c.e_band, c.cs));
            big_ev(c, p, c.e_int);
            CK(hipStreamWaitEvent(c.s, c.e_band, 0));
            CK(hipStreamWaitEvent(c.cs, c.e_int, 0));
        } else if (mode == 8 || mode == 9) {
            // the stencil schedule with a long band stand-in; 8 re-records
            // two events every pass, 9 takes fresh events for every pass
            hipEvent_t eb = c.e_band, ei = c.e_int;
            if (mode == 9) {
                eb = c.pool[(2 * p) % kPool];
                ei = c.pool[(2 * p + 1) % kPool];
            }
            small_long(c, c.cs);
            CK(hipEventRecord(eb, c.cs));
            big(c, p);
            CK(hipEventRecord(ei, c.s));
            CK(hipStreamWaitEvent(c.s, eb, 0));
            CK(hipStreamWaitEvent(c.cs, ei, 0));
        } else if (mode == 7) {
            // as 2 with stream memory operations: monotone pass counters
            small(c, c.cs);
            CK(hipStreamWriteValue32(c.cs, c.f_band, (uint32_t)(p + 1), 0));
            big(c, p);
            CK(hipStreamWriteValue32(c.s, c.f_int, (uint32_t)(p + 1), 0));
            CK(hipStreamWaitValue32(c.s, c.f_band, (uint32_t)(p + 1), hipStreamWaitValueGte, 0xFFFFFFFFu));
            CK(hipStreamWaitValue32(c.cs, c.f_int, (uint32_t)(p + 1), hipStreamWaitValueGte, 0xFFFFFFFFu));
        } else if (mode == 12) {
            // one stream: the band stand-in, then the big kernel launched
            // with hipExtAnyOrderLaunch (no barrier bit: may it overlap?)
            small(c, c.s);
            hipExtLaunchKernelGGL(copy_kernel, dim3(4096), dim3(256), 0, c.s, nullptr, nullptr, hipExtAnyOrderLaunch,
                                  p & 1 ? c.b : c.a, p & 1 ? c.a : c.b, c.n);
        } else if (mode == 13) {
            // cs: [wait big(t-1)] band(t) -> flag = t + 1 (its last block);
            // s: big(t) back to back, its blocks wait for flag >= t (band(t-1))
            if (p > 0) CK(hipStreamWaitEvent(c.cs, c.e_int, 0));
            hipLaunchKernelGGL(small_flag_kernel, dim3(800), dim3(64), 0, c.cs, c.sink, 2000, c.dcount, c.dflag,
                               (unsigned)(p + 1));
            hipExtLaunchKernelGGL(copy_wait_kernel, dim3(4096), dim3(256), 0, c.s, nullptr, c.e_int, 0,
                                  p & 1 ? c.b : c.a, p & 1 ? c.a : c.b, c.n, (const unsigned *)c.dflag, (unsigned)p);
        } else if (mode == 16 || mode == 17) {
            // cs: [wait big(t-1)] band(t), set flag = t + 1;
            // s: big(t) back to back, no wait packet; its checking blocks
            // wait for flag >= t (band(t-1) done)
            if (p > 0) CK(hipStreamWaitEvent(c.cs, c.e_int, 0));
            small(c, c.cs);
            hipLaunchKernelGGL(set_flag_kernel, dim3(1), dim3(1), 0, c.cs, c.dflag, (unsigned)(p + 1));
            hipExtLaunchKernelGGL(copy_check_kernel, dim3(4096), dim3(256), 0, c.s, nullptr, c.e_int, 0,
                                  p & 1 ? c.b : c.a, p & 1 ? c.a : c.b, c.n, (const unsigned *)c.dflag, (unsigned)p,
                                  mode == 16 ? 64u : 4096u);
        } else if (mode == 18) {
            if (p > 0) CK(hipStreamWaitEvent(c.cs, c.e_int, 0));
            small(c, c.cs);
            hipLaunchKernelGGL(set_flag_kernel, dim3(1), dim3(1), 0, c.cs, c.dflag, (unsigned)(p + 1));
            hipLaunchKernelGGL(gate_kernel, dim3(1), dim3(64), 0, c.s, (const unsigned *)c.dflag, (unsigned)p);
            big_ev(c, p, c.e_int);
        } else if (mode == 14 || mode == 15) {
            // streams swap roles every pass: big(p) on A = (p even ? s : cs),
            // small(p) on B after big(p-1) by queue order (big(p-1) ran on B),
            // then B waits for big(p) -- a wait armed long before big(p) ends
            // -- and runs big(p + 1).  15: the same with the long small kernel.
            hipStream_t A = (p & 1) ? c.cs : c.s, B = (p & 1) ? c.s : c.cs;
            if (p == 0) big_ev(c, p, c.pool[0], A);  // big(0) on A
            if (mode == 14) small(c, B); else small_long(c, B);
            CK(hipStreamWaitEvent(B, c.pool[p % kPool], 0));  // big(p) done
            big_ev(c, p + 1, c.pool[(p + 1) % kPool], B);   // big(p + 1), on B
        } else if (mode == 3) {
            small(c, c.s);
            big(c, p);
        } else {
            // 4: as 2 with dispatch-carried events; 5: without the main
            // stream's wait; 6: without the second stream's wait
            if (p > 0 && mode != 6) CK(hipStreamWaitEvent(c.cs, c.e_int, 0));
            small_ev(c, c.cs, c.e_band);
            if (p > 0 && mode != 5) CK(hipStreamWaitEvent(c.s, c.e_band, 0));
            big_ev(c, p, c.e_int);
        }
    }
    CK(hipStreamSynchronize(c.s));
    CK(hipStreamSynchronize(c.cs));
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / passes;
}

int main(int argc, char **argv) {
    const int passes = argc > 1 ? atoi(argv[1]) : 200;
    Ctx c;
    c.n = (256u << 20) / 16;
    CK(hipMalloc(&c.a, c.n * 16));
    CK(hipMalloc(&c.b, c.n * 16));
    CK(hipMalloc(&c.sink, 4096));
    CK(hipMalloc(&c.dflag, 256));
    CK(hipMalloc(&c.dcount, 256));
    CK(hipMemset(c.a, 0, c.n * 16));
    int can_wait = 0;
    CK(hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, 0));
    CK(hipExtMallocWithFlags((void **)&c.f_int, 8, hipMallocSignalMemory));
    CK(hipExtMallocWithFlags((void **)&c.f_band, 8, hipMallocSignalMemory));
    printf("{\"can_use_stream_wait_value\": %d}\n", can_wait);
    for (int i = 0; i < kPool; ++i) CK(hipEventCreateWithFlags(&c.pool[i], hipEventDisableTiming));
    int least, greatest;
    CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    const char *evname[3] = {"default", "disable_timing", "disable_timing_sysfence"};
    const unsigned evflags[3] = {hipEventDefault, hipEventDisableTiming,
                                 hipEventDisableTiming | hipEventDisableSystemFence};
    for (int prio = 1; prio < 2; ++prio) {
        for (int ef = 1; ef < 2; ++ef) {
            CK(hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking));
            CK(hipStreamCreateWithPriority(&c.cs, hipStreamNonBlocking, prio ? greatest : least));
            CK(hipEventCreateWithFlags(&c.e_int, evflags[ef]));
            CK(hipEventCreateWithFlags(&c.e_band, evflags[ef]));
            for (int mode = 0; mode < 19; mode += (mode == 2 ? 6 : 1)) {
                run(c, mode, 20);  // warm-up
                const double us = run(c, mode, passes);
                printf("{\"mode\": %d, \"comm_prio\": \"%s\", \"events\": \"%s\", \"us_per_pass\": %.2f}\n", mode,
                       prio ? "high" : "low", evname[ef], us);
                fflush(stdout);
            }
            CK(hipEventDestroy(c.e_int));
            CK(hipEventDestroy(c.e_band));
            CK(hipStreamDestroy(c.s));
            CK(hipStreamDestroy(c.cs));
        }
    }
    return 0;
}
