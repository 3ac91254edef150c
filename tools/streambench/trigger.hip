// trigger.hip -- can a running kernel release work queued on another stream?
// A long "producer" kernel on stream s bumps a counter early (each block,
// after a release fence, one atomic add); stream cs waits for the counter with
// hipStreamWaitValue32 and then runs a tiny "consumer" kernel.  Both record
// s_memrealtime (100 MHz) stamps: if the consumer starts long before the
// producer ends, a kernel can trigger another stream's work mid-flight.
// Counter memory: hipMallocSignalMemory (argv[1] = 0) or fine-grained device
// memory (argv[1] = 1).  JSON line per trial.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                                 \
        }                                                                            \
    } while (0)

__global__ void producer(unsigned *counter, unsigned long long *stamps, int iters, float *sink) {
    if (threadIdx.x == 0 && blockIdx.x == 0) stamps[0] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    float v = threadIdx.x;
    for (int i = 0; i < iters; ++i) v = v * 1.0000001f + 0.5f;
    if (v == -1.0f) sink[threadIdx.x] = v;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&stamps[1], __builtin_amdgcn_s_memrealtime());
}

__global__ void consumer(unsigned long long *stamps) {
    if (threadIdx.x == 0) stamps[2] = __builtin_amdgcn_s_memrealtime();
}

int main(int argc, char **argv) {
    const int fine = argc > 1 ? atoi(argv[1]) : 0;
    unsigned *counter;
    if (fine) CK(hipExtMallocWithFlags((void **)&counter, 64, hipDeviceMallocFinegrained));
    else CK(hipExtMallocWithFlags((void **)&counter, 8, hipMallocSignalMemory));
    unsigned long long *stamps;
    CK(hipHostMalloc((void **)&stamps, 64));
    float *sink;
    CK(hipMalloc(&sink, 4096));
    hipStream_t s, cs;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    const int blocks = 64;
    CK(hipStreamWriteValue32(s, counter, 0u, 0));
    CK(hipStreamSynchronize(s));
    for (int trial = 0; trial < 6; ++trial) {
        stamps[0] = stamps[1] = stamps[2] = 0;
        const unsigned target = (unsigned)blocks * (trial + 1);
        CK(hipStreamWaitValue32(cs, counter, target, hipStreamWaitValueGte, 0xFFFFFFFFu));
        hipLaunchKernelGGL(consumer, dim3(1), dim3(64), 0, cs, stamps);
        hipLaunchKernelGGL(producer, dim3(blocks), dim3(256), 0, s, counter, stamps, 200000, sink);
        CK(hipStreamSynchronize(s));
        CK(hipStreamSynchronize(cs));
        const double t_prod = (stamps[1] - stamps[0]) / 100.0, t_cons = ((long long)stamps[2] - (long long)stamps[0]) / 100.0;
        printf("{\"memory\": \"%s\", \"trial\": %d, \"producer_us\": %.1f, \"consumer_start_us\": %.1f}\n",
               fine ? "finegrained" : "signal", trial, t_prod, t_cons);
        fflush(stdout);
    }
    return 0;
}
