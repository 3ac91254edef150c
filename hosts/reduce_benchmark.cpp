// reduce_benchmark.cpp -- the SMI_Reduce microbenchmark as a C++ host on the
// C ABI (microbenchmarks/host/reduce_benchmark.cpp:19-158 with the app kernel
// of microbenchmarks/kernels/reduce.cl:9-27).
//
// Every rank contributes rank + 1 for each of n elements (fp32 add); the root
// checks every element against n_ranks (n_ranks + 1) / 2 and reports the
// mean run time, its standard deviation and the 99 % confidence interval
// (2.58 sigma / sqrt(runs)) like the reference harness (:120-155).  Ranks are
// host threads of an in-process group (smi_local_group_create +
// smi_init_local) standing in for the reference's MPI processes; a barrier
// brackets every run as MPI_Barrier does (:99-105).
//
//   reduce_benchmark -n <elements> -r <root> -i <runs> -p <ranks>
//                    [-m bulk|element] [-o <file.dat>] [-d <device>]
//
// -m element runs the reference's own per-element API (SMI_Open_reduce_channel
// + one SMI_Reduce per element with host values, as reduce.cl does);
// -m bulk (default) one smi_reduce over the ranks' device buffers.
// Exit codes: 0 every run checked ok, 1 usage, 2 SMI/HIP error, 3 wrong result.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include <smi.h>

namespace {

struct Args {
    int n = 1024, root = 0, runs = 10, ranks = 4, device = 0;
    bool element = false;
    std::string out;
};

pthread_barrier_t g_barrier;
std::vector<double> g_times_us;  // root only
std::atomic<int> g_bad{0};

#define SMI_OK(call)                                                                    \
    do {                                                                                \
        const int rc_ = (call);                                                         \
        if (rc_ != SMI_SUCCESS) {                                                       \
            std::fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, smi_last_error()); \
            return 2;                                                                   \
        }                                                                               \
    } while (0)
#define HIP_OK(call)                                                                    \
    do {                                                                                \
        const hipError_t e_ = (call);                                                   \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s failed: %s\n", #call, hipGetErrorString(e_));     \
            return 2;                                                                   \
        }                                                                               \
    } while (0)

int RunRank(int group, int rank, const Args &a) {
    SMI_Comm comm;
    SMI_OK(smi_init_local(group, rank, a.device, &comm));
    const int my_rank = SMI_Comm_rank(comm), num_ranks = SMI_Comm_size(comm);
    const float expected = (float)(num_ranks * (num_ranks + 1)) / 2;  // reduce.cl:13
    float *snd = nullptr, *rcv = nullptr;
    hipStream_t stream;
    std::vector<float> host(a.n, (float)(my_rank + 1)), res(a.n, 0.0f);
    if (!a.element) {
        HIP_OK(hipMalloc(&snd, a.n * sizeof(float)));
        HIP_OK(hipMalloc(&rcv, a.n * sizeof(float)));
        HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        HIP_OK(hipMemcpy(snd, host.data(), a.n * sizeof(float), hipMemcpyHostToDevice));
    }
    for (int it = 0; it < a.runs; ++it) {
        pthread_barrier_wait(&g_barrier);  // wait for the other ranks (:99)
        bool ok = true;
        const auto t0 = std::chrono::steady_clock::now();
        if (a.element) {
            // reduce.cl:15-24: open the channel, one SMI_Reduce per element
            SMI_RChannel chan = SMI_Open_reduce_channel(a.n, SMI_FLOAT, SMI_ADD, 0, a.root, comm);
            for (int i = 0; i < a.n; ++i) {
                float to_comm = (float)(my_rank + 1), to_rcv = 0.0f;
                SMI_Reduce(&chan, &to_comm, &to_rcv);
                if (my_rank == a.root) ok &= to_rcv == expected;
            }
        } else {
            SMI_OK(smi_reduce(comm, snd, rcv, a.n, SMI_FLOAT, SMI_ADD, a.root, 0, (SMI_Stream)stream));
            SMI_OK(smi_stream_synchronize((SMI_Stream)stream));
        }
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        pthread_barrier_wait(&g_barrier);  // (:105)
        if (my_rank == a.root) {
            if (!a.element) {
                HIP_OK(hipMemcpy(res.data(), rcv, a.n * sizeof(float), hipMemcpyDeviceToHost));
                ok = std::all_of(res.begin(), res.end(), [&](float v) { return v == expected; });
            }
            g_times_us.push_back(us);
            std::printf("Rank: %d %s\n", my_rank, ok ? "Result is Ok!" : "Error!!!!");
            if (!ok) g_bad = 1;
        }
    }
    if (!a.element) {
        HIP_OK(hipStreamDestroy(stream));
        HIP_OK(hipFree(snd));
        HIP_OK(hipFree(rcv));
    }
    SMI_OK(smi_finalize(comm));
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    Args a;
    int c;
    while ((c = getopt(argc, argv, "n:r:i:p:m:o:d:")) != -1) {
        switch (c) {
        case 'n': a.n = std::atoi(optarg); break;
        case 'r': a.root = std::atoi(optarg); break;
        case 'i': a.runs = std::atoi(optarg); break;
        case 'p': a.ranks = std::atoi(optarg); break;
        case 'm': a.element = std::string(optarg) == "element"; break;
        case 'o': a.out = optarg; break;
        case 'd': a.device = std::atoi(optarg); break;
        default:
            std::fprintf(stderr, "usage: %s -n <length> -r <root> -i <runs> -p <ranks> [-m bulk|element] [-o file]\n",
                         argv[0]);
            return 1;
        }
    }
    if (a.n <= 0 || a.runs <= 0 || a.ranks <= 0 || a.root < 0 || a.root >= a.ranks) {
        std::fprintf(stderr, "bad arguments\n");
        return 1;
    }
    int group = -1;
    SMI_OK(smi_local_group_create(a.ranks, &group));
    pthread_barrier_init(&g_barrier, nullptr, a.ranks);
    std::vector<int> rcs(a.ranks, 0);
    std::vector<std::thread> th;
    for (int r = 0; r < a.ranks; ++r) th.emplace_back([&, r] { rcs[r] = RunRank(group, r, a); });
    for (auto &t : th) t.join();
    pthread_barrier_destroy(&g_barrier);
    for (int rc : rcs)
        if (rc) return rc;

    // statistics as reduce_benchmark.cpp:120-136
    double mean = 0;
    for (double t : g_times_us) mean += t;
    mean /= a.runs;
    double stddev = 0;
    for (double t : g_times_us) stddev += (t - mean) * (t - mean);
    stddev = std::sqrt(stddev / a.runs);
    const double ci99 = 2.58 * stddev / std::sqrt((double)a.runs);
    const double kb = (double)a.n * sizeof(float) / 1024.0;
    const double gbit = (kb * 8 / (mean / 1e6)) / (1024 * 1024);
    std::printf("-------------------------------------------------------------------\n");
    std::printf("Computation time (usec): %g (sttdev: %g)\n", mean, stddev);
    std::printf("Conf interval 99: %g\n", ci99);
    std::printf("Conf interval 99 within %g%% from mean\n", ci99 / mean * 100);
    std::printf("Sent (KB): %g\n", kb);
    std::printf("Average bandwidth (Gbit/s): %g\n", gbit);
    std::printf("-------------------------------------------------------------------\n");
    if (!a.out.empty()) {
        FILE *f = std::fopen(a.out.c_str(), "w");
        if (!f) return 2;
        std::fprintf(f, "#SMI Reduce (%s), executed with %d ranks, streaming: %d elements\n",
                     a.element ? "element API" : "bulk", a.ranks, a.n);
        std::fprintf(f, "#Sent (KB) = %g, Runs = %d\n", kb, a.runs);
        std::fprintf(f, "#Average Computation time (usecs): %g\n", mean);
        std::fprintf(f, "#Standard deviation (usecs): %g\n", stddev);
        std::fprintf(f, "#Confidence interval 99%%: +- %g\n", ci99);
        std::fprintf(f, "#Average bandwidth (Gbit/s): %g\n", gbit);
        std::fprintf(f, "#Execution times (usecs):\n");
        for (double t : g_times_us) std::fprintf(f, "%g\n", t);
        std::fclose(f);
    }
    return g_bad ? 3 : 0;
}
