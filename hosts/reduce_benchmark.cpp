// reduce_benchmark.cpp -- the SMI_Reduce microbenchmark as a C++ host on the
// C ABI (microbenchmarks/host/reduce_benchmark.cpp:19-158 with the app kernel
// of microbenchmarks/kernels/reduce.cl:9-27).
//
// Every rank contributes rank + 1 for each of n elements (fp32 add); the root
// checks every element against n_ranks (n_ranks + 1) / 2 and reports the
// mean run time, its standard deviation and the 99 % confidence interval
// (2.58 sigma / sqrt(runs)) like the reference harness (:120-155).  Ranks run
// either as host threads of one process (-p <ranks>) or one process per rank
// (--rank/--size/--uid, smi_init over RCCL; host_rt.h); a barrier on the
// communicator brackets every run as MPI_Barrier does (:99-105).
//
//   reduce_benchmark -n <elements> -r <root> -i <runs> [-p <ranks>]
//                    [-m bulk|element] [-o <file.dat>]
//                    [--device D] [--rank R --size N --uid FILE]
//
// -m element runs the reference's own per-element API (SMI_Open_reduce_channel
// + one SMI_Reduce per element with host values, as reduce.cl does);
// -m bulk (default) one smi_reduce over the ranks' device buffers.
// Exit codes: 0 every run checked ok, 1 usage, 2 SMI/HIP error, 3 wrong result.
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "host_rt.h"

namespace {

struct Args {
    int n = 1024, root = 0, runs = 10, ranks = 4;
    bool element = false;
    std::string out;
};

int RankMain(SMI_Comm comm, const Args &a) {
    const int my_rank = SMI_Comm_rank(comm), num_ranks = SMI_Comm_size(comm);
    if (a.root >= num_ranks) host::die(1, "root %d out of range for %d ranks\n", a.root, num_ranks);
    const float expected = (float)(num_ranks * (num_ranks + 1)) / 2;  // reduce.cl:13
    hipStream_t stream;
    HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    host::Barrier barrier(comm, stream);
    float *snd = nullptr, *rcv = nullptr;
    std::vector<float> host_v(a.n, (float)(my_rank + 1)), res(a.n, 0.0f);
    if (!a.element) {
        HIP_OK(hipMalloc(&snd, a.n * sizeof(float)));
        HIP_OK(hipMalloc(&rcv, a.n * sizeof(float)));
        HIP_OK(hipMemcpy(snd, host_v.data(), a.n * sizeof(float), hipMemcpyHostToDevice));
    }
    std::vector<double> times_us;
    bool all_ok = true;
    for (int it = 0; it < a.runs; ++it) {
        barrier.wait();  // wait for the other ranks (:99)
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
        barrier.wait();  // (:105)
        if (my_rank == a.root) {
            if (!a.element) {
                HIP_OK(hipMemcpy(res.data(), rcv, a.n * sizeof(float), hipMemcpyDeviceToHost));
                ok = std::all_of(res.begin(), res.end(), [&](float v) { return v == expected; });
            }
            times_us.push_back(us);
            std::printf("Rank: %d %s\n", my_rank, ok ? "Result is Ok!" : "Error!!!!");
            all_ok &= ok;
        }
    }
    if (my_rank == a.root)
        host::report("Reduce", a.element ? "element API" : "bulk", num_ranks, a.n, sizeof(float), times_us, a.out);
    if (!a.element) {
        HIP_OK(hipFree(snd));
        HIP_OK(hipFree(rcv));
    }
    HIP_OK(hipStreamDestroy(stream));
    return all_ok ? 0 : 3;
}

}  // namespace

int main(int argc, char **argv) {
    host::Launch launch;
    if (!host::parse_launch(argc, argv, &launch)) {
        std::fprintf(stderr, "bad --rank/--size/--uid\n");
        return 1;
    }
    Args a;
    int c;
    while ((c = getopt(argc, argv, "n:r:i:p:m:o:")) != -1) {
        switch (c) {
        case 'n': a.n = std::atoi(optarg); break;
        case 'r': a.root = std::atoi(optarg); break;
        case 'i': a.runs = std::atoi(optarg); break;
        case 'p': a.ranks = std::atoi(optarg); break;
        case 'm': a.element = std::string(optarg) == "element"; break;
        case 'o': a.out = optarg; break;
        default:
            std::fprintf(stderr,
                         "usage: %s -n <length> -r <root> -i <runs> [-p <ranks>] [-m bulk|element] [-o file]"
                         " [--rank R --size N --uid FILE]\n",
                         argv[0]);
            return 1;
        }
    }
    const int ranks = launch.process() ? launch.size : a.ranks;
    if (a.n <= 0 || a.runs <= 0 || ranks <= 0 || a.root < 0 || a.root >= ranks) {
        std::fprintf(stderr, "bad arguments\n");
        return 1;
    }
    return host::run_ranks(launch, a.ranks, [&](SMI_Comm comm) { return RankMain(comm, a); });
}
