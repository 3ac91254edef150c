// broadcast_benchmark.cpp -- the SMI_Bcast microbenchmark as a C++ host on
// the C ABI (microbenchmarks/host/broadcast_benchmark.cpp:20-166 with the app
// kernel of microbenchmarks/kernels/broadcast.cl:9-22).
//
// The root broadcasts the sequence 0, 1, ..., n-1 as floats; every other rank
// checks that element i arrived as i and prints "Result is Ok!" per run
// (:114-122).  The root times each run between two barriers and reports the
// mean, the standard deviation, the 99 % confidence interval and the
// bandwidth like the reference harness (:126-163).  Ranks run as host
// threads of one process (-p <ranks>) or one process per rank
// (--rank/--size/--uid, smi_init over RCCL; host_rt.h).
//
//   broadcast_benchmark -n <elements> -r <root> -i <runs> [-p <ranks>]
//                       [-m bulk|element] [-o <file.dat>]
//                       [--device D] [--rank R --size N --uid FILE]
//
// -m element: the reference's own per-element API (SMI_Open_bcast_channel +
// one SMI_Bcast per element with host values, as broadcast.cl does);
// -m bulk (default): one smi_bcast of the whole device buffer.
// Exit codes: 0 every run checked ok, 1 usage, 2 SMI/HIP error, 3 wrong result.
#include <unistd.h>

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
    hipStream_t stream;
    HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    host::Barrier barrier(comm, stream);
    // the root's buffer holds the sequence broadcast.cl sends (to_comm = i)
    std::vector<float> seq(a.n), got(a.n);
    for (int i = 0; i < a.n; ++i) seq[i] = (float)i;
    float *buf = nullptr;
    if (!a.element) HIP_OK(hipMalloc(&buf, a.n * sizeof(float)));
    std::vector<double> times_us;
    bool all_ok = true;
    for (int it = 0; it < a.runs; ++it) {
        if (!a.element) {
            // the root sends the sequence; the others start from a poisoned
            // buffer so that a stale result cannot pass
            if (my_rank == a.root) HIP_OK(hipMemcpy(buf, seq.data(), a.n * sizeof(float), hipMemcpyHostToDevice));
            else HIP_OK(hipMemsetAsync(buf, 0xff, a.n * sizeof(float), stream));
        }
        barrier.wait();  // (:106)
        char check = 1;
        const auto t0 = std::chrono::steady_clock::now();
        if (a.element) {
            // broadcast.cl:12-19
            SMI_BChannel chan = SMI_Open_bcast_channel(a.n, SMI_FLOAT, 0, a.root, comm);
            for (int i = 0; i < a.n; ++i) {
                float to_comm = (float)i;
                if (my_rank != a.root) to_comm = -1.0f;
                SMI_Bcast(&chan, &to_comm);
                check &= to_comm == (float)i;
            }
        } else {
            SMI_OK(smi_bcast(comm, buf, a.n, SMI_FLOAT, a.root, 0, (SMI_Stream)stream));
            SMI_OK(smi_stream_synchronize((SMI_Stream)stream));
        }
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        barrier.wait();  // (:110)
        if (my_rank == a.root) times_us.push_back(us);
        if (my_rank != a.root) {
            if (!a.element) {
                HIP_OK(hipMemcpy(got.data(), buf, a.n * sizeof(float), hipMemcpyDeviceToHost));
                for (int i = 0; i < a.n; ++i) check &= got[i] == (float)i;
            }
            std::printf("Rank: %d %s\n", my_rank, check ? "Result is Ok!" : "Error!!!!");
            all_ok &= check != 0;
        }
    }
    if (my_rank == a.root)
        host::report("Broadcast", a.element ? "element API" : "bulk", num_ranks, a.n, sizeof(float), times_us, a.out);
    if (buf) HIP_OK(hipFree(buf));
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
    if (a.n <= 0 || a.runs <= 0 || ranks <= 1 || a.root < 0 || a.root >= ranks) {
        std::fprintf(stderr, "bad arguments (at least 2 ranks)\n");
        return 1;
    }
    std::printf("Performing broadcast with  %d elements, root: %d\n", a.n, a.root);
    return host::run_ranks(launch, a.ranks, [&](SMI_Comm comm) { return RankMain(comm, a); });
}
