// latency_benchmark.cpp -- the ping-pong latency microbenchmark as a C++ host
// on the C ABI (microbenchmarks/host/latency_benchmark.cpp with the app
// kernels of microbenchmarks/kernels/latency_0.cl / latency_1.cl).
//
// Rank 0 and the receiving rank exchange one int n times: rank 0 pushes,
// pops and adds one, the receiver pops, adds one and pushes it back, each
// message on a fresh channel of one element (latency_0.cl:21-34,
// latency_1.cl:20-33), so the value ends at 2n.  Rank 0 checks that value
// every run (and, in element mode, every increment on the way), times each
// run between two barriers and reports the mean run time, its standard
// deviation and the 99 % confidence interval as the reference does
// (:150-170), plus the one-way latency (run time / 2n).  Ranks run as host
// threads of one process (-p <ranks>) or one process per rank
// (--rank/--size/--uid or a launcher's environment; host_rt.h).
//
//   latency_benchmark -n <round trips> -r <receiver rank> -i <runs> [-p <ranks>]
//                     [-m element|bulk] [-o <file.dat>]
//
// -m element (default): the reference's element API from the host
// (SMI_Open_send_channel / SMI_Push, SMI_Open_receive_channel / SMI_Pop):
// every message goes host -> device -> peer -> host.  -m bulk: the int stays
// in device memory and the whole exchange is one stream-ordered chain per
// rank -- smi_send / smi_recv and a one-lane increment kernel, as the
// reference's pop / +1 / push inside the kernel -- with no host
// synchronisation until the run ends: the round trip the GPU itself sees.
// Exit codes: 0 every run checked ok, 1 usage, 2 SMI/HIP error, 3 wrong result.
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "host_rt.h"

namespace {

__global__ void bump(int *v) { *v += 1; }  // to_send++ (latency_0.cl:30, latency_1.cl:29)

struct Args {
    int n = 1000, recv = 1, runs = 10, ranks = 2;
    bool bulk = false;
    std::string out;
};

int RankMain(SMI_Comm comm, const Args &a) {
    const int rank = SMI_Comm_rank(comm), ranks = SMI_Comm_size(comm);
    if (a.recv <= 0 || a.recv >= ranks) host::die(1, "receiver rank %d out of range for %d ranks\n", a.recv, ranks);
    hipStream_t stream;
    HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    host::Barrier barrier(comm, stream);
    int *dv = nullptr;
    if (a.bulk) HIP_OK(hipMalloc(&dv, sizeof(int)));
    auto send = [&](int v, int peer) {
        SMI_Channel ch = SMI_Open_send_channel(1, SMI_INT, peer, 0, comm);
        SMI_Push(&ch, &v);
        if (ch.status != SMI_SUCCESS) host::die(2, "SMI_Push: %s\n", smi_last_error());
    };
    auto recv = [&](int peer) {
        int v = -1;
        SMI_Channel ch = SMI_Open_receive_channel(1, SMI_INT, peer, 0, comm);
        SMI_Pop(&ch, &v);
        if (ch.status != SMI_SUCCESS) host::die(2, "SMI_Pop: %s\n", smi_last_error());
        return v;
    };
    auto inc = [&] {
        hipLaunchKernelGGL(bump, dim3(1), dim3(1), 0, stream, dv);
        HIP_OK(hipGetLastError());
    };
    const SMI_Stream ss = (SMI_Stream)stream;
    std::vector<double> times_us;
    bool all_ok = true;
    for (int it = 0; it < a.runs; ++it) {
        if (a.bulk && rank == 0) {
            HIP_OK(hipMemsetAsync(dv, 0, sizeof(int), stream));
            HIP_OK(hipStreamSynchronize(stream));
        }
        barrier.wait();
        bool ok = true;
        int v = 0;
        const auto t0 = std::chrono::steady_clock::now();
        if (a.bulk) {
            if (rank == 0) {
                for (int i = 0; i < a.n; ++i) {  // latency_0.cl: push, pop, +1
                    SMI_OK(smi_send(comm, dv, 1, SMI_INT, a.recv, 0, ss));
                    SMI_OK(smi_recv(comm, dv, 1, SMI_INT, a.recv, 0, ss));
                    inc();
                }
            } else if (rank == a.recv) {
                for (int i = 0; i < a.n; ++i) {  // latency_1.cl: pop, +1, push
                    SMI_OK(smi_recv(comm, dv, 1, SMI_INT, 0, 0, ss));
                    inc();
                    SMI_OK(smi_send(comm, dv, 1, SMI_INT, 0, 0, ss));
                }
            }
            SMI_OK(smi_stream_synchronize(ss));
        } else if (rank == 0) {
            for (int i = 0; i < a.n; ++i) {  // latency_0.cl: push, pop, +1
                send(v, a.recv);
                const int back = recv(a.recv);
                ok &= back == v + 1;
                v = back + 1;
            }
        } else if (rank == a.recv) {
            for (int i = 0; i < a.n; ++i) send(recv(0) + 1, 0);  // latency_1.cl: pop, +1, push
        }
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        if (a.bulk && rank == 0) HIP_OK(hipMemcpy(&v, dv, sizeof(int), hipMemcpyDeviceToHost));
        if (rank == 0) ok &= v == 2 * a.n;
        barrier.wait();
        if (rank == 0) {
            times_us.push_back(us);
            std::printf("%s\n", ok ? "Result is Ok!" : "Error!!!!");
            all_ok &= ok;
        }
    }
    if (rank == 0) {
        const host::Stats st = host::stats_of(times_us);
        std::printf("-------------------------------------------------------------------\n");
        std::printf("Average Latency (usec): %g (sttdev: %g)\n", st.mean, st.stddev);
        std::printf("Conf interval 99: %g\n", st.ci99);
        std::printf("Conf interval 99 within %g%% from mean\n", st.ci99 / st.mean * 100);
        std::printf("One-way latency (usec): %g (run time / 2n)\n", st.mean / (2.0 * a.n));
        std::printf("-------------------------------------------------------------------\n");
        if (!a.out.empty()) {
            FILE *f = std::fopen(a.out.c_str(), "w");
            if (!f) host::die(2, "cannot write %s\n", a.out.c_str());
            std::fprintf(f, "#SMI latency (%s), %d round trips, %d ranks\n", a.bulk ? "bulk" : "element API", a.n, ranks);
            std::fprintf(f, "#Average Latency (usecs): %g\n", st.mean);
            std::fprintf(f, "#Standard deviation (usecs): %g\n", st.stddev);
            std::fprintf(f, "#Confidence interval 99%%: +- %g\n", st.ci99);
            std::fprintf(f, "#Execution times (usecs):\n");
            for (double t : times_us) std::fprintf(f, "%g\n", t);
            std::fclose(f);
        }
    }
    if (dv) HIP_OK(hipFree(dv));
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
        case 'r': a.recv = std::atoi(optarg); break;
        case 'i': a.runs = std::atoi(optarg); break;
        case 'p': a.ranks = std::atoi(optarg); break;
        case 'm': a.bulk = std::string(optarg) == "bulk"; break;
        case 'o': a.out = optarg; break;
        default:
            std::fprintf(stderr,
                         "usage: %s -n <round trips> -r <receiver rank> -i <runs> [-p <ranks>] [-m element|bulk]"
                         " [-o file] [--rank R --size N --uid FILE]\n",
                         argv[0]);
            return 1;
        }
    }
    const int ranks = launch.process() ? launch.size : a.ranks;
    if (a.n <= 0 || a.runs <= 0 || ranks < 2 || a.recv <= 0 || a.recv >= ranks) {
        std::fprintf(stderr, "bad arguments (at least 2 ranks, receiver rank 1 .. ranks - 1)\n");
        return 1;
    }
    return host::run_ranks(launch, a.ranks, [&](SMI_Comm comm) { return RankMain(comm, a); });
}
