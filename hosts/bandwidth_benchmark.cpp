// bandwidth_benchmark.cpp -- the point-to-point bandwidth microbenchmark as a
// C++ host on the C ABI (microbenchmarks/host/bandwidth_benchmark.cpp with
// the app kernels of microbenchmarks/kernels/bandwidth_0.cl / bandwidth_1.cl).
//
// Rank 0 streams n doubles (0.1f + i) to the receiving rank on each of two
// ports at once (the reference's two app kernels, ports 0 and 1); the
// receiver checks every element and prints "Result is Ok!" per run; it times
// each run between two barriers and reports the mean, the standard
// deviation, the 99 % confidence interval and the bandwidth as the reference
// does.  -k gives the payload per port in KiB (n = KiB * 1024 / 8 doubles;
// the reference derived n from its 28-byte network packets).  Ranks run as
// host threads of one process (-p <ranks>) or one process per rank
// (--rank/--size/--uid or a launcher's environment; host_rt.h).
//
//   bandwidth_benchmark -k <KiB per port> -r <receiver rank> -i <runs> [-p <ranks>]
//                       [-m bulk|element] [-o <file.dat>]
//
// -m element: the reference's element API, one host thread per port
// (SMI_Open_send_channel_ad / SMI_Push with asynch degree 2048, as
// bandwidth_0.cl; SMI_Open_receive_channel_ad / SMI_Pop); -m bulk (default):
// smi_send / smi_recv of device buffers, one per port.
// Exit codes: 0 every run checked ok, 1 usage, 2 SMI/HIP error, 3 wrong result.
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "host_rt.h"

namespace {

struct Args {
    int kb = 64, recv = 1, runs = 10, ranks = 2;
    bool element = false;
    std::string out;
};

constexpr double kStart = 0.1f;  // bandwidth_0.cl: const double start = 0.1f

// one port of the element-API run (the body of app / app_1)
bool element_port(SMI_Comm comm, bool sender, int peer, int port, int n) {
    bool ok = true;
    if (sender) {
        SMI_Channel ch = SMI_Open_send_channel_ad(n, SMI_DOUBLE, peer, port, comm, 2048);
        for (int i = 0; i < n; ++i) {
            double v = kStart + i;
            SMI_Push(&ch, &v);
        }
    } else {
        SMI_Channel ch = SMI_Open_receive_channel_ad(n, SMI_DOUBLE, 0, port, comm, 2048);
        for (int i = 0; i < n; ++i) {
            double v = 0;
            SMI_Pop(&ch, &v);
            ok &= v == kStart + i;
        }
    }
    return ok;
}

int RankMain(SMI_Comm comm, const Args &a) {
    const int rank = SMI_Comm_rank(comm), ranks = SMI_Comm_size(comm);
    if (a.recv <= 0 || a.recv >= ranks) host::die(1, "receiver rank %d out of range for %d ranks\n", a.recv, ranks);
    const int n = (int)((long)a.kb * 1024 / 8);  // kb < 2^24 (checked in main): n < 2^31
    hipStream_t stream;
    HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    host::Barrier barrier(comm, stream);
    const bool active = rank == 0 || rank == a.recv;
    std::vector<double> seq(n), got(n);
    for (int i = 0; i < n; ++i) seq[i] = kStart + i;
    double *buf[2] = {nullptr, nullptr};
    if (!a.element && active)
        for (auto &b : buf) {
            HIP_OK(hipMalloc(&b, (size_t)n * sizeof(double)));
            if (rank == 0) HIP_OK(hipMemcpy(b, seq.data(), (size_t)n * sizeof(double), hipMemcpyHostToDevice));
        }
    std::vector<double> times_us;
    bool all_ok = true;
    for (int it = 0; it < a.runs; ++it) {
        if (!a.element && rank == a.recv)
            for (auto &b : buf) HIP_OK(hipMemsetAsync(b, 0, (size_t)n * sizeof(double), stream));
        barrier.wait();
        bool ok = true;
        const auto t0 = std::chrono::steady_clock::now();
        if (active) {
            if (a.element) {
                // the two app kernels run concurrently: one host thread per port
                bool ok1 = true;
                std::thread port1([&] { ok1 = element_port(comm, rank == 0, a.recv, 1, n); });
                ok = element_port(comm, rank == 0, a.recv, 0, n);
                port1.join();
                ok &= ok1;
            } else {
                for (int p = 0; p < 2; ++p) {
                    if (rank == 0) SMI_OK(smi_send(comm, buf[p], n, SMI_DOUBLE, a.recv, p, (SMI_Stream)stream));
                    else SMI_OK(smi_recv(comm, buf[p], n, SMI_DOUBLE, 0, p, (SMI_Stream)stream));
                }
                SMI_OK(smi_stream_synchronize((SMI_Stream)stream));
            }
        }
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        barrier.wait();
        if (rank == a.recv) {
            if (!a.element)
                for (auto &b : buf) {
                    HIP_OK(hipMemcpy(got.data(), b, (size_t)n * sizeof(double), hipMemcpyDeviceToHost));
                    for (int i = 0; i < n; ++i) ok &= got[i] == seq[i];
                }
            times_us.push_back(us);
            std::printf("%s\n", ok ? "Result is Ok!" : "Error!!!!");
            std::fflush(stdout);
            all_ok &= ok;
        }
    }
    if (rank == a.recv)
        host::report("Bandwidth", a.element ? "element API" : "bulk", ranks, 2L * n, sizeof(double), times_us, a.out);
    for (auto &b : buf)
        if (b) HIP_OK(hipFree(b));
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
    while ((c = getopt(argc, argv, "k:r:i:p:m:o:")) != -1) {
        switch (c) {
        case 'k': a.kb = std::atoi(optarg); break;
        case 'r': a.recv = std::atoi(optarg); break;
        case 'i': a.runs = std::atoi(optarg); break;
        case 'p': a.ranks = std::atoi(optarg); break;
        case 'm': a.element = std::string(optarg) == "element"; break;
        case 'o': a.out = optarg; break;
        default:
            std::fprintf(stderr,
                         "usage: %s -k <KiB per port> -r <receiver rank> -i <runs> [-p <ranks>] [-m bulk|element]"
                         " [-o file] [--rank R --size N --uid FILE]\n",
                         argv[0]);
            return 1;
        }
    }
    const int ranks = launch.process() ? launch.size : a.ranks;
    if (a.kb <= 0 || a.kb >= (1 << 24) || a.runs <= 0 || ranks < 2 || a.recv <= 0 || a.recv >= ranks) {
        std::fprintf(stderr, "bad arguments (1 <= KiB < 2^24, at least 2 ranks, receiver rank 1 .. ranks - 1)\n");
        return 1;
    }
    return host::run_ranks(launch, a.ranks, [&](SMI_Comm comm) { return RankMain(comm, a); });
}
