// kmeans_smi_host.cpp -- a C++ host of kmeans_smi on the C ABI
// (examples/host/kmeans_smi.cpp:41-311 with the kernels of
// examples/kernels/kmeans_smi.cl).
//
// Rank 0 generates the reference host's input with the reference's own
// generator: libstdc++'s std::default_random_engine seeded with 5, cluster
// means uniform in [-5, 5), point i drawn around mean i % K from
// std::normal_distribution, and K initial centroids copied from input points
// picked by uniform_int_distribution(0, num_points) (:96-147).  That
// distribution is inclusive, so the reference can copy a centroid from one
// past the end of its input.  This host stops with exit code 1 in that case
// instead of reading past the end.  The centroids go to every rank
// (smi_bcast, the reference's MPI_Bcast :164), the points in equal
// contiguous shares (smi_scatter, MPI_Scatter :165-166).  Then the whole
// program -- ComputeDistance, ComputeMeans, SMI_Reduce to rank 0, SMI_Bcast,
// divide -- runs `iterations` times in one smi_kmeans call per rank, timed
// between two barriers like the reference's kernels (:255-284).  Rank 0
// prints the final centroids (:296-306); -o writes them as raw float32 for
// bitwise checks.  Ranks run as host threads of one process (-p <ranks>) or
// one process per rank (--rank/--size/--uid or a launcher's environment;
// host_rt.h).
//
//   kmeans_smi_host [emulator|hardware] <num_points> <iterations> [-k clusters]
//                   [-d dims] [-w width] [-p ranks] [-o centroids.f32] [-q]
//
// The leading mode word of the reference's command line is accepted and
// ignored.  Defaults are the reference build's: 8 clusters, 64 dimensions,
// vector width 16 (examples/CMakeLists.txt:9-11, kmeans.h.in).  -q skips
// the printing of means and centroids.
// Exit codes: 0 done, 1 usage or the generator's out-of-range pick,
// 2 SMI/HIP error.
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <type_traits>
#include <vector>

#include "host_rt.h"

namespace {

static_assert(std::is_same<std::default_random_engine, std::minstd_rand0>::value,
              "the reference's input comes from libstdc++'s default_random_engine (minstd_rand0)");

struct Args {
    int num_points = 0, iterations = 0, clusters = 8, dims = 64, width = 16, ranks = 8;
    bool quiet = false;
    std::string out;
};

void print_rows(const char *title, const std::vector<float> &v, int rows, int dims) {
    std::printf("[0] %s\n", title);
    for (int k = 0; k < rows; ++k) {
        std::printf("  {%g", v[(size_t)k * dims]);
        for (int d = 1; d < dims; ++d) std::printf(", %g", v[(size_t)k * dims + d]);
        std::printf("}\n");
    }
}

// kmeans_smi.cpp:96-147 on rank 0.  Returns false when the reference would
// copy a centroid from one past the end of its input.
bool generate(const Args &a, std::vector<float> *input, std::vector<float> *centroids) {
    const int K = a.clusters, D = a.dims;
    std::default_random_engine rng(5);
    std::uniform_real_distribution<float> dist_means(-5, 5);
    std::vector<float> means((size_t)K * D);
    for (int k = 0; k < K; ++k)
        for (int d = 0; d < D; ++d) means[(size_t)k * D + d] = dist_means(rng);
    if (!a.quiet) print_rows("Means used to generate data:", means, K, D);
    std::normal_distribution<float> normal_dist;
    input->assign((size_t)a.num_points * D, 0.0f);
    for (int i = 0; i < a.num_points; ++i) {
        const int k = i % K;
        for (int d = 0; d < D; ++d) (*input)[(size_t)i * D + d] = normal_dist(rng) + means[(size_t)k * D + d];
    }
    std::uniform_int_distribution<size_t> index_dist(0, a.num_points);
    centroids->assign((size_t)K * D, 0.0f);
    for (int k = 0; k < K; ++k) {
        const size_t i = index_dist(rng);
        if (i >= (size_t)a.num_points) {
            std::fprintf(stderr, "initial centroid %d would be input point %zu of %d: the reference reads past "
                                 "the end of its input here; choose another num_points\n",
                         k, i, a.num_points);
            return false;
        }
        for (int d = 0; d < D; ++d) (*centroids)[(size_t)k * D + d] = (*input)[i * D + d];
    }
    if (!a.quiet) print_rows("Initial centroids:", *centroids, K, D);
    return true;
}

int RankMain(SMI_Comm comm, const Args &a) {
    const int rank = SMI_Comm_rank(comm), ranks = SMI_Comm_size(comm);
    const int K = a.clusters, D = a.dims;
    if (a.num_points % ranks != 0) host::die(1, "Number of points must be divisible by number of ranks.\n");
    const int per_rank = a.num_points / ranks;
    hipStream_t stream;
    HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    const SMI_Stream ss = (SMI_Stream)stream;
    host::Barrier barrier(comm, stream);

    std::vector<float> input, centroids((size_t)K * D);
    float *d_input = nullptr, *d_points = nullptr, *d_centroids = nullptr;
    HIP_OK(hipMalloc(&d_points, (size_t)per_rank * D * sizeof(float)));
    HIP_OK(hipMalloc(&d_centroids, (size_t)K * D * sizeof(float)));
    if (rank == 0) {
        if (!generate(a, &input, &centroids)) host::die(1, "");
        HIP_OK(hipMalloc(&d_input, input.size() * sizeof(float)));
        HIP_OK(hipMemcpy(d_input, input.data(), input.size() * sizeof(float), hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(d_centroids, centroids.data(), centroids.size() * sizeof(float), hipMemcpyHostToDevice));
    }
    // distribute: the centroids to every rank, the points in equal shares
    SMI_OK(smi_bcast(comm, d_centroids, (size_t)K * D, SMI_FLOAT, 0, 0, ss));
    SMI_OK(smi_scatter(comm, d_input, d_points, (size_t)per_rank * D, SMI_FLOAT, 0, 0, ss));
    SMI_OK(smi_stream_synchronize(ss));

    barrier.wait();
    const auto t0 = std::chrono::steady_clock::now();
    SMI_OK(smi_kmeans(comm, d_points, per_rank, D, K, a.width, d_centroids, a.iterations, ss));
    SMI_OK(smi_stream_synchronize(ss));
    const double elapsed = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("[%d] Finished in %g seconds.\n", rank, elapsed);
    std::fflush(stdout);
    barrier.wait();

    HIP_OK(hipMemcpy(centroids.data(), d_centroids, centroids.size() * sizeof(float), hipMemcpyDeviceToHost));
    if (rank == 0) {
        if (!a.quiet) print_rows("Final centroids:", centroids, K, D);
        if (!a.out.empty()) {
            FILE *f = std::fopen(a.out.c_str(), "wb");
            if (!f || std::fwrite(centroids.data(), sizeof(float), centroids.size(), f) != centroids.size())
                host::die(2, "cannot write %s\n", a.out.c_str());
            std::fclose(f);
        }
    }
    if (d_input) HIP_OK(hipFree(d_input));
    HIP_OK(hipFree(d_points));
    HIP_OK(hipFree(d_centroids));
    HIP_OK(hipStreamDestroy(stream));
    return 0;
}

int usage(const char *prog) {
    std::fprintf(stderr,
                 "Usage: %s [emulator|hardware] <num_points> <iterations> [-k clusters] [-d dims] [-w width]"
                 " [-p ranks] [-o centroids.f32] [-q] [--rank R --size N --uid FILE]\n",
                 prog);
    return 1;
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
    while ((c = getopt(argc, argv, "k:d:w:p:o:q")) != -1) {  // GNU getopt: positionals move to the end
        switch (c) {
        case 'k': a.clusters = std::atoi(optarg); break;
        case 'd': a.dims = std::atoi(optarg); break;
        case 'w': a.width = std::atoi(optarg); break;
        case 'p': a.ranks = std::atoi(optarg); break;
        case 'o': a.out = optarg; break;
        case 'q': a.quiet = true; break;
        default: return usage(argv[0]);
        }
    }
    std::vector<std::string> pos(argv + optind, argv + argc);
    if (!pos.empty() && (pos[0] == "emulator" || pos[0] == "hardware")) pos.erase(pos.begin());
    if (pos.size() != 2) return usage(argv[0]);
    const int ranks = launch.process() ? launch.size : a.ranks;
    a.num_points = std::atoi(pos[0].c_str());
    a.iterations = std::atoi(pos[1].c_str());
    if (a.num_points <= 0 || a.iterations < 0 || a.clusters < 1 || a.clusters > 256 || a.dims <= 0 || a.width <= 0 ||
        a.dims % a.width != 0 || ranks < 1 || a.num_points % ranks != 0) {
        std::fprintf(stderr, "bad arguments (num_points divisible by the ranks, dims a multiple of width, "
                             "1 <= clusters <= 256)\n");
        return 1;
    }
    return host::run_ranks(launch, a.ranks, [&](SMI_Comm comm) { return RankMain(comm, a); });
}
