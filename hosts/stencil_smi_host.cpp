// stencil_smi_host.cpp -- a C++ host of the stencil_smi program on the C ABI.
//
// The reference host (examples/host/stencil_smi.cpp:126-413) runs one MPI
// process per rank: rank 0 builds the grid (0 inside, 1 on the edges,
// :175-187), cuts it into PX x PY tiles (SplitMemory, :48-62) and sends each
// rank its tile (:191-200), every rank runs Read/Stencil/Write for T steps
// between two barriers (:301-329), rank 0 collects the tiles (:361-373,
// CombineMemory :80-93), runs Reference() (:33-46) and accepts when every
// cell is within 1e-4 * mean of it (:391-405).  This host does the same
// against libsmi_amd.so with no Python in the loop, with either launch of
// host_rt.h: one process per rank (--rank/--size/--uid, smi_init over RCCL)
// or rank threads of one process.  Tiles go out with smi_scatter and come
// back with smi_gather from device memory; every rank calls smi_stencil_run
// on its tile.
//
//   stencil_smi_host X Y PX PY T [--init edges|uniform] [--out result.f32]
//                    [--repeat N] [--device D] [--rank R --size PX*PY --uid FILE]
//
// Exit codes: 0 verified, 1 usage, 2 SMI/HIP error, 3 mismatch (as :398).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "host_rt.h"

namespace {

using Grid = std::vector<float>;

struct Shape {
    int X, Y, PX, PY;
    int XL() const { return X / PX; }
    int YL() const { return Y / PY; }
    size_t tile() const { return (size_t)XL() * YL(); }
};

struct Opts {
    std::string init = "edges", out;
    int T = 0, repeat = 1;
};

// rank r owns tile (r / PY, r % PY) (stencil_smi.cpp:133-134); the tiles are
// laid out one after another in rank order, as smi_scatter hands them out
Grid SplitMemory(const Grid &g, const Shape &s) {
    Grid tiles(s.tile() * s.PX * s.PY);
    for (int r = 0; r < s.PX * s.PY; ++r) {
        const int px = r / s.PY, py = r % s.PY;
        for (int x = 0; x < s.XL(); ++x)
            std::memcpy(&tiles[r * s.tile() + (size_t)x * s.YL()],
                        &g[((size_t)px * s.XL() + x) * s.Y + (size_t)py * s.YL()], sizeof(float) * s.YL());
    }
    return tiles;
}

Grid CombineMemory(const Grid &tiles, const Shape &s) {
    Grid g((size_t)s.X * s.Y);
    for (int r = 0; r < s.PX * s.PY; ++r) {
        const int px = r / s.PY, py = r % s.PY;
        for (int x = 0; x < s.XL(); ++x)
            std::memcpy(&g[((size_t)px * s.XL() + x) * s.Y + (size_t)py * s.YL()],
                        &tiles[r * s.tile() + (size_t)x * s.YL()], sizeof(float) * s.YL());
    }
    return g;
}

// The reference host's check order: 0.25 * (N + S + W + E), edges kept
// (stencil_smi.cpp:33-46).  The device order differs (S + W + E + N,
// stencil_smi.cl:153-156), which is why the acceptance test is a tolerance.
void Reference(Grid &d, const Shape &s, int T) {
    Grid b(d);
    for (int t = 0; t < T; ++t) {
        for (int i = 1; i < s.X - 1; ++i)
            for (int j = 1; j < s.Y - 1; ++j)
                b[(size_t)i * s.Y + j] = 0.25f * (d[(size_t)(i - 1) * s.Y + j] + d[(size_t)(i + 1) * s.Y + j] +
                                                  d[(size_t)i * s.Y + j - 1] + d[(size_t)i * s.Y + j + 1]);
        d.swap(b);
    }
}

// the reference test pattern (stencil_smi.cpp:175-187), or a seeded uniform
// [0, 1) grid (the kernels keep the global edges either way)
Grid InitialGrid(const Shape &s, const std::string &init) {
    Grid g((size_t)s.X * s.Y, 0.0f);
    if (init == "edges") {
        for (int j = 0; j < s.Y; ++j) g[j] = g[(size_t)(s.X - 1) * s.Y + j] = 1.0f;
        for (int i = 0; i < s.X; ++i) g[(size_t)i * s.Y] = g[(size_t)i * s.Y + s.Y - 1] = 1.0f;
    } else {
        std::mt19937 gen(1234);
        std::uniform_real_distribution<float> u(0.0f, 1.0f);
        for (auto &v : g) v = u(gen);
    }
    return g;
}

// Rank 0's side after the run: combine, write, check against Reference().
int Verify(const Grid &gathered, const Shape &s, const Opts &o, double seconds) {
    std::printf("ranks %d (%dx%d), tile %dx%d, %d steps: %.6f s (best of %d), %.3f GCell/s\n", s.PX * s.PY, s.PX,
                s.PY, s.XL(), s.YL(), o.T, seconds, o.repeat, (double)s.X * s.Y * o.T / seconds / 1e9);
    const Grid result = CombineMemory(gathered, s);
    if (!o.out.empty()) {
        FILE *f = std::fopen(o.out.c_str(), "wb");
        if (!f || std::fwrite(result.data(), sizeof(float), result.size(), f) != result.size()) {
            std::fprintf(stderr, "cannot write %s\n", o.out.c_str());
            return 2;
        }
        std::fclose(f);
    }
    Grid reference = InitialGrid(s, o.init);
    Reference(reference, s, o.T);
    // the mean is accumulated in double and stored as float (:391-393)
    const float average = (float)(std::accumulate(reference.begin(), reference.end(), 0.0) / reference.size());
    for (int i = 0; i < s.X; ++i)
        for (int j = 0; j < s.Y; ++j) {
            const float res = result[(size_t)i * s.Y + j], ref = reference[(size_t)i * s.Y + j];
            if (std::abs(ref - res) >= 1e-4 * average) {
                std::fprintf(stderr, "Mismatch found at (%d, %d): %g (should be %g).\n", i, j, res, ref);
                return 3;
            }
        }
    std::printf("Successfully verified result.\n");
    return 0;
}

// One rank: its tile from rank 0, `repeat` runs of T steps from it between
// two barriers (the best run's time reported by rank 0), the last result
// back to rank 0.
int RankMain(SMI_Comm comm, const Shape &s, const Opts &o) {
    const int rank = SMI_Comm_rank(comm), ranks = SMI_Comm_size(comm);
    const size_t n = s.tile();
    hipStream_t stream;
    HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    float *buf[2] = {nullptr, nullptr}, *init = nullptr, *all = nullptr;
    HIP_OK(hipMalloc(&buf[0], n * sizeof(float)));
    HIP_OK(hipMalloc(&buf[1], n * sizeof(float)));
    HIP_OK(hipMalloc(&init, n * sizeof(float)));
    if (rank == 0) {
        HIP_OK(hipMalloc(&all, n * ranks * sizeof(float)));
        const Grid tiles = SplitMemory(InitialGrid(s, o.init), s);
        HIP_OK(hipMemcpy(all, tiles.data(), tiles.size() * sizeof(float), hipMemcpyHostToDevice));
    }
    // rank 0 sends each rank its tile (:191-200)
    SMI_OK(smi_scatter(comm, all, init, n, SMI_FLOAT, 0, 0, (SMI_Stream)stream));
    host::Barrier barrier(comm, stream);
    int half = 0;
    double best = 1e30;
    for (int it = 0; it < o.repeat; ++it) {
        HIP_OK(hipMemcpyAsync(buf[0], init, n * sizeof(float), hipMemcpyDeviceToDevice, stream));
        barrier.wait();  // (:301)
        const auto t0 = std::chrono::steady_clock::now();
        SMI_OK(smi_stencil_run(comm, buf[0], buf[1], s.XL(), s.YL(), s.PX, s.PY, o.T, (SMI_Stream)stream, &half));
        SMI_OK(smi_stream_synchronize((SMI_Stream)stream));
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        best = std::min(best, sec);
        if (rank == 0 && o.repeat > 1) {
            std::printf("run %d: %.6f s\n", it, sec);
            std::fflush(stdout);
        }
        barrier.wait();  // (:329)
    }
    // the result lies in half timesteps % 2 of the ping-pong pair (:344);
    // rank 0 collects every tile (:361-373)
    SMI_OK(smi_gather(comm, buf[half], all, n, SMI_FLOAT, 0, 0, (SMI_Stream)stream));
    SMI_OK(smi_stream_synchronize((SMI_Stream)stream));
    int rc = 0;
    if (rank == 0) {
        Grid gathered(n * ranks);
        HIP_OK(hipMemcpy(gathered.data(), all, gathered.size() * sizeof(float), hipMemcpyDeviceToHost));
        rc = Verify(gathered, s, o, best);
        HIP_OK(hipFree(all));
    }
    HIP_OK(hipFree(init));
    HIP_OK(hipFree(buf[0]));
    HIP_OK(hipFree(buf[1]));
    HIP_OK(hipStreamDestroy(stream));
    return rc;
}

}  // namespace

int main(int argc, char **argv) {
    host::Launch launch;
    if (!host::parse_launch(argc, argv, &launch) || argc < 6) {
        std::fprintf(stderr,
                     "usage: %s X Y PX PY T [--init edges|uniform] [--out file] [--repeat N] [--device D]"
                     " [--rank R --size PX*PY --uid FILE]\n",
                     argv[0]);
        return 1;
    }
    const Shape s{std::atoi(argv[1]), std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4])};
    Opts o;
    o.T = std::atoi(argv[5]);
    for (int i = 6; i + 1 < argc; i += 2) {
        const std::string k = argv[i];
        if (k == "--init") o.init = argv[i + 1];
        else if (k == "--out") o.out = argv[i + 1];
        else if (k == "--repeat") o.repeat = std::max(1, std::atoi(argv[i + 1]));
        else {
            std::fprintf(stderr, "unknown option %s\n", k.c_str());
            return 1;
        }
    }
    if (s.PX <= 0 || s.PY <= 0 || s.X % s.PX || s.Y % s.PY || o.T < 0) {
        std::fprintf(stderr, "X, Y must split evenly into PX x PY tiles\n");
        return 1;
    }
    if (launch.process() && launch.size != s.PX * s.PY) {
        std::fprintf(stderr, "--size must be PX * PY = %d\n", s.PX * s.PY);
        return 1;
    }
    return host::run_ranks(launch, s.PX * s.PY, [&](SMI_Comm comm) { return RankMain(comm, s, o); });
}
