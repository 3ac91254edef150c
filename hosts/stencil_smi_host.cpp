// stencil_smi_host.cpp -- a C++ host of the stencil_smi program on the C ABI.
//
// The reference host (examples/host/stencil_smi.cpp:126-413) runs one MPI
// process per rank: rank 0 builds the grid (0 inside, 1 on the edges,
// :175-187), cuts it into PX x PY tiles (SplitMemory, :48-62), every rank runs
// Read/Stencil/Write for T steps, rank 0 gathers the tiles (CombineMemory,
// :80-93), runs Reference() (:33-46) and accepts when every cell is within
// 1e-4 * mean of it (:391-405).  This host does the same against
// libsmi_amd.so with no Python in the loop: one host thread per rank on an
// in-process group (smi_local_group_create + smi_init_local, the threads
// standing in for the MPI ranks), each calling smi_stencil_run on its tile in
// device memory.  A process per GPU would call smi_init with an RCCL unique
// id distributed by the launcher instead.
//
//   stencil_smi_host X Y PX PY T [--init edges|uniform] [--out result.f32]
//                               [--repeat N] [--device D]
//
// Exit codes: 0 verified, 1 usage, 2 SMI/HIP error, 3 mismatch (as :398).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include <smi.h>

namespace {

using Grid = std::vector<float>;

struct Shape {
    int X, Y, PX, PY;
    int XL() const { return X / PX; }
    int YL() const { return Y / PY; }
};

// rank r owns tile (r / PY, r % PY) (stencil_smi.cpp:133-134)
std::vector<Grid> SplitMemory(const Grid &g, const Shape &s) {
    std::vector<Grid> tiles(s.PX * s.PY, Grid((size_t)s.XL() * s.YL()));
    for (int r = 0; r < s.PX * s.PY; ++r) {
        const int px = r / s.PY, py = r % s.PY;
        for (int x = 0; x < s.XL(); ++x)
            std::memcpy(&tiles[r][(size_t)x * s.YL()], &g[((size_t)px * s.XL() + x) * s.Y + (size_t)py * s.YL()],
                        sizeof(float) * s.YL());
    }
    return tiles;
}

Grid CombineMemory(const std::vector<Grid> &tiles, const Shape &s) {
    Grid g((size_t)s.X * s.Y);
    for (int r = 0; r < s.PX * s.PY; ++r) {
        const int px = r / s.PY, py = r % s.PY;
        for (int x = 0; x < s.XL(); ++x)
            std::memcpy(&g[((size_t)px * s.XL() + x) * s.Y + (size_t)py * s.YL()], &tiles[r][(size_t)x * s.YL()],
                        sizeof(float) * s.YL());
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

#define SMI_OK(call)                                                                          \
    do {                                                                                      \
        const int rc_ = (call);                                                               \
        if (rc_ != SMI_SUCCESS) {                                                             \
            std::fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, smi_last_error());       \
            return 2;                                                                         \
        }                                                                                     \
    } while (0)
#define HIP_OK(call)                                                                          \
    do {                                                                                      \
        const hipError_t e_ = (call);                                                         \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s failed: %s\n", #call, hipGetErrorString(e_));           \
            return 2;                                                                         \
        }                                                                                     \
    } while (0)

// One rank: its own communicator, device buffers and stream; `repeat` runs
// of T steps from the same input, the last one's tile returned.
int RunRank(int group, int rank, int device, const Shape &s, int T, int repeat, Grid &tile, double *seconds) {
    SMI_Comm comm;
    SMI_OK(smi_init_local(group, rank, device, &comm));
    const size_t n = (size_t)s.XL() * s.YL();
    float *buf[2] = {nullptr, nullptr};
    hipStream_t stream;
    HIP_OK(hipMalloc(&buf[0], n * sizeof(float)));
    HIP_OK(hipMalloc(&buf[1], n * sizeof(float)));
    HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    int half = 0;
    double best = 1e30;
    for (int it = 0; it < repeat; ++it) {
        HIP_OK(hipMemcpy(buf[0], tile.data(), n * sizeof(float), hipMemcpyHostToDevice));
        const auto t0 = std::chrono::steady_clock::now();
        SMI_OK(smi_stencil_run(comm, buf[0], buf[1], s.XL(), s.YL(), s.PX, s.PY, T, (SMI_Stream)stream, &half));
        SMI_OK(smi_stream_synchronize((SMI_Stream)stream));
        best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    // the result lies in half timesteps % 2 of the ping-pong pair (:344)
    HIP_OK(hipMemcpy(tile.data(), buf[half], n * sizeof(float), hipMemcpyDeviceToHost));
    *seconds = best;
    HIP_OK(hipStreamDestroy(stream));
    HIP_OK(hipFree(buf[0]));
    HIP_OK(hipFree(buf[1]));
    SMI_OK(smi_finalize(comm));
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s X Y PX PY T [--init edges|uniform] [--out file] [--repeat N] [--device D]\n",
                     argv[0]);
        return 1;
    }
    const Shape s{std::atoi(argv[1]), std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4])};
    const int T = std::atoi(argv[5]);
    std::string init = "edges", out;
    int repeat = 1, device = 0;
    for (int i = 6; i + 1 < argc; i += 2) {
        const std::string k = argv[i];
        if (k == "--init") init = argv[i + 1];
        else if (k == "--out") out = argv[i + 1];
        else if (k == "--repeat") repeat = std::max(1, std::atoi(argv[i + 1]));
        else if (k == "--device") device = std::atoi(argv[i + 1]);
        else {
            std::fprintf(stderr, "unknown option %s\n", k.c_str());
            return 1;
        }
    }
    if (s.PX <= 0 || s.PY <= 0 || s.X % s.PX || s.Y % s.PY || T < 0) {
        std::fprintf(stderr, "X, Y must split evenly into PX x PY tiles\n");
        return 1;
    }

    // the reference test pattern (stencil_smi.cpp:175-187), or a seeded
    // uniform [0, 1) grid with the same edges rule applied by the kernels
    Grid reference((size_t)s.X * s.Y, 0.0f);
    if (init == "edges") {
        for (int j = 0; j < s.Y; ++j) reference[j] = reference[(size_t)(s.X - 1) * s.Y + j] = 1.0f;
        for (int i = 0; i < s.X; ++i) reference[(size_t)i * s.Y] = reference[(size_t)i * s.Y + s.Y - 1] = 1.0f;
    } else {
        std::mt19937 gen(1234);
        std::uniform_real_distribution<float> u(0.0f, 1.0f);
        for (auto &v : reference) v = u(gen);
    }
    std::vector<Grid> tiles = SplitMemory(reference, s);

    int group = -1;
    SMI_OK(smi_local_group_create(s.PX * s.PY, &group));
    std::vector<int> rcs(s.PX * s.PY, 0);
    std::vector<double> secs(s.PX * s.PY, 0.0);
    std::vector<std::thread> ranks;
    for (int r = 0; r < s.PX * s.PY; ++r)
        ranks.emplace_back([&, r] { rcs[r] = RunRank(group, r, device, s, T, repeat, tiles[r], &secs[r]); });
    for (auto &t : ranks) t.join();
    for (int r = 0; r < s.PX * s.PY; ++r)
        if (rcs[r]) return rcs[r];
    const double elapsed = *std::max_element(secs.begin(), secs.end());
    std::printf("ranks %d (%dx%d), tile %dx%d, %d steps: %.6f s (best of %d), %.3f GCell/s\n", s.PX * s.PY, s.PX,
                s.PY, s.XL(), s.YL(), T, elapsed, repeat, (double)s.X * s.Y * T / elapsed / 1e9);

    const Grid result = CombineMemory(tiles, s);
    if (!out.empty()) {
        FILE *f = std::fopen(out.c_str(), "wb");
        if (!f || std::fwrite(result.data(), sizeof(float), result.size(), f) != result.size()) {
            std::fprintf(stderr, "cannot write %s\n", out.c_str());
            return 2;
        }
        std::fclose(f);
    }

    Reference(reference, s, T);
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
