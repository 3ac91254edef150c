// host_rt.h -- how the C++ hosts stand up their ranks on the C ABI, without
// MPI (absent from this image).
//
// The reference's host programs are one MPI process per rank: MPI_Init, rank
// and size from MPI_COMM_WORLD, SmiInit_<program>(rank, ranks, ...), and
// MPI_Barrier around every timed run (examples/host/stencil_smi.cpp:126-135,
// 301-329; microbenchmarks/host/*_benchmark.cpp).  Here a host runs its ranks
// one of two ways, with the same per-rank body:
//
//   threads (default)       -- one process, `ranks` host threads on an
//                              in-process group (smi_local_group_create +
//                              smi_init_local), all on one device;
//   --rank R --size N --uid FILE [--device D]
//                           -- one process per rank, the deployment of an
//                              8-GPU node: rank 0 writes smi_get_unique_id's
//                              bytes to FILE (written beside it and renamed,
//                              so a reader never sees part of it), the other
//                              ranks wait for FILE to appear and every rank
//                              calls smi_init (RCCL); rank 0 removes FILE
//                              once smi_init has returned.  FILE must not
//                              exist when the ranks start.  The device
//                              defaults to R modulo the visible devices.
//
// MPI_Barrier is restated on the communicator (Barrier below); tiles and
// results move with smi_scatter / smi_gather where the reference used
// MPI_Send / MPI_Recv.  A failing SMI or HIP call prints the error and ends
// the whole process with exit code 2: a rank that returned early would leave
// its peers waiting at a barrier or in a transfer forever.
#pragma once

#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <initializer_list>
#include <string>
#include <thread>
#include <vector>

#include <smi.h>

namespace host {

[[noreturn]] inline void die(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vfprintf(stderr, fmt, ap);
    va_end(ap);
    std::fflush(stderr);
    std::fflush(stdout);
    std::_Exit(code);
}

#define SMI_OK(call)                                                                         \
    do {                                                                                     \
        const int rc_ = (call);                                                              \
        if (rc_ != SMI_SUCCESS) host::die(2, "%s failed (%d): %s\n", #call, rc_, smi_last_error()); \
    } while (0)
#define HIP_OK(call)                                                                         \
    do {                                                                                     \
        const hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess) host::die(2, "%s failed: %s\n", #call, hipGetErrorString(e_)); \
    } while (0)

struct Launch {
    int ranks = 0;     // threads mode: rank threads (0 = the host's default)
    int rank = -1;     // process mode: this process's rank (-1 = threads mode)
    int size = 0;      // process mode: ranks in the job
    std::string uid;   // process mode: unique-id file
    int device = -1;   // -1: threads mode 0, process mode rank % devices
    bool process() const { return rank >= 0; }
};

inline const char *env_of(std::initializer_list<const char *> names) {
    for (const char *n : names)
        if (const char *v = std::getenv(n)) return v;
    return nullptr;
}

// Takes --rank/--size/--uid/--device/--fake-host out of argv (the host
// parses the rest).  Without --rank, a launcher's environment selects the
// one-process-per-rank mode as mpirun does for the reference's hosts:
// torchrun (RANK, WORLD_SIZE, LOCAL_RANK; `torchrun --no-python
// --nproc-per-node 8 hosts/_build/stencil_smi_host ...`), Open MPI
// (OMPI_COMM_WORLD_*), MPICH / Slurm (PMI_RANK / PMI_SIZE, SLURM_PROCID /
// SLURM_NTASKS).  The id file then defaults to $TMPDIR/smi_uid.<job>, the
// job named by MASTER_PORT, SLURM_JOB_ID or the launcher's process id.
// --fake-host gives every rank its own NCCL_HOSTID (bench.py --fake-host):
// several ranks on one GPU, RCCL over its socket transport -- testing only.
// Returns false on a malformed launch.
inline bool parse_launch(int &argc, char **argv, Launch *l) {
    int out = 1;
    bool fake_host = false;
    bool device_given = false;
    for (int i = 1; i < argc; ++i) {
        const std::string k = argv[i];
        if ((k == "--rank" || k == "--size" || k == "--uid" || k == "--device") && i + 1 < argc) {
            const char *v = argv[++i];
            if (k == "--rank") l->rank = std::atoi(v);
            else if (k == "--size") l->size = std::atoi(v);
            else if (k == "--uid") l->uid = v;
            else {
                l->device = std::atoi(v);
                device_given = true;
            }
        } else if (k == "--fake-host") {
            fake_host = true;
        } else {
            argv[out++] = argv[i];
        }
    }
    argc = out;
    argv[argc] = nullptr;
    if (l->rank < 0) {
        const char *r = env_of({"RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "SLURM_PROCID"});
        const char *n = env_of({"WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "SLURM_NTASKS"});
        if (r && n) {
            l->rank = std::atoi(r);
            l->size = std::atoi(n);
            if (l->device < 0)
                if (const char *lr = env_of({"LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID",
                                             "SLURM_LOCALID"}))
                    l->device = std::atoi(lr);
            if (l->uid.empty()) {
                const char *job = env_of({"MASTER_PORT", "SLURM_JOB_ID"});
                const char *tmp = env_of({"TMPDIR"});
                l->uid = std::string(tmp ? tmp : "/tmp") + "/smi_uid." +
                         (job ? std::string(job) : std::to_string(getppid()));
            }
        }
    }
    if (l->rank >= 0 && (l->size <= 0 || l->rank >= l->size || l->uid.empty())) return false;
    if (fake_host && l->rank >= 0) {
        // before the first HIP / RCCL call: RCCL reads it at communicator set-up
        const std::string id = "smi-fake-host-" + std::to_string(l->rank);
        setenv("NCCL_HOSTID", id.c_str(), 1);
        if (!device_given) l->device = 0;  // every rank on GPU 0
    }
    return true;
}

inline void publish_uid(const std::string &path, const char *id) {
    const std::string tmp = path + ".tmp." + std::to_string(getpid());
    FILE *f = std::fopen(tmp.c_str(), "wb");
    if (!f || std::fwrite(id, 1, SMI_UNIQUE_ID_BYTES, f) != (size_t)SMI_UNIQUE_ID_BYTES || std::fclose(f) != 0)
        die(2, "cannot write the unique id to %s\n", tmp.c_str());
    if (std::rename(tmp.c_str(), path.c_str()) != 0) die(2, "cannot rename %s to %s\n", tmp.c_str(), path.c_str());
}

inline void await_uid(const std::string &path, char *id) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        if (FILE *f = std::fopen(path.c_str(), "rb")) {
            const size_t n = std::fread(id, 1, SMI_UNIQUE_ID_BYTES, f);
            std::fclose(f);
            if (n == (size_t)SMI_UNIQUE_ID_BYTES) return;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(300))
            die(2, "no unique id in %s after 300 s (is rank 0 running?)\n", path.c_str());
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
}

// Runs body(comm) on every rank this process hosts and returns the largest
// of their exit codes.  Threads mode: `ranks` threads (l.ranks if set);
// process mode: this process's rank.
inline int run_ranks(const Launch &l, int ranks, const std::function<int(SMI_Comm)> &body) {
    if (l.process()) {
        int dev = l.device;
        if (dev < 0) {
            int n = 0;
            SMI_OK(smi_device_count(&n));
            dev = n > 0 ? l.rank % n : 0;
        }
        char id[SMI_UNIQUE_ID_BYTES];
        if (l.rank == 0) {
            SMI_OK(smi_get_unique_id(id, SMI_UNIQUE_ID_BYTES));
            publish_uid(l.uid, id);
        } else {
            await_uid(l.uid, id);
        }
        SMI_Comm comm;
        SMI_OK(smi_init(l.rank, l.size, dev, id, SMI_UNIQUE_ID_BYTES, &comm));
        // smi_init is collective: once it returns every rank has read the
        // id, so rank 0 removes the file (a later job on the same path then
        // cannot pick up this job's id)
        if (l.rank == 0) std::remove(l.uid.c_str());
        const int rc = body(comm);
        SMI_OK(smi_finalize(comm));
        return rc;
    }
    const int n = l.ranks > 0 ? l.ranks : ranks;
    const int dev = l.device >= 0 ? l.device : 0;
    int group = -1;
    SMI_OK(smi_local_group_create(n, &group));
    std::vector<int> rcs(n, 0);
    std::vector<std::thread> th;
    for (int r = 0; r < n; ++r)
        th.emplace_back([&, r] {
            SMI_Comm comm;
            SMI_OK(smi_init_local(group, r, dev, &comm));
            rcs[r] = body(comm);
            SMI_OK(smi_finalize(comm));
        });
    for (auto &t : th) t.join();
    int rc = 0;
    for (int v : rcs) rc = std::max(rc, v);
    return rc;
}

// MPI_Barrier on the communicator: an int sum-reduce to rank 0, then a
// broadcast back from it.  No rank's broadcast completes before rank 0 has
// every rank's contribution, i.e. before every rank has entered.
class Barrier {
  public:
    Barrier(SMI_Comm comm, hipStream_t s) : comm_(comm), s_(s) {
        HIP_OK(hipMalloc(&buf_, 8 * sizeof(int)));  // send word, receive word 16 B apart
        HIP_OK(hipMemsetAsync(buf_, 0, 8 * sizeof(int), s_));
    }
    ~Barrier() { (void)hipFree(buf_); }
    Barrier(const Barrier &) = delete;
    Barrier &operator=(const Barrier &) = delete;
    void wait() {
        SMI_OK(smi_reduce(comm_, buf_, buf_ + 4, 1, SMI_INT, SMI_ADD, 0, 0, (SMI_Stream)s_));
        SMI_OK(smi_bcast(comm_, buf_ + 4, 1, SMI_INT, 0, 0, (SMI_Stream)s_));
        SMI_OK(smi_stream_synchronize((SMI_Stream)s_));
    }

  private:
    SMI_Comm comm_;
    hipStream_t s_;
    int *buf_ = nullptr;
};

// The reference harness's statistics (reduce_benchmark.cpp:120-155,
// broadcast_benchmark.cpp:129-147): mean, population standard deviation and
// the 99 % confidence interval 2.58 sigma / sqrt(runs), all in usecs.
struct Stats {
    double mean = 0, stddev = 0, ci99 = 0;
};
inline Stats stats_of(const std::vector<double> &t) {
    Stats s;
    if (t.empty()) return s;
    for (double v : t) s.mean += v;
    s.mean /= t.size();
    for (double v : t) s.stddev += (v - s.mean) * (v - s.mean);
    s.stddev = std::sqrt(s.stddev / t.size());
    s.ci99 = 2.58 * s.stddev / std::sqrt((double)t.size());
    return s;
}

// The harness's report on the root (reduce_benchmark.cpp:129-155,
// broadcast_benchmark.cpp:129-163): the summary on stdout and, when `path` is
// set, the .dat file ("#"-lines, then one run time per line).
inline void report(const char *what, const char *mode, int ranks, long n, size_t elem_bytes,
                   const std::vector<double> &times_us, const std::string &path) {
    const Stats st = stats_of(times_us);
    const double kb = (double)n * elem_bytes / 1024.0;
    const double gbit = (kb * 8 / (st.mean / 1e6)) / (1024 * 1024);
    std::printf("-------------------------------------------------------------------\n");
    std::printf("Computation time (usec): %g (sttdev: %g)\n", st.mean, st.stddev);
    std::printf("Conf interval 99: %g\n", st.ci99);
    std::printf("Conf interval 99 within %g%% from mean\n", st.ci99 / st.mean * 100);
    std::printf("Sent (KB): %g\n", kb);
    std::printf("Average bandwidth (Gbit/s): %g\n", gbit);
    std::printf("-------------------------------------------------------------------\n");
    if (path.empty()) return;
    FILE *f = std::fopen(path.c_str(), "w");
    if (!f) die(2, "cannot write %s\n", path.c_str());
    std::fprintf(f, "#SMI %s (%s), executed with %d ranks, streaming: %ld elements\n", what, mode, ranks, n);
    std::fprintf(f, "#Sent (KB) = %g, Runs = %zu\n", kb, times_us.size());
    std::fprintf(f, "#Average Computation time (usecs): %g\n", st.mean);
    std::fprintf(f, "#Standard deviation (usecs): %g\n", st.stddev);
    std::fprintf(f, "#Confidence interval 99%%: +- %g\n", st.ci99);
    std::fprintf(f, "#Average bandwidth (Gbit/s): %g\n", gbit);
    std::fprintf(f, "#Execution times (usecs):\n");
    for (double t : times_us) std::fprintf(f, "%g\n", t);
    std::fclose(f);
}

}  // namespace host
