// runtime.cpp -- communicator table, error reporting, workspace, profiling.
//
// Replaces the generated host initialiser SmiInit_<program>
// (codegen/templates/host_hlslib.cl:8-90): there are no routing tables to
// load and no support kernels to fork -- rank r is GPU r, and the transport
// is an RCCL communicator (or an in-process device-copy group for tests).
#include <algorithm>
#include <mutex>
#include <unordered_map>

#include <cstdlib>

#include "smi_internal.h"

namespace smi {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

size_t type_size(int type) {
    switch (type) {  // include/smi/network_message.h:27-31
    case SMI_CHAR: return 1;
    case SMI_SHORT: return 2;
    case SMI_INT: return 4;
    case SMI_FLOAT: return 4;
    case SMI_DOUBLE: return 8;
    default: return 0;
    }
}

// ---------------------------------------------------------- comm table --
static std::mutex g_comm_mu;
static std::unordered_map<int, std::unique_ptr<Comm>> g_comms;
static int g_next_handle = 1;

Comm *lookup_comm(SMI_Comm c) {
    std::lock_guard<std::mutex> lk(g_comm_mu);
    auto it = g_comms.find(c.handle);
    if (it == g_comms.end()) return nullptr;
    Comm *p = it->second.get();
    if (p->rank != c.rank || p->size != c.size) return nullptr;
    return p;
}

static int register_comm(std::unique_ptr<Comm> c, SMI_Comm *out) {
    std::lock_guard<std::mutex> lk(g_comm_mu);
    int h = g_next_handle++;
    out->rank = c->rank;
    out->size = c->size;
    out->handle = h;
    g_comms[h] = std::move(c);
    return SMI_SUCCESS;
}

int comm_workspace(Comm *c, size_t bytes, void **ptr) {
    if (bytes > c->work_bytes) {
        if (c->work) SMI_HIP_CHECK(hipFree(c->work));
        c->work = nullptr;
        c->work_bytes = 0;
        size_t want = bytes < (1u << 20) ? (1u << 20) : bytes;
        SMI_HIP_CHECK(hipMalloc(&c->work, want));
        c->work_bytes = want;
    }
    *ptr = c->work;
    return SMI_SUCCESS;
}

int comm_event(Comm *c, int idx, hipEvent_t *ev) {
    while ((int)c->events.size() <= idx) {
        hipEvent_t e;
        // device-side ordering between this communicator's streams only: no
        // system-scope release at the record (it made the kernel before it
        // write its L2 back to memory, ~10 us between stencil passes)
        SMI_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
        c->events.push_back(e);
    }
    *ev = c->events[idx];
    return SMI_SUCCESS;
}

static int finish_init(std::unique_ptr<Comm> c, SMI_Comm *out) {
    // highest priority: the ring kernels and the exchange it carries are on
    // the critical path, the interior sweep beside them is not
    int least = 0, greatest = 0;
    SMI_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    int prio = greatest;
#ifdef SMI_LOOPBACK_REHEARSAL
    if (getenv("SMI_COMM_LOW_PRIORITY")) prio = least;  // experiment: ring in the interior's tail
#endif
    SMI_HIP_CHECK(hipStreamCreateWithPriority(&c->comm_stream, hipStreamNonBlocking, prio));
    return register_comm(std::move(c), out);
}

// ------------------------------------------------------------ profiling --
struct ProfRec {
    int kernel;
    int tag;
    double units;
    hipEvent_t a, b;
    bool owns_a;  // false: `a` is the previous record's `b` (chained)
};
static std::mutex g_prof_mu;
static bool g_prof_on = false;
static std::vector<ProfRec> g_prof_recs;
static std::vector<hipEvent_t> g_prof_pool;
// the last record's end marker, while nothing else has been recorded since:
// a chained begin on the same stream reuses it instead of recording another
static int g_prof_last = -1;
static hipStream_t g_prof_last_stream = nullptr;

bool prof_enabled() { return g_prof_on; }

static int prof_get_event(hipEvent_t *e) {
    if (!g_prof_pool.empty()) {
        *e = g_prof_pool.back();
        g_prof_pool.pop_back();
        return SMI_SUCCESS;
    }
    // timing markers only: no system-scope release/acquire (a default event
    // fences at system scope, which cost ~1 us per marker between
    // back-to-back sweep launches)
    SMI_HIP_CHECK(hipEventCreateWithFlags(e, hipEventDisableSystemFence));
    return SMI_SUCCESS;
}

// chain = true: the caller enqueued nothing on `stream` since the previous
// prof_end on it (back-to-back passes), so that end marker is this launch's
// begin -- one marker per launch instead of two (the markers cost ~2 us each
// between back-to-back 0.11 ms sweeps, 4 % of a 200-pass run with two).
int prof_begin(int kernel, hipStream_t stream, int *token, int tag, double units, bool chain) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    ProfRec r;
    r.kernel = kernel;
    r.tag = tag;
    r.units = units;
    if (chain && g_prof_last >= 0 && g_prof_last_stream == stream) {
        r.a = g_prof_recs[g_prof_last].b;
        r.owns_a = false;
    } else {
        SMI_TRY(prof_get_event(&r.a));
        r.owns_a = true;
        SMI_HIP_CHECK(hipEventRecord(r.a, stream));
    }
    SMI_TRY(prof_get_event(&r.b));
    *token = (int)g_prof_recs.size();
    g_prof_recs.push_back(r);
    g_prof_last = -1;
    return SMI_SUCCESS;
}

// A record whose two events the caller hands to the launch itself
// (hipExtLaunchKernelGGL start / stop events): the dispatch stamps the
// kernel's own start and end, and no marker packet sits between kernels.
int prof_launch(int kernel, int *token, int tag, double units, hipEvent_t *start, hipEvent_t *stop) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    ProfRec r;
    r.kernel = kernel;
    r.tag = tag;
    r.units = units;
    SMI_TRY(prof_get_event(&r.a));
    SMI_TRY(prof_get_event(&r.b));
    r.owns_a = true;
    *start = r.a;
    *stop = r.b;
    *token = (int)g_prof_recs.size();
    g_prof_recs.push_back(r);
    g_prof_last = -1;  // nothing to chain to
    return SMI_SUCCESS;
}

// the next prof_begin records its own marker (a caller's own work may
// follow the last one on the stream)
void prof_break_chain() {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_last = -1;
}

int prof_end(int token, hipStream_t stream) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    SMI_HIP_CHECK(hipEventRecord(g_prof_recs[token].b, stream));
    g_prof_last = token;
    g_prof_last_stream = stream;
    return SMI_SUCCESS;
}

}  // namespace smi

using namespace smi;

extern "C" {

const char *smi_last_error(void) { return g_last_error.c_str(); }

int smi_device_count(int *count) {
    SMI_ARG_CHECK(count, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return SMI_SUCCESS;
}

int smi_stream_synchronize(SMI_Stream stream) {
    SMI_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
    return SMI_SUCCESS;
}

size_t smi_type_size(SMI_Datatype type) { return type_size(type); }

int smi_init(int rank, int size, int device, const void *unique_id, int id_bytes,
             SMI_Comm *comm) {
    SMI_ARG_CHECK(comm && unique_id, "NULL comm or unique id");
    SMI_ARG_CHECK(size >= 1 && rank >= 0 && rank < size, "rank/size");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        set_error("no GPU visible");
        return SMI_ERR_NO_DEVICE;
    }
    SMI_ARG_CHECK(device >= 0 && device < ndev, "device out of range");
    SMI_HIP_CHECK(hipSetDevice(device));
    auto c = std::make_unique<Comm>();
    c->rank = rank;
    c->size = size;
    c->device = device;
    int rc = SMI_SUCCESS;
    c->transport = make_rccl_transport(rank, size, unique_id, id_bytes, &rc);
    if (rc != SMI_SUCCESS) return rc;
    return finish_init(std::move(c), comm);
}

int smi_init_local(int group_id, int rank, int device, SMI_Comm *comm) {
    SMI_ARG_CHECK(comm, "NULL comm");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        set_error("no GPU visible");
        return SMI_ERR_NO_DEVICE;
    }
    SMI_ARG_CHECK(device >= 0 && device < ndev, "device out of range");
    SMI_HIP_CHECK(hipSetDevice(device));
    int rc = SMI_SUCCESS;
    auto t = make_local_transport(group_id, rank, device, &rc);
    if (rc != SMI_SUCCESS) return rc;
    auto c = std::make_unique<Comm>();
    c->rank = rank;
    c->size = local_group_size(group_id);
    c->device = device;
    c->transport = std::move(t);
    return finish_init(std::move(c), comm);
}

int smi_comm_dup(SMI_Comm comm, SMI_Comm *out) {
    SMI_ARG_CHECK(out, "NULL output");
    Comm *c = lookup_comm(comm);
    if (!c) {
        set_error("unknown communicator");
        return SMI_ERR_BAD_COMM;
    }
    SMI_HIP_CHECK(hipSetDevice(c->device));
    int rc = SMI_SUCCESS;
    auto t = c->transport->dup(&rc);
    if (rc != SMI_SUCCESS) return rc;
    auto d = std::make_unique<Comm>();
    d->rank = c->rank;
    d->size = c->size;
    d->device = c->device;
    d->transport = std::move(t);
    return finish_init(std::move(d), out);
}

int smi_finalize(SMI_Comm comm) {
    std::unique_ptr<Comm> c;
    {
        std::lock_guard<std::mutex> lk(g_comm_mu);
        auto it = g_comms.find(comm.handle);
        if (it == g_comms.end()) {
            set_error("unknown communicator");
            return SMI_ERR_BAD_COMM;
        }
        c = std::move(it->second);
        g_comms.erase(it);
    }
    SMI_HIP_CHECK(hipSetDevice(c->device));
    if (c->comm_stream) SMI_HIP_CHECK(hipStreamSynchronize(c->comm_stream));
    if (c->interior_stream) SMI_HIP_CHECK(hipStreamSynchronize(c->interior_stream));
    SMI_HIP_CHECK(hipDeviceSynchronize());
    int drain_rc = channels_drain(c.get());
    c->chan_engine.reset();
    c->transport.reset();
    for (auto e : c->events) SMI_HIP_CHECK(hipEventDestroy(e));
    if (c->work) SMI_HIP_CHECK(hipFree(c->work));
    if (c->halo) SMI_HIP_CHECK(hipFree(c->halo));
    if (c->comm_stream) SMI_HIP_CHECK(hipStreamDestroy(c->comm_stream));
    if (c->interior_stream) SMI_HIP_CHECK(hipStreamDestroy(c->interior_stream));
    return drain_rc;
}

int smi_prof_enable(int enable) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_on = enable != 0;
    return SMI_SUCCESS;
}

int smi_prof_reset(void) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    for (auto &r : g_prof_recs) {
        SMI_HIP_CHECK(hipEventSynchronize(r.b));
        if (r.owns_a) g_prof_pool.push_back(r.a);
        g_prof_pool.push_back(r.b);
    }
    g_prof_recs.clear();
    g_prof_last = -1;
    return SMI_SUCCESS;
}

int smi_prof_read(int kernel, double *total_ms, long *launches) {
    return smi_prof_read_tag(kernel, -1, total_ms, launches, nullptr);
}

int smi_prof_read_tag(int kernel, int tag, double *total_ms, long *launches, double *units) {
    SMI_ARG_CHECK(total_ms && launches, "NULL output");
    std::lock_guard<std::mutex> lk(g_prof_mu);
    double sum = 0.0, u = 0.0;
    long n = 0;
    for (auto &r : g_prof_recs) {
        if (r.kernel != kernel || (tag >= 0 && r.tag != tag)) continue;
        SMI_HIP_CHECK(hipEventSynchronize(r.b));
        float ms = 0.f;
        SMI_HIP_CHECK(hipEventElapsedTime(&ms, r.a, r.b));
        sum += ms;
        u += r.units;
        ++n;
    }
    *total_ms = sum;
    *launches = n;
    if (units) *units = u;
    return SMI_SUCCESS;
}

int smi_prof_list(int *kernels, int *tags, int max_entries, int *n_entries) {
    SMI_ARG_CHECK(n_entries && (max_entries == 0 || (kernels && tags)), "NULL output");
    std::lock_guard<std::mutex> lk(g_prof_mu);
    // distinct (kernel, tag) pairs in first-recorded order, independent of
    // the caller's buffer (a max_entries = 0 size query counts them too)
    std::vector<std::pair<int, int>> keys;
    for (auto &r : g_prof_recs) {
        const std::pair<int, int> k(r.kernel, r.tag);
        if (std::find(keys.begin(), keys.end(), k) == keys.end()) keys.push_back(k);
    }
    for (int i = 0; i < (int)keys.size() && i < max_entries; ++i) {
        kernels[i] = keys[i].first;
        tags[i] = keys[i].second;
    }
    *n_entries = (int)keys.size();
    return SMI_SUCCESS;
}

}  // extern "C"
