// transport.cpp -- the two point-to-point transports behind the channels.
//
// The reference moves 32-byte packets through CK_S/CK_R kernels and QSFP
// links chosen by routing tables (codegen/templates/cks.cl:3-84, ckr.cl:
// 3-88); on one MI355X node every GPU pair is a direct xGMI link, so a
// transfer is a plain RCCL send/recv between the two ranks.
//
//  * RcclTransport  -- production: one process per GPU, RCCL over xGMI.
//  * LocalTransport -- ranks are host threads of one process sharing one (or
//    several) devices; a transfer is a device-to-device hipMemcpyAsync
//    ordered by HIP events.  It exists so that multi-rank parity tests can run
//    on a single GPU (RCCL refuses two ranks on one device).
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <tuple>

#include "smi_internal.h"

namespace smi {

// ================================================================= RCCL ==
class RcclTransport final : public Transport {
  public:
    // `chan`: a second communicator over the same ranks (ncclCommSplit) that
    // carries only the element-granular channel packets, so they never
    // match a bulk receive of a collective or a stencil exchange -- the
    // reference's ports keep those streams apart the same way (one FIFO
    // per port).
    RcclTransport(ncclComm_t c, ncclComm_t chan) : comm_(c), chan_(chan) {}
    ~RcclTransport() override {
        if (chan_) ncclCommDestroy(chan_);
        if (comm_) ncclCommDestroy(comm_);
    }
    // begin() holds the bulk mutex until end(): two host threads can never
    // interleave their groups on the one RCCL communicator (RCCL
    // communicators are not thread-safe).  Matching stays in issue order per
    // rank pair, so every rank must issue its bulk operations in the same
    // order (include/smi/communicator.h).
    int begin(hipStream_t stream) override {
        bulk_mu_.lock();
        stream_ = stream;
        const int rc = check(ncclGroupStart(), "ncclGroupStart");
        if (rc != SMI_SUCCESS) bulk_mu_.unlock();
        return rc;
    }
    int send(const void *buf, size_t bytes, int peer) override {
        if (bytes == 0) return SMI_SUCCESS;
        return check(ncclSend(buf, bytes, ncclUint8, peer, comm_, stream_), "ncclSend");
    }
    int recv(void *buf, size_t bytes, int peer) override {
        if (bytes == 0) return SMI_SUCCESS;
        return check(ncclRecv(buf, bytes, ncclUint8, peer, comm_, stream_), "ncclRecv");
    }
    int end() override {
        const int rc = check(ncclGroupEnd(), "ncclGroupEnd");
        bulk_mu_.unlock();
        return rc;
    }

    // Channel packets travel on `chan_`, whose connections to every peer
    // were set up at init (connect_all), so a send never waits for a
    // connection handshake with a peer that is busy elsewhere.  A packet
    // (2 KiB) fits one slot of the connection's FIFO, so the send completes
    // without a posted receive while the peer has fewer than NCCL_STEPS (8)
    // unpopped packets from this rank; past that the send stream stalls
    // until the peer pops -- the credit window of push.cl:21-31.  The
    // ticket's event tells when the staging slot may be reused.
    int send_detached(const void *buf, size_t bytes, int peer, hipStream_t stream, SendTicket *t) override {
        std::lock_guard<std::mutex> lk(chan_mu_);
        SMI_TRY(check(ncclGroupStart(), "ncclGroupStart"));
        SMI_TRY(check(ncclSend(buf, bytes, ncclUint8, peer, chan_, stream), "ncclSend"));
        SMI_TRY(check(ncclGroupEnd(), "ncclGroupEnd"));
        if (!t->ev) SMI_HIP_CHECK(hipEventCreateWithFlags(&t->ev, hipEventDisableTiming));
        SMI_HIP_CHECK(hipEventRecord(t->ev, stream));
        t->live = true;
        return SMI_SUCCESS;
    }
    int ticket_wait(SendTicket *t) override {
        if (!t->live) return SMI_SUCCESS;
        SMI_HIP_CHECK(hipEventSynchronize(t->ev));
        t->live = false;
        return SMI_SUCCESS;
    }
    int recv_now(void *buf, size_t bytes, int peer, hipStream_t stream) override {
        std::lock_guard<std::mutex> lk(chan_mu_);
        SMI_TRY(check(ncclGroupStart(), "ncclGroupStart"));
        SMI_TRY(check(ncclRecv(buf, bytes, ncclUint8, peer, chan_, stream), "ncclRecv"));
        return check(ncclGroupEnd(), "ncclGroupEnd");
    }

    // One byte to and from every peer on the channel communicator: RCCL
    // connects point-to-point peers lazily inside ncclGroupEnd, with a
    // handshake both sides must join; doing it here, collectively, means no
    // later detached send depends on what its peer is doing.
    int connect_all(int rank, int size) {
        if (size == 1) return SMI_SUCCESS;
        char *d = nullptr;
        hipStream_t st = nullptr;
        SMI_HIP_CHECK(hipMalloc(&d, 2 * (size_t)size));
        int rc = hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess ? SMI_SUCCESS : SMI_ERR_HIP;
        if (rc == SMI_SUCCESS) rc = check(ncclGroupStart(), "ncclGroupStart");
        for (int p = 0; p < size && rc == SMI_SUCCESS; ++p) {
            if (p == rank) continue;
            rc = check(ncclSend(d + p, 1, ncclUint8, p, chan_, st), "ncclSend");
            if (rc == SMI_SUCCESS) rc = check(ncclRecv(d + size + p, 1, ncclUint8, p, chan_, st), "ncclRecv");
        }
        if (rc == SMI_SUCCESS) rc = check(ncclGroupEnd(), "ncclGroupEnd");
        if (rc == SMI_SUCCESS && hipStreamSynchronize(st) != hipSuccess) {
            set_error("channel connect: stream synchronize failed");
            rc = SMI_ERR_HIP;
        }
        if (st) hipStreamDestroy(st);
        hipFree(d);
        return rc;
    }

    static int check(ncclResult_t r, const char *what) {
        if (r == ncclSuccess) return SMI_SUCCESS;
        set_error(std::string(what) + ": " + ncclGetErrorString(r));
        return SMI_ERR_COMM;
    }

  private:
    ncclComm_t comm_ = nullptr, chan_ = nullptr;
    hipStream_t stream_ = nullptr;
    std::mutex bulk_mu_, chan_mu_;
};

std::unique_ptr<Transport> make_rccl_transport(int rank, int size,
                                               const void *unique_id,
                                               int id_bytes, int *rc) {
    if (id_bytes < (int)sizeof(ncclUniqueId)) {
        set_error("unique id too short");
        *rc = SMI_ERR_INVALID_ARG;
        return nullptr;
    }
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof(id));
    ncclComm_t comm = nullptr, chan = nullptr;
    *rc = RcclTransport::check(ncclCommInitRank(&comm, size, id, rank), "ncclCommInitRank");
    if (*rc != SMI_SUCCESS) return nullptr;
    *rc = RcclTransport::check(ncclCommSplit(comm, 0, rank, &chan, nullptr), "ncclCommSplit");
    if (*rc != SMI_SUCCESS) {
        ncclCommDestroy(comm);
        return nullptr;
    }
    auto t = std::make_unique<RcclTransport>(comm, chan);
    *rc = t->connect_all(rank, size);
    if (*rc != SMI_SUCCESS) return nullptr;
    return t;
}

// ================================================================ local ==
namespace {

struct Post {
    const void *buf = nullptr;
    size_t bytes = 0;
    hipEvent_t ready = nullptr;  // sender's stream reached the send
    hipEvent_t done = nullptr;   // receiver's copy finished
    bool copied = false;         // `done` has been recorded
    int status = SMI_SUCCESS;
};

struct LocalGroup {
    int size = 0;
    std::mutex mu;
    std::condition_variable cv;
    // (src, dst, space): space 0 = bulk groups, 1 = element-channel packets
    // (send_detached / recv_now), matched FIFO within each space only
    std::map<std::tuple<int, int, int>, std::deque<std::shared_ptr<Post>>> mailbox;
    int joined = 0;
};

std::mutex g_groups_mu;
std::map<int, std::shared_ptr<LocalGroup>> g_groups;
int g_next_group = 1;

std::shared_ptr<LocalGroup> find_group(int id) {
    std::lock_guard<std::mutex> lk(g_groups_mu);
    auto it = g_groups.find(id);
    return it == g_groups.end() ? nullptr : it->second;
}

}  // namespace

int local_group_size(int group_id) {
    auto g = find_group(group_id);
    return g ? g->size : 0;
}

class LocalTransport final : public Transport {
  public:
    LocalTransport(std::shared_ptr<LocalGroup> g, int rank) : g_(std::move(g)), rank_(rank) {}

    // begin() .. end() hold the bulk mutex (see RcclTransport::begin)
    int begin(hipStream_t stream) override {
        bulk_mu_.lock();
        stream_ = stream;
        sends_.clear();
        recvs_.clear();
        return SMI_SUCCESS;
    }
    int send(const void *buf, size_t bytes, int peer) override {
        if (peer < 0 || peer >= g_->size) {
            set_error("send: peer out of range");
            return SMI_ERR_INVALID_ARG;
        }
        sends_.push_back({const_cast<void *>(buf), bytes, peer});
        return SMI_SUCCESS;
    }
    int recv(void *buf, size_t bytes, int peer) override {
        if (peer < 0 || peer >= g_->size) {
            set_error("recv: peer out of range");
            return SMI_ERR_INVALID_ARG;
        }
        recvs_.push_back({buf, bytes, peer});
        return SMI_SUCCESS;
    }

    // Rendezvous: (1) post every send with a `ready` event on our stream;
    // (2) for every receive, wait for the matching post (FIFO per
    // (src, dst) pair, like the reference's per-port FIFO order), make our
    // stream wait on its `ready`, copy, record `done`; (3) make our stream
    // wait for the `done` of each of our sends, so later work may reuse the
    // send buffers.
    int end() override {
        const int rc = end_group();
        bulk_mu_.unlock();
        return rc;
    }
    int end_group() {
        std::vector<std::shared_ptr<Post>> mine;
        for (auto &s : sends_) {
            auto p = std::make_shared<Post>();
            p->buf = s.buf;
            p->bytes = s.bytes;
            SMI_HIP_CHECK(hipEventCreateWithFlags(&p->ready, hipEventDisableTiming));
            SMI_HIP_CHECK(hipEventCreateWithFlags(&p->done, hipEventDisableTiming));
            SMI_HIP_CHECK(hipEventRecord(p->ready, stream_));
            mine.push_back(p);
        }
        {
            std::lock_guard<std::mutex> lk(g_->mu);
            for (size_t i = 0; i < sends_.size(); ++i)
                g_->mailbox[{rank_, sends_[i].peer, 0}].push_back(mine[i]);
        }
        g_->cv.notify_all();

        int rc = SMI_SUCCESS;
        for (auto &r : recvs_) {
            const int st = take(r.buf, r.bytes, r.peer, 0, stream_);
            if (st != SMI_SUCCESS && rc == SMI_SUCCESS) rc = st;
        }
        for (auto &p : mine) {
            {
                std::unique_lock<std::mutex> lk(g_->mu);
                g_->cv.wait(lk, [&] { return p->copied; });
            }
            if (p->status != SMI_SUCCESS && rc == SMI_SUCCESS) {
                set_error("local transport: peer failed to receive");
                rc = p->status;
            }
            SMI_HIP_CHECK(hipStreamWaitEvent(stream_, p->done, 0));
            SMI_TRY(retire(p));
        }
        sends_.clear();
        recvs_.clear();
        return rc;
    }

    // Post the send and return; the peer's receive performs the copy later.
    int send_detached(const void *buf, size_t bytes, int peer, hipStream_t stream, SendTicket *t) override {
        if (peer < 0 || peer >= g_->size) {
            set_error("send: peer out of range");
            return SMI_ERR_INVALID_ARG;
        }
        auto p = std::make_shared<Post>();
        p->buf = buf;
        p->bytes = bytes;
        SMI_HIP_CHECK(hipEventCreateWithFlags(&p->ready, hipEventDisableTiming));
        SMI_HIP_CHECK(hipEventCreateWithFlags(&p->done, hipEventDisableTiming));
        SMI_HIP_CHECK(hipEventRecord(p->ready, stream));
        {
            std::lock_guard<std::mutex> lk(g_->mu);
            g_->mailbox[{rank_, peer, 1}].push_back(p);
        }
        g_->cv.notify_all();
        t->impl = p;
        t->live = true;
        return SMI_SUCCESS;
    }
    int recv_now(void *buf, size_t bytes, int peer, hipStream_t stream) override {
        if (peer < 0 || peer >= g_->size) {
            set_error("recv: peer out of range");
            return SMI_ERR_INVALID_ARG;
        }
        return take(buf, bytes, peer, 1, stream);
    }
    int ticket_wait(SendTicket *t) override {
        if (!t->live) return SMI_SUCCESS;
        auto p = std::static_pointer_cast<Post>(t->impl);
        {
            std::unique_lock<std::mutex> lk(g_->mu);
            g_->cv.wait(lk, [&] { return p->copied; });
        }
        t->live = false;
        t->impl.reset();
        int st = p->status;
        SMI_HIP_CHECK(hipEventSynchronize(p->done));
        SMI_TRY(retire(p));
        if (st != SMI_SUCCESS) set_error("local transport: peer failed to receive");
        return st;
    }

    ~LocalTransport() override {
        // finalize has synchronised the device: no queue references them now
        for (auto e : retired_) hipEventDestroy(e);
    }

  private:
    // A post's events may still be referenced by barrier packets that another
    // rank's stream has not processed yet, so they are destroyed only after a
    // device-wide synchronisation (at teardown, or when many have piled up).
    int retire(const std::shared_ptr<Post> &p) {
        std::lock_guard<std::mutex> lk(retire_mu_);
        retired_.push_back(p->ready);
        retired_.push_back(p->done);
        if (retired_.size() >= 8192) {
            SMI_HIP_CHECK(hipDeviceSynchronize());
            for (auto e : retired_) SMI_HIP_CHECK(hipEventDestroy(e));
            retired_.clear();
        }
        return SMI_SUCCESS;
    }
    std::mutex retire_mu_;
    std::vector<hipEvent_t> retired_;

    // Wait for the next post from `peer` (FIFO per (src, dst), like the
    // reference's per-port FIFO order), order `stream` after the sender's
    // `ready` event, copy, and mark the post consumed.
    int take(void *buf, size_t bytes, int peer, int space, hipStream_t stream) {
        std::shared_ptr<Post> p;
        {
            std::unique_lock<std::mutex> lk(g_->mu);
            auto &q = g_->mailbox[{peer, rank_, space}];
            g_->cv.wait(lk, [&] { return !q.empty(); });
            p = q.front();
            q.pop_front();
        }
        int st = SMI_SUCCESS;
        if (p->bytes != bytes) {
            set_error("local transport: send/recv size mismatch");
            st = SMI_ERR_COMM;
        } else if (hipStreamWaitEvent(stream, p->ready, 0) != hipSuccess ||
                   (bytes && hipMemcpyAsync(buf, p->buf, bytes, hipMemcpyDeviceToDevice, stream) != hipSuccess)) {
            set_error("local transport: HIP copy failed");
            st = SMI_ERR_HIP;
        }
        if (hipEventRecord(p->done, stream) != hipSuccess && st == SMI_SUCCESS) st = SMI_ERR_HIP;
        {
            std::lock_guard<std::mutex> lk(g_->mu);
            p->status = st;
            p->copied = true;
        }
        g_->cv.notify_all();
        return st;
    }

    struct Op {
        void *buf;
        size_t bytes;
        int peer;
    };
    std::shared_ptr<LocalGroup> g_;
    int rank_;
    std::mutex bulk_mu_;
    hipStream_t stream_ = nullptr;
    std::vector<Op> sends_, recvs_;
};

std::unique_ptr<Transport> make_local_transport(int group_id, int rank, int *rc) {
    auto g = find_group(group_id);
    if (!g) {
        set_error("unknown local group");
        *rc = SMI_ERR_BAD_COMM;
        return nullptr;
    }
    if (rank < 0 || rank >= g->size) {
        set_error("rank out of range for local group");
        *rc = SMI_ERR_INVALID_ARG;
        return nullptr;
    }
    *rc = SMI_SUCCESS;
    return std::make_unique<LocalTransport>(g, rank);
}

}  // namespace smi

extern "C" {

int smi_get_unique_id(void *id, int id_bytes) {
    using namespace smi;
    SMI_ARG_CHECK(id && id_bytes >= (int)sizeof(ncclUniqueId), "unique id buffer too small");
    ncclUniqueId u;
    SMI_TRY(RcclTransport::check(ncclGetUniqueId(&u), "ncclGetUniqueId"));
    memcpy(id, &u, sizeof(u));
    return SMI_SUCCESS;
}

int smi_local_group_create(int size, int *group_id) {
    using namespace smi;
    SMI_ARG_CHECK(group_id && size >= 1, "size/group_id");
    auto g = std::make_shared<LocalGroup>();
    g->size = size;
    std::lock_guard<std::mutex> lk(g_groups_mu);
    int id = g_next_group++;
    g_groups[id] = g;
    *group_id = id;
    return SMI_SUCCESS;
}

}  // extern "C"
