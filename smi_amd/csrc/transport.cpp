// transport.cpp -- the two point-to-point transports behind the channels.
//
// The reference moves 32-byte packets through CK_S/CK_R kernels and QSFP
// links chosen by routing tables (codegen/templates/cks.cl:3-84, ckr.cl:
// 3-88); on one MI355X node every GPU pair is a direct xGMI link, so a
// transfer is a plain RCCL send/recv between the two ranks.
//
//  * RcclTransport  -- production: one process per GPU, RCCL over xGMI.
//  * LocalTransport -- ranks are host threads of one process sharing one
//    device; a group's transfers are one copy kernel that reads the sender's
//    buffer directly, ordered by HIP events without a system-scope fence
//    (both valid only on one device: smi_init_local refuses a second one).
//    It exists so that multi-rank parity tests can run on a single GPU (RCCL
//    refuses two ranks on one device).
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstring>
#include <deque>
#include <algorithm>
#include <map>
#include <mutex>
#include <tuple>
#include <type_traits>

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
    RcclTransport(ncclComm_t c, ncclComm_t chan, int rank, int size)
        : comm_(c), chan_(chan), rank_(rank), size_(size) {}
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
    // Collective: every peer blocks in this handshake until this rank joins
    // it, so a local failure must not skip it.  If the device buffer or the
    // stream cannot be had, the handshake still runs -- from pinned host
    // memory / on the null stream -- and the error is returned after it, on
    // this rank only; the peers complete their init and see the failure at
    // their first operation with this rank instead of hanging here.
    int connect_all(int rank, int size) {
        if (size == 1) return SMI_SUCCESS;
        char *d = nullptr, *h = nullptr;
        hipStream_t st = nullptr;
        int local = SMI_SUCCESS;
        if (hipMalloc(&d, 2 * (size_t)size) != hipSuccess) {
            d = nullptr;
            local = SMI_ERR_HIP;
            set_error("channel connect: hipMalloc failed");
            if (hipHostMalloc(&h, 2 * (size_t)size, hipHostMallocMapped) != hipSuccess) h = nullptr;
        }
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
            st = nullptr;  // the null stream carries the handshake instead
            local = SMI_ERR_HIP;
            set_error("channel connect: stream creation failed");
        }
        char *buf = d ? d : h;
        int rc = buf ? check(ncclGroupStart(), "ncclGroupStart") : SMI_ERR_HIP;
        for (int p = 0; p < size && rc == SMI_SUCCESS; ++p) {
            if (p == rank) continue;
            rc = check(ncclSend(buf + p, 1, ncclUint8, p, chan_, st), "ncclSend");
            if (rc == SMI_SUCCESS) rc = check(ncclRecv(buf + size + p, 1, ncclUint8, p, chan_, st), "ncclRecv");
        }
        if (buf && rc != SMI_ERR_HIP) {
            const int e = check(ncclGroupEnd(), "ncclGroupEnd");  // close the group on every path
            if (rc == SMI_SUCCESS) rc = e;
        }
        if (rc == SMI_SUCCESS && hipStreamSynchronize(st) != hipSuccess) {
            set_error("channel connect: stream synchronize failed");
            rc = SMI_ERR_HIP;
        }
        if (st) (void)hipStreamDestroy(st);
        if (d) (void)hipFree(d);
        if (h) (void)hipHostFree(h);
        return rc != SMI_SUCCESS ? rc : local;
    }

    // Both communicators split again (color 0, same rank order): RCCL
    // matches the new pair's operations separately from this pair's.
    std::unique_ptr<Transport> dup(int *rc) override {
        // chan_ carries the element channels (send_detached / recv_now take
        // chan_mu_ from any host thread): no channel traffic may run on it
        // while it is split, so both locks are held
        std::scoped_lock lk(bulk_mu_, chan_mu_);
        ncclComm_t c2 = nullptr, ch2 = nullptr;
        *rc = check(ncclCommSplit(comm_, 0, rank_, &c2, nullptr), "ncclCommSplit");
        if (*rc != SMI_SUCCESS) return nullptr;
        *rc = check(ncclCommSplit(chan_, 0, rank_, &ch2, nullptr), "ncclCommSplit");
        if (*rc != SMI_SUCCESS) {
            ncclCommDestroy(c2);
            return nullptr;
        }
        auto t = std::make_unique<RcclTransport>(c2, ch2, rank_, size_);
        *rc = t->connect_all(rank_, size_);
        if (*rc != SMI_SUCCESS) return nullptr;
        return t;
    }

    static int check(ncclResult_t r, const char *what) {
        if (r == ncclSuccess) return SMI_SUCCESS;
        set_error(std::string(what) + ": " + ncclGetErrorString(r));
        return SMI_ERR_COMM;
    }

  private:
    ncclComm_t comm_ = nullptr, chan_ = nullptr;
    int rank_ = 0, size_ = 1;
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
    auto t = std::make_unique<RcclTransport>(comm, chan, rank, size);
    *rc = t->connect_all(rank, size);
    if (*rc != SMI_SUCCESS) return nullptr;
    return t;
}

// ================================================================ local ==
namespace {

// Events of the in-process transport come from a pool owned by the group, so
// that an event recorded by one rank outlives that rank's transport while
// another rank may still wait on it (a detached send's `done` is recorded by
// the receiver and waited for by the sender when it finalizes).  A handle
// returns its event to the pool when the last Post holding it is gone, i.e.
// once every wait on it has been enqueued (a wait captures the event's
// current record, so re-recording it afterwards is safe).
struct EventPool {
    std::mutex mu;
    std::vector<hipEvent_t> free;
    ~EventPool() {
        for (auto e : free) (void)hipEventDestroy(e);
    }
};
using Ev = std::shared_ptr<std::remove_pointer<hipEvent_t>::type>;

int pooled_event(const std::shared_ptr<EventPool> &pool, Ev *out) {
    hipEvent_t e = nullptr;
    {
        std::lock_guard<std::mutex> lk(pool->mu);
        if (!pool->free.empty()) {
            e = pool->free.back();
            pool->free.pop_back();
        }
    }
    // ordering between the ranks' streams on the device (no host reads device
    // data behind them): no system-scope release at the record
    if (!e) SMI_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
    *out = Ev(e, [pool](hipEvent_t x) {
        std::lock_guard<std::mutex> lk(pool->mu);
        pool->free.push_back(x);
    });
    return SMI_SUCCESS;
}

struct Post {
    const void *buf = nullptr;
    size_t bytes = 0;
    Ev ready;                    // sender's stream reached the send (one per sender group)
    Ev done;                     // receiver's copy finished (recorded by the receiver)
    bool copied = false;         // `done` has been recorded
    int status = SMI_SUCCESS;
};

struct LocalGroup {
    std::shared_ptr<EventPool> events = std::make_shared<EventPool>();
    int size = 0;
    std::mutex mu;
    std::condition_variable cv;
    // (src, dst, space): space 0 = bulk groups, 1 = element-channel packets
    // (send_detached / recv_now), matched FIFO within each space only
    std::map<std::tuple<int, int, int>, std::deque<std::shared_ptr<Post>>> mailbox;
    int device = -1;  // the one device every rank of the group runs on
    int joined = 0;   // transports created for it (its ranks)
    int live = 0;     // transports not yet destroyed
    std::map<int, int> dups;  // k-th smi_comm_dup of this group -> its group id
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
    LocalTransport(std::shared_ptr<LocalGroup> g, int rank, int id) : g_(std::move(g)), rank_(rank), id_(id) {
        std::lock_guard<std::mutex> lk(g_->mu);
        ++g_->joined;
        ++g_->live;
    }
    ~LocalTransport() override {
        // The rank whose transport goes last in a fully joined group drops
        // the registry's reference too, so the group -- and the events of its
        // pool -- go with this transport (finalize, HIP alive), not at
        // process exit.  Counted under the group's mutex: ranks finalizing on
        // their threads at the same time see distinct counts.  (g_->mu is
        // released before g_groups_mu is taken: dup() nests them the other
        // way round.)
        bool last = false;
        {
            std::lock_guard<std::mutex> lk(g_->mu);
            last = --g_->live == 0 && g_->joined >= g_->size;
        }
        if (last) {
            std::lock_guard<std::mutex> lk(g_groups_mu);
            auto it = g_groups.find(id_);
            if (it != g_groups.end() && it->second == g_) g_groups.erase(it);
        }
    }

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

    // Rendezvous, with a constant number of host calls per group (an
    // interior rank's K-step exchange is 8 sends + 8 receives per pass; one
    // copy + two events per message cost more host time than the pass):
    // (1) post every send, all sharing one `ready` event recorded on our
    // stream; (2) take the matching post of every receive (FIFO per (src,
    // dst) pair, like the reference's per-port FIFO order), make our stream
    // wait on each distinct `ready`, copy them all with one kernel, record
    // one `done`; (3) make our stream wait for the `done` of each receiver of
    // our sends, so later work may reuse the send buffers.
    int end() override {
        const int rc = end_group();
        bulk_mu_.unlock();
        return rc;
    }
    int end_group() {
        std::vector<std::shared_ptr<Post>> mine;
        Ev ready;
        if (!sends_.empty()) {
            SMI_TRY(pooled_event(g_->events, &ready));
            SMI_HIP_CHECK(hipEventRecord(ready.get(), stream_));
        }
        for (auto &sd : sends_) {
            auto p = std::make_shared<Post>();
            p->buf = sd.buf;
            p->bytes = sd.bytes;
            p->ready = ready;
            mine.push_back(p);
        }
        if (!mine.empty()) {
            {
                std::lock_guard<std::mutex> lk(g_->mu);
                for (size_t i = 0; i < sends_.size(); ++i) g_->mailbox[{rank_, sends_[i].peer, 0}].push_back(mine[i]);
            }
            g_->cv.notify_all();
        }

        int rc = SMI_SUCCESS;
        if (!recvs_.empty()) {
            std::vector<std::shared_ptr<Post>> got;
            std::vector<const void *> src;
            std::vector<void *> dst;
            std::vector<size_t> by;
            for (auto &r : recvs_) {
                auto p = next_post(r.peer, 0);
                if (p->bytes != r.bytes) {
                    set_error("local transport: send/recv size mismatch");
                    p->status = SMI_ERR_COMM;
                    if (rc == SMI_SUCCESS) rc = SMI_ERR_COMM;
                } else {
                    src.push_back(p->buf);
                    dst.push_back(r.buf);
                    by.push_back(r.bytes);
                }
                got.push_back(p);
            }
            std::vector<hipEvent_t> waited;
            int st = SMI_SUCCESS;
            for (auto &p : got)
                if (p->status == SMI_SUCCESS &&
                    std::find(waited.begin(), waited.end(), p->ready.get()) == waited.end()) {
                    waited.push_back(p->ready.get());
                    if (hipStreamWaitEvent(stream_, p->ready.get(), 0) != hipSuccess) st = SMI_ERR_HIP;
                }
            if (st == SMI_SUCCESS) st = launch_copies(src.data(), dst.data(), by.data(), (int)src.size(), stream_);
            Ev done;
            if (pooled_event(g_->events, &done) != SMI_SUCCESS || hipEventRecord(done.get(), stream_) != hipSuccess)
                st = SMI_ERR_HIP;
            if (st != SMI_SUCCESS) {
                set_error("local transport: HIP copy failed");
                if (rc == SMI_SUCCESS) rc = st;
            }
            {
                std::lock_guard<std::mutex> lk(g_->mu);
                for (auto &p : got) {
                    p->done = done;
                    if (p->status == SMI_SUCCESS) p->status = st;
                    p->copied = true;
                }
            }
            g_->cv.notify_all();
        }

        std::vector<hipEvent_t> joined;
        for (auto &p : mine) {
            {
                std::unique_lock<std::mutex> lk(g_->mu);
                g_->cv.wait(lk, [&] { return p->copied; });
            }
            if (p->status != SMI_SUCCESS && rc == SMI_SUCCESS) {
                set_error("local transport: peer failed to receive");
                rc = p->status;
            }
            if (p->done && std::find(joined.begin(), joined.end(), p->done.get()) == joined.end()) {
                joined.push_back(p->done.get());
                SMI_HIP_CHECK(hipStreamWaitEvent(stream_, p->done.get(), 0));
            }
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
        SMI_TRY(pooled_event(g_->events, &p->ready));
        SMI_HIP_CHECK(hipEventRecord(p->ready.get(), stream));
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
        auto p = next_post(peer, 1);
        int st = SMI_SUCCESS;
        if (p->bytes != bytes) {
            set_error("local transport: send/recv size mismatch");
            st = SMI_ERR_COMM;
        } else if (hipStreamWaitEvent(stream, p->ready.get(), 0) != hipSuccess ||
                   (bytes && hipMemcpyAsync(buf, p->buf, bytes, hipMemcpyDeviceToDevice, stream) != hipSuccess)) {
            set_error("local transport: HIP copy failed");
            st = SMI_ERR_HIP;
        }
        Ev done;
        if (pooled_event(g_->events, &done) != SMI_SUCCESS || hipEventRecord(done.get(), stream) != hipSuccess) {
            if (st == SMI_SUCCESS) st = SMI_ERR_HIP;
        }
        {
            std::lock_guard<std::mutex> lk(g_->mu);
            p->done = done;
            p->status = st;
            p->copied = true;
        }
        g_->cv.notify_all();
        return st;
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
        // the Post holds `done`: it cannot have been recycled yet
        if (p->done) SMI_HIP_CHECK(hipEventSynchronize(p->done.get()));
        if (st != SMI_SUCCESS) set_error("local transport: peer failed to receive");
        return st;
    }

    // The k-th dup of every rank of a group lands in one new group (created
    // by whichever rank gets there first).
    std::unique_ptr<Transport> dup(int *rc) override;

    // the next post from `peer` in `space` (FIFO per (src, dst, space))
    std::shared_ptr<Post> next_post(int peer, int space) {
        std::unique_lock<std::mutex> lk(g_->mu);
        auto &q = g_->mailbox[{peer, rank_, space}];
        g_->cv.wait(lk, [&] { return !q.empty(); });
        auto p = q.front();
        q.pop_front();
        return p;
    }

    struct Op {
        void *buf;
        size_t bytes;
        int peer;
    };
    std::shared_ptr<LocalGroup> g_;
    int rank_;
    int id_;
    int ndup_ = 0;
    std::mutex bulk_mu_;
    hipStream_t stream_ = nullptr;
    std::vector<Op> sends_, recvs_;
};

std::unique_ptr<Transport> LocalTransport::dup(int *rc) {
    const int k = ++ndup_;
    int id = 0;
    {
        std::lock_guard<std::mutex> lk(g_->mu);
        auto it = g_->dups.find(k);
        if (it != g_->dups.end()) {
            id = it->second;
        } else {
            auto ng = std::make_shared<LocalGroup>();
            ng->size = g_->size;
            std::lock_guard<std::mutex> lk2(g_groups_mu);
            id = g_next_group++;
            g_groups[id] = ng;
            g_->dups[k] = id;
        }
    }
    int dev = 0;
    {
        std::lock_guard<std::mutex> lk(g_->mu);
        dev = g_->device;
    }
    return make_local_transport(id, rank_, dev, rc);
}

std::unique_ptr<Transport> make_local_transport(int group_id, int rank, int device, int *rc) {
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
    {
        // one device per group: the copy kernel reads the sender's buffer
        // and the ordering events skip the system-scope fence
        std::lock_guard<std::mutex> lk(g->mu);
        if (g->device < 0) g->device = device;
        if (g->device != device) {
            set_error("in-process group: every rank must use the group's device (" + std::to_string(g->device) + ")");
            *rc = SMI_ERR_INVALID_ARG;
            return nullptr;
        }
    }
    *rc = SMI_SUCCESS;
    return std::make_unique<LocalTransport>(g, rank, group_id);
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
