// channels.cpp -- element-granular transient channels (host-callable).
//
// Reference replaced (ryutakashino/SMI, codegen/templates/):
//   push.cl:3-70 / pop.cl:3-83        SMI_Push / SMI_Pop, 28-byte packets,
//                                     credit-based flow control
//   bcast.cl:3-149                    SMI_Bcast, root fan-out of packets
//   reduce.cl:184-245                 SMI_Reduce, one element per packet
//   scatter.cl:3-164 / gather.cl:3-162
// Elements are packed into fixed-size messages (16-byte header + 16,368-byte
// payload) that travel over the communicator's transport (RCCL over xGMI,
// or the in-process device-copy transport).  Every message is tagged with its
// port, and a per-communicator inbox demultiplexes them, so channels on
// different ports between the same pair of ranks keep separate FIFOs like the
// reference's per-port channels.  Sends are detached through a ring of 32
// staging slots -- the counterpart of the reference's credit window -- so a
// rank may push before its peer pops.  Element reduce folds each element's
// contributions on the root with fold.h's fold_one, the same source as the
// device fold kernel of smi_reduce.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <unordered_map>

#include "fold.h"
#include "smi_internal.h"

namespace smi {
namespace {

// A message costs about the same host and transport time at 2 KiB and at
// 16 KiB (a host-to-device copy, the transport, a device-to-host copy and a
// synchronisation on the receiver); 16 KiB streams 8x the elements per
// message (profiles/r06/p2p/: element bandwidth 0.15 Gbit/s at 2 KiB).
constexpr size_t kMsgBytes = 16384;
constexpr size_t kHdrBytes = 16;
constexpr size_t kPayload = kMsgBytes - kHdrBytes;
constexpr int kSlots = 32;

enum Kind { K_P2P = 1, K_BCAST = 2, K_REDUCE = 3, K_SCATTER = 4, K_GATHER = 5 };

struct MsgHeader {
    int32_t port, nelems, kind, src;
};

struct Msg {
    int kind = 0;
    int nelems = 0;
    std::vector<char> payload;
};

struct ChanEngine {
    int device = 0;
    hipStream_t send_stream = nullptr, recv_stream = nullptr;
    char *host_slots = nullptr, *dev_slots = nullptr;   // kSlots x kMsgBytes
    char *host_rslot = nullptr, *dev_rslot = nullptr;   // one receive message
    std::vector<char> red_row;                          // element-reduce contributions (64 ranks x 8 B)
    SendTicket tickets[kSlots];
    int next_slot = 0;
    std::mutex send_mu, recv_mu, red_mu;
    std::map<std::pair<int, int>, std::deque<Msg>> inbox;  // (src, port)

    ~ChanEngine() {
        hipSetDevice(device);
        if (send_stream) hipStreamSynchronize(send_stream);
        if (recv_stream) hipStreamSynchronize(recv_stream);
        for (auto &t : tickets)
            if (t.ev) hipEventDestroy(t.ev);
        if (host_slots) hipHostFree(host_slots);
        if (host_rslot) hipHostFree(host_rslot);
        if (dev_slots) hipFree(dev_slots);
        if (dev_rslot) hipFree(dev_rslot);
        if (send_stream) hipStreamDestroy(send_stream);
        if (recv_stream) hipStreamDestroy(recv_stream);
    }
};

std::mutex g_engine_mu;

int get_engine(Comm *c, ChanEngine **out) {
    std::lock_guard<std::mutex> lk(g_engine_mu);
    if (!c->chan_engine) {
        auto e = std::make_shared<ChanEngine>();
        e->device = c->device;
        SMI_HIP_CHECK(hipSetDevice(c->device));
        SMI_HIP_CHECK(hipStreamCreateWithFlags(&e->send_stream, hipStreamNonBlocking));
        SMI_HIP_CHECK(hipStreamCreateWithFlags(&e->recv_stream, hipStreamNonBlocking));
        SMI_HIP_CHECK(hipHostMalloc(&e->host_slots, kSlots * kMsgBytes));
        SMI_HIP_CHECK(hipHostMalloc(&e->host_rslot, kMsgBytes));
        e->red_row.resize(64 * 8);
        SMI_HIP_CHECK(hipMalloc(&e->dev_slots, kSlots * kMsgBytes));
        SMI_HIP_CHECK(hipMalloc(&e->dev_rslot, kMsgBytes));
        c->chan_engine = e;
    }
    *out = static_cast<ChanEngine *>(c->chan_engine.get());
    return SMI_SUCCESS;
}

int send_msg(Comm *c, ChanEngine *e, int peer, int port, int kind, const char *payload, int nelems, size_t esz) {
    std::lock_guard<std::mutex> lk(e->send_mu);
    const int slot = e->next_slot;
    e->next_slot = (e->next_slot + 1) % kSlots;
    SMI_TRY(c->transport->ticket_wait(&e->tickets[slot]));  // slot free again
    char *h = e->host_slots + (size_t)slot * kMsgBytes;
    char *d = e->dev_slots + (size_t)slot * kMsgBytes;
    MsgHeader hdr{port, nelems, kind, c->rank};
    memcpy(h, &hdr, sizeof(hdr));
    memcpy(h + kHdrBytes, payload, (size_t)nelems * esz);
    SMI_HIP_CHECK(hipSetDevice(c->device));
    // only the header and the elements cross to the device; the transport
    // moves the whole fixed-size message (the tail is never read)
    SMI_HIP_CHECK(hipMemcpyAsync(d, h, kHdrBytes + (size_t)nelems * esz, hipMemcpyHostToDevice, e->send_stream));
    return c->transport->send_detached(d, kMsgBytes, peer, e->send_stream, &e->tickets[slot]);
}

// Next message from (src, port); messages for other ports of the same source
// are parked in the inbox.
int recv_msg(Comm *c, ChanEngine *e, int src, int port, int kind, Msg *out) {
    std::lock_guard<std::mutex> lk(e->recv_mu);
    auto key = std::make_pair(src, port);
    while (e->inbox[key].empty()) {
        SMI_HIP_CHECK(hipSetDevice(c->device));
        SMI_TRY(c->transport->recv_now(e->dev_rslot, kMsgBytes, src, e->recv_stream));
        SMI_HIP_CHECK(hipMemcpyAsync(e->host_rslot, e->dev_rslot, kMsgBytes, hipMemcpyDeviceToHost, e->recv_stream));
        SMI_HIP_CHECK(hipStreamSynchronize(e->recv_stream));
        MsgHeader hdr;
        memcpy(&hdr, e->host_rslot, sizeof(hdr));
        if (hdr.src != src || hdr.nelems < 0 || (size_t)hdr.nelems > kPayload) {
            set_error("channel: corrupt message");
            return SMI_ERR_COMM;
        }
        Msg m;
        m.kind = hdr.kind;
        m.nelems = hdr.nelems;
        // elements are at most 8 bytes (type_size): keep what the header covers
        m.payload.assign(e->host_rslot + kHdrBytes,
                         e->host_rslot + kHdrBytes + std::min(kPayload, (size_t)hdr.nelems * 8));
        e->inbox[{src, hdr.port}].push_back(std::move(m));
    }
    Msg &m = e->inbox[key].front();
    if (m.kind != kind) {
        set_error("channel: operation mismatch on port " + std::to_string(port));
        return SMI_ERR_COMM;
    }
    *out = std::move(m);
    e->inbox[key].pop_front();
    return SMI_SUCCESS;
}

// ------------------------------------------------------- channel state --
struct ChanState {
    Comm *comm = nullptr;
    ChanEngine *eng = nullptr;
    int kind = 0;
    bool sender = false;      // p2p: push side
    int type = 0;
    size_t esz = 0;
    int per_msg = 0;          // elements per message
    int port = 0, peer = 0;   // peer: destination / source / root
    int op = 0;
    long count = 0;           // elements per (rank, peer) stream
    long recv_count = 0;
    // packing (send side)
    std::vector<char> pkt;
    int fill = 0;
    long sent = 0;            // elements sent in the current segment
    // unpacking (receive side), per source rank (indexed, no lookup per element)
    std::vector<Msg> cur;
    std::vector<int> pos;
    // scatter / gather progress
    int next = 0;
    long seg = 0;
};

std::mutex g_chan_mu;
std::unordered_map<int, std::unique_ptr<ChanState>> g_chans;
int g_next_chan = 1;

template <typename D>
D open_desc(int kind, int count, int type, int peer, int port, SMI_Comm comm, int op, int recv_count) {
    D d{};
    d.status = SMI_SUCCESS;
    d.my_rank = comm.rank;
    d.num_ranks = comm.size;
    d.peer = peer;
    d.port = port;
    d.data_type = (SMI_Datatype)type;
    d.message_size = count < 0 ? 0u : (unsigned)count;
    d.processed_elements = 0;
    Comm *c = lookup_comm(comm);
    const size_t esz = type_size(type);
    if (!c) {
        set_error("unknown communicator");
        d.status = SMI_ERR_BAD_COMM;
        return d;
    }
    if (esz == 0 || count < 0 || peer < 0 || peer >= c->size) {
        set_error("channel: bad type, count or rank");
        d.status = esz == 0 ? SMI_ERR_UNSUPPORTED : SMI_ERR_INVALID_ARG;
        return d;
    }
    auto st = std::make_unique<ChanState>();
    st->comm = c;
    if ((d.status = get_engine(c, &st->eng)) != SMI_SUCCESS) return d;
    st->kind = kind;
    st->type = type;
    st->esz = esz;
    st->per_msg = (int)(kPayload / esz);
    st->port = port;
    st->peer = peer;
    st->op = op;
    st->count = count;
    st->recv_count = recv_count;
    st->pkt.resize(kPayload);
    st->cur.resize(c->size);
    st->pos.assign(c->size, 0);
    std::lock_guard<std::mutex> lk(g_chan_mu);
    d.handle = g_next_chan++;
    g_chans[d.handle] = std::move(st);
    return d;
}

// Every element call looks its channel up.  A thread keeps its last lookup
// and reuses it until any channel closes (the epoch moves under g_chan_mu):
// a run of pushes or pops on one channel takes no lock.  Handles are never
// reused.  A descriptor is used by one thread at a time, as its
// processed_elements count already requires.
std::atomic<unsigned> g_chan_epoch{0};
struct ChanCache {
    int handle = 0;
    unsigned epoch = ~0u;
    ChanState *s = nullptr;
};
thread_local ChanCache t_chan_cache;

ChanState *state(int handle) {
    ChanCache &cc = t_chan_cache;
    if (cc.handle == handle && cc.epoch == g_chan_epoch.load(std::memory_order_acquire)) return cc.s;
    std::lock_guard<std::mutex> lk(g_chan_mu);
    auto it = g_chans.find(handle);
    ChanState *s = it == g_chans.end() ? nullptr : it->second.get();
    cc = ChanCache{handle, g_chan_epoch.load(std::memory_order_relaxed), s};
    return s;
}

void close_chan(int *handle) {
    std::lock_guard<std::mutex> lk(g_chan_mu);
    g_chans.erase(*handle);
    g_chan_epoch.fetch_add(1, std::memory_order_release);
    *handle = 0;
}

int flush(ChanState *s, int dst) {
    if (s->fill == 0) return SMI_SUCCESS;
    const int n = s->fill;
    s->fill = 0;
    return send_msg(s->comm, s->eng, dst, s->port, s->kind, s->pkt.data(), n, s->esz);
}

int append(ChanState *s, const void *data) {
    memcpy(s->pkt.data() + (size_t)s->fill * s->esz, data, s->esz);
    ++s->fill;
    return SMI_SUCCESS;
}

// Next element from `src` (unpacking its current message).
int take(ChanState *s, int src, void *data) {
    int &p = s->pos[src];
    Msg &m = s->cur[src];
    if (p >= m.nelems) {
        SMI_TRY(recv_msg(s->comm, s->eng, src, s->port, s->kind, &m));
        p = 0;
        if (m.nelems == 0) {
            set_error("channel: empty message");
            return SMI_ERR_COMM;
        }
    }
    memcpy(data, m.payload.data() + (size_t)p * s->esz, s->esz);
    ++p;
    return SMI_SUCCESS;
}

// asynch_degree (the `_ad` open variants): the reference sizes the channel's
// FIFO in elements with it (codegen/rewrite.py:26-35), i.e. how far a pusher
// runs ahead of the wire.  Here it bounds the elements a sender packs before
// the message leaves (at most one payload); receivers unpack whatever message
// sizes arrive, so the two ends need not agree and the data never changes.
template <typename D>
D with_asynch_degree(D d, int asynch_degree) {
    if (d.handle && asynch_degree > 0) {
        ChanState *s = nullptr;
        {
            std::lock_guard<std::mutex> lk(g_chan_mu);
            auto it = g_chans.find(d.handle);
            if (it != g_chans.end()) s = it->second.get();
        }
        if (s) s->per_msg = std::min(s->per_msg, asynch_degree);
    }
    return d;
}

template <typename D>
ChanState *begin_call(D *chan) {
    if (!chan) return nullptr;
    if (chan->handle == 0) {
        if (chan->status == SMI_SUCCESS) {
            set_error("channel already completed (transient channels end after their count)");
            chan->status = SMI_ERR_INVALID_ARG;
        }
        return nullptr;
    }
    ChanState *s = state(chan->handle);
    if (!s) chan->status = SMI_ERR_INVALID_ARG;
    return s;
}

}  // namespace

template <typename T, int S>
int fold_element_t(const void *row, void *out, int n, int op) {
    T v;
    switch (op) {
    case SMI_ADD: v = fold_one<T, S, SMI_ADD>((const T *)row, n); break;
    case SMI_MAX: v = fold_one<T, S, SMI_MAX>((const T *)row, n); break;
    case SMI_MIN: v = fold_one<T, S, SMI_MIN>((const T *)row, n); break;
    default: set_error("unsupported reduce op"); return SMI_ERR_UNSUPPORTED;
    }
    memcpy(out, &v, sizeof(T));
    return SMI_SUCCESS;
}

// one element of n contributions (row[k] = rank k's), SHIFT_REG per type
// (codegen/ops.py:110-116)
int fold_element(const void *row, void *out, int n, int type, int op) {
    switch (type) {
    case SMI_FLOAT: return fold_element_t<float, 4>(row, out, n, op);
    case SMI_DOUBLE: return fold_element_t<double, 4>(row, out, n, op);
    case SMI_INT: return fold_element_t<int32_t, 1>(row, out, n, op);
    case SMI_SHORT: return fold_element_t<int16_t, 1>(row, out, n, op);
    case SMI_CHAR: return fold_element_t<int8_t, 1>(row, out, n, op);
    default: set_error("unsupported data type"); return SMI_ERR_UNSUPPORTED;
    }
}

// The last packets of a channel are detached sends: their staging slots must
// outlive them, so finalize waits until the peers have received them.
int channels_drain(Comm *c) {
    if (!c->chan_engine) return SMI_SUCCESS;
    auto *e = static_cast<ChanEngine *>(c->chan_engine.get());
    std::lock_guard<std::mutex> lk(e->send_mu);
    int rc = SMI_SUCCESS;
    for (auto &t : e->tickets) {
        const int r = c->transport->ticket_wait(&t);
        if (rc == SMI_SUCCESS) rc = r;
    }
    return rc;
}

}  // namespace smi

using namespace smi;

extern "C" {

// ------------------------------------------------------------------ p2p --
SMI_Channel SMI_Open_send_channel(int count, SMI_Datatype data_type, int destination, int port, SMI_Comm comm) {
    SMI_Channel d = open_desc<SMI_Channel>(K_P2P, count, data_type, destination, port, comm, 0, count);
    if (d.handle) state(d.handle)->sender = true;
    return d;
}
SMI_Channel SMI_Open_send_channel_ad(int count, SMI_Datatype data_type, int destination, int port, SMI_Comm comm,
                                     int asynch_degree) {
    return with_asynch_degree(SMI_Open_send_channel(count, data_type, destination, port, comm), asynch_degree);
}
SMI_Channel SMI_Open_receive_channel(int count, SMI_Datatype data_type, int source, int port, SMI_Comm comm) {
    return open_desc<SMI_Channel>(K_P2P, count, data_type, source, port, comm, 0, count);
}
SMI_Channel SMI_Open_receive_channel_ad(int count, SMI_Datatype data_type, int source, int port, SMI_Comm comm,
                                        int asynch_degree) {
    return with_asynch_degree(SMI_Open_receive_channel(count, data_type, source, port, comm), asynch_degree);
}

void SMI_Push_flush(SMI_Channel *chan, void *data, int immediate) {
    ChanState *s = begin_call(chan);
    if (!s) return;
    if (!s->sender) {
        set_error("SMI_Push on a receive channel");
        chan->status = SMI_ERR_INVALID_ARG;
        return;
    }
    append(s, data);
    ++chan->processed_elements;
    int rc = SMI_SUCCESS;
    if (s->fill == s->per_msg || immediate || chan->processed_elements == chan->message_size)
        rc = flush(s, s->peer);
    chan->status = rc;
    if (chan->processed_elements == chan->message_size) close_chan(&chan->handle);
}

void SMI_Push(SMI_Channel *chan, void *data) { SMI_Push_flush(chan, data, 0); }

void SMI_Pop(SMI_Channel *chan, void *data) {
    ChanState *s = begin_call(chan);
    if (!s) return;
    if (s->sender) {
        set_error("SMI_Pop on a send channel");
        chan->status = SMI_ERR_INVALID_ARG;
        return;
    }
    chan->status = take(s, s->peer, data);
    ++chan->processed_elements;
    if (chan->processed_elements == chan->message_size) close_chan(&chan->handle);
}

// ---------------------------------------------------------------- bcast --
SMI_BChannel SMI_Open_bcast_channel(int count, SMI_Datatype data_type, int port, int root, SMI_Comm comm) {
    return open_desc<SMI_BChannel>(K_BCAST, count, data_type, root, port, comm, 0, count);
}
SMI_BChannel SMI_Open_bcast_channel_ad(int count, SMI_Datatype data_type, int port, int root, SMI_Comm comm,
                                       int asynch_degree) {
    return with_asynch_degree(SMI_Open_bcast_channel(count, data_type, port, root, comm), asynch_degree);
}

void SMI_Bcast(SMI_BChannel *chan, void *data) {
    ChanState *s = begin_call(chan);
    if (!s) return;
    int rc = SMI_SUCCESS;
    ++chan->processed_elements;
    const bool last = chan->processed_elements == chan->message_size;
    if (chan->my_rank == s->peer) {  // root: pack, fan the packet out
        append(s, data);
        if (s->fill == s->per_msg || last) {
            const int n = s->fill;
            s->fill = 0;
            for (int k = 0; k < chan->num_ranks && rc == SMI_SUCCESS; ++k)
                if (k != s->peer)
                    rc = send_msg(s->comm, s->eng, k, s->port, s->kind, s->pkt.data(), n, s->esz);
        }
    } else {
        rc = take(s, s->peer, data);
    }
    chan->status = rc;
    if (last) close_chan(&chan->handle);
}

// --------------------------------------------------------------- reduce --
SMI_RChannel SMI_Open_reduce_channel(int count, SMI_Datatype data_type, SMI_Op op, int port, int root,
                                     SMI_Comm comm) {
    SMI_RChannel d = open_desc<SMI_RChannel>(K_REDUCE, count, data_type, root, port, comm, op, count);
    d.reduce_op = op;
    if (d.handle && (op < SMI_ADD || op > SMI_MIN)) {
        close_chan(&d.handle);
        d.status = SMI_ERR_UNSUPPORTED;
    }
    return d;
}
SMI_RChannel SMI_Open_reduce_channel_ad(int count, SMI_Datatype data_type, SMI_Op op, int port, int root,
                                        SMI_Comm comm, int asynch_degree) {
    return with_asynch_degree(SMI_Open_reduce_channel(count, data_type, op, port, root, comm), asynch_degree);
}

void SMI_Reduce(SMI_RChannel *chan, void *data_snd, void *data_rcv) {
    ChanState *s = begin_call(chan);
    if (!s) return;
    int rc = SMI_SUCCESS;
    ++chan->processed_elements;
    const bool last = chan->processed_elements == chan->message_size;
    const int n = chan->num_ranks, root = s->peer;
    if (chan->my_rank != root) {  // contributors stream their elements to the root
        append(s, data_snd);
        if (s->fill == s->per_msg || last) rc = flush(s, root);
    } else {
        // root: the element of every rank in rank order (the packets the
        // contributors streamed ahead are already unpacked host-side), folded
        // by the support kernel's fold (fold.h, reduce.cl:65-69,100-105,
        // 120-125) as they complete -- no device round trip per element (the
        // previous per-element fold launch + sync ran at 47 k elements/s)
        ChanEngine *e = s->eng;
        std::lock_guard<std::mutex> lk(e->red_mu);
        char *row = e->red_row.data();
        for (int k = 0; k < n && rc == SMI_SUCCESS; ++k) {
            if (k == root) memcpy(row + (size_t)k * s->esz, data_snd, s->esz);
            else rc = take(s, k, row + (size_t)k * s->esz);
        }
        if (rc == SMI_SUCCESS) rc = fold_element(row, data_rcv, n, s->type, s->op);
    }
    chan->status = rc;
    if (last) close_chan(&chan->handle);
}

// -------------------------------------------------------------- scatter --
SMI_ScatterChannel SMI_Open_scatter_channel(int send_count, int recv_count, SMI_Datatype data_type, int port,
                                            int root, SMI_Comm comm) {
    // root: send_count per rank for num_ranks ranks; others: recv_count
    const int mine = comm.rank == root ? send_count * comm.size : recv_count;
    SMI_ScatterChannel d =
        open_desc<SMI_ScatterChannel>(K_SCATTER, mine, data_type, root, port, comm, 0, recv_count);
    d.recv_count = (unsigned)recv_count;
    if (d.handle) state(d.handle)->count = send_count;
    return d;
}
SMI_ScatterChannel SMI_Open_scatter_channel_ad(int send_count, int recv_count, SMI_Datatype data_type, int port,
                                               int root, SMI_Comm comm, int asynch_degree) {
    return with_asynch_degree(SMI_Open_scatter_channel(send_count, recv_count, data_type, port, root, comm),
                              asynch_degree);
}

void SMI_Scatter(SMI_ScatterChannel *chan, void *data_snd, void *data_rcv) {
    ChanState *s = begin_call(chan);
    if (!s) return;
    int rc = SMI_SUCCESS;
    ++chan->processed_elements;
    const bool last = chan->processed_elements == chan->message_size;
    if (chan->my_rank == s->peer) {  // root: segment for rank `next`
        if (s->next == chan->my_rank) {
            memcpy(data_rcv, data_snd, s->esz);
        } else {
            append(s, data_snd);
        }
        ++s->seg;
        const bool seg_done = s->seg == s->count;
        if (s->next != chan->my_rank && (s->fill == s->per_msg || seg_done)) rc = flush(s, s->next);
        if (seg_done) {
            s->seg = 0;
            ++s->next;
        }
    } else {
        rc = take(s, s->peer, data_rcv);
    }
    chan->status = rc;
    if (last) close_chan(&chan->handle);
}

// --------------------------------------------------------------- gather --
SMI_GatherChannel SMI_Open_gather_channel(int send_count, int recv_count, SMI_Datatype data_type, int port,
                                          int root, SMI_Comm comm) {
    const int mine = comm.rank == root ? recv_count * comm.size : send_count;
    SMI_GatherChannel d = open_desc<SMI_GatherChannel>(K_GATHER, mine, data_type, root, port, comm, 0, recv_count);
    d.recv_count = (unsigned)recv_count;
    if (d.handle) state(d.handle)->count = recv_count;
    return d;
}
SMI_GatherChannel SMI_Open_gather_channel_ad(int send_count, int recv_count, SMI_Datatype data_type, int port,
                                             int root, SMI_Comm comm, int asynch_degree) {
    return with_asynch_degree(SMI_Open_gather_channel(send_count, recv_count, data_type, port, root, comm),
                              asynch_degree);
}

void SMI_Gather(SMI_GatherChannel *chan, void *send_data, void *rcv_data) {
    ChanState *s = begin_call(chan);
    if (!s) return;
    int rc = SMI_SUCCESS;
    ++chan->processed_elements;
    const bool last = chan->processed_elements == chan->message_size;
    if (chan->my_rank == s->peer) {  // root: contributor `next`'s segment
        if (s->next == chan->my_rank) memcpy(rcv_data, send_data, s->esz);
        else rc = take(s, s->next, rcv_data);
        if (++s->seg == s->count) {
            s->seg = 0;
            ++s->next;
        }
    } else {
        append(s, send_data);
        if (s->fill == s->per_msg || last) rc = flush(s, s->peer);
    }
    chan->status = rc;
    if (last) close_chan(&chan->handle);
}

// ----------------------------------------------- bulk scatter / gather --
int smi_scatter(SMI_Comm comm, const void *sendbuf, void *recvbuf, size_t count, SMI_Datatype type, int root,
                int port, SMI_Stream stream) {
    (void)port;
    Comm *c = lookup_comm(comm);
    if (!c) {
        set_error("unknown communicator");
        return SMI_ERR_BAD_COMM;
    }
    const size_t esz = type_size(type);
    if (esz == 0) {
        set_error("unsupported data type");
        return SMI_ERR_UNSUPPORTED;
    }
    SMI_ARG_CHECK(root >= 0 && root < c->size, "root out of range");
    if (count == 0) return SMI_SUCCESS;
    SMI_ARG_CHECK(recvbuf && (c->rank != root || sendbuf), "NULL buffer");
    hipStream_t s = (hipStream_t)stream;
    const size_t bytes = count * esz;
    if (c->rank == root)
        SMI_HIP_CHECK(hipMemcpyAsync(recvbuf, (const char *)sendbuf + (size_t)root * bytes, bytes,
                                     hipMemcpyDeviceToDevice, s));
    if (c->size == 1) return SMI_SUCCESS;
    Transport *tp = c->transport.get();
    Group grp(tp);
    SMI_TRY(grp.begin(s));
    if (c->rank == root) {
        for (int k = 0; k < c->size; ++k)
            if (k != root) SMI_TRY(tp->send((const char *)sendbuf + (size_t)k * bytes, bytes, k));
    } else {
        SMI_TRY(tp->recv(recvbuf, bytes, root));
    }
    return grp.end();
}

// Bulk point-to-point on device buffers, stream-ordered: the GPU-native form
// of a transient channel that carries `count` elements from one rank to
// another (push.h / pop.h; the reference's bandwidth microbenchmark streams
// N elements through SMI_Push/SMI_Pop, microbenchmarks/kernels/
// bandwidth_0.cl:13-35, bandwidth_1.cl:12-44).  One transport message (an
// RCCL send/recv over xGMI, or a device copy in-process).  Messages between
// a pair of ranks are matched in the order they are issued, whatever their
// port (RCCL keeps one FIFO per pair), so a port here is informational.
static int p2p_check(Comm *c, size_t esz, int peer) {
    if (esz == 0) {
        set_error("unsupported data type");
        return SMI_ERR_UNSUPPORTED;
    }
    SMI_ARG_CHECK(peer >= 0 && peer < c->size, "peer rank out of range");
    SMI_ARG_CHECK(peer != c->rank, "point-to-point to self");
    return SMI_SUCCESS;
}

int smi_gather(SMI_Comm comm, const void *sendbuf, void *recvbuf, size_t count, SMI_Datatype type, int root,
               int port, SMI_Stream stream) {
    (void)port;
    Comm *c = lookup_comm(comm);
    if (!c) {
        set_error("unknown communicator");
        return SMI_ERR_BAD_COMM;
    }
    const size_t esz = type_size(type);
    if (esz == 0) {
        set_error("unsupported data type");
        return SMI_ERR_UNSUPPORTED;
    }
    SMI_ARG_CHECK(root >= 0 && root < c->size, "root out of range");
    if (count == 0) return SMI_SUCCESS;
    SMI_ARG_CHECK(sendbuf && (c->rank != root || recvbuf), "NULL buffer");
    hipStream_t s = (hipStream_t)stream;
    const size_t bytes = count * esz;
    if (c->rank == root)
        SMI_HIP_CHECK(hipMemcpyAsync((char *)recvbuf + (size_t)root * bytes, sendbuf, bytes,
                                     hipMemcpyDeviceToDevice, s));
    if (c->size == 1) return SMI_SUCCESS;
    Transport *tp = c->transport.get();
    Group grp(tp);
    SMI_TRY(grp.begin(s));
    if (c->rank == root) {
        for (int k = 0; k < c->size; ++k)
            if (k != root) SMI_TRY(tp->recv((char *)recvbuf + (size_t)k * bytes, bytes, k));
    } else {
        SMI_TRY(tp->send(sendbuf, bytes, root));
    }
    return grp.end();
}


int smi_send(SMI_Comm comm, const void *buf, size_t count, SMI_Datatype type, int destination, int port,
             SMI_Stream stream) {
    (void)port;
    Comm *c = lookup_comm(comm);
    if (!c) {
        set_error("unknown communicator");
        return SMI_ERR_BAD_COMM;
    }
    const size_t esz = type_size(type);
    SMI_TRY(p2p_check(c, esz, destination));
    if (count == 0) return SMI_SUCCESS;
    SMI_ARG_CHECK(buf, "NULL buffer");
    Transport *tp = c->transport.get();
    Group grp(tp);
    SMI_TRY(grp.begin((hipStream_t)stream));
    SMI_TRY(tp->send(buf, count * esz, destination));
    return grp.end();
}

int smi_recv(SMI_Comm comm, void *buf, size_t count, SMI_Datatype type, int source, int port, SMI_Stream stream) {
    (void)port;
    Comm *c = lookup_comm(comm);
    if (!c) {
        set_error("unknown communicator");
        return SMI_ERR_BAD_COMM;
    }
    const size_t esz = type_size(type);
    SMI_TRY(p2p_check(c, esz, source));
    if (count == 0) return SMI_SUCCESS;
    SMI_ARG_CHECK(buf, "NULL buffer");
    Transport *tp = c->transport.get();
    Group grp(tp);
    SMI_TRY(grp.begin((hipStream_t)stream));
    SMI_TRY(tp->recv(buf, count * esz, source));
    return grp.end();
}

}  // extern "C"
