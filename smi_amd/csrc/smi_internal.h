// smi_internal.h -- shared internals of libsmi_amd.so (not installed).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "smi.h"

namespace smi {

// ---------------------------------------------------------------- errors --
void set_error(const std::string &msg);

#define SMI_HIP_CHECK(expr)                                                    \
    do {                                                                       \
        hipError_t _e = (expr);                                                \
        if (_e != hipSuccess) {                                                \
            ::smi::set_error(std::string(#expr) + ": " + hipGetErrorString(_e) \
                             + " (" + __FILE__ + ":" + std::to_string(__LINE__) \
                             + ")");                                           \
            return SMI_ERR_HIP;                                                \
        }                                                                      \
    } while (0)

#define SMI_ARG_CHECK(cond, msg)                                               \
    do {                                                                       \
        if (!(cond)) {                                                         \
            ::smi::set_error(std::string("invalid argument: ") + (msg));       \
            return SMI_ERR_INVALID_ARG;                                        \
        }                                                                      \
    } while (0)

#define SMI_TRY(expr)                                                          \
    do {                                                                       \
        int _rc = (expr);                                                      \
        if (_rc != SMI_SUCCESS) return _rc;                                    \
    } while (0)

// ------------------------------------------------------------- transport --
// Point-to-point byte transport between the ranks of one communicator.
// Usage mirrors an RCCL group: begin(stream); send/recv ...; end().  All ops
// of a group are ordered after the work already queued on `stream`, and work
// queued on `stream` after end() observes every receive of the group and may
// overwrite every send buffer of the group.
// A detached send (used by the element-granular channels) returns at once;
// the ticket completes when the bytes have left the send buffer, so the
// sender can keep pushing while the receiver has not popped yet -- the
// buffering the reference gets from its credit window (push.cl:21-31).
struct SendTicket {
    std::shared_ptr<void> impl;
    hipEvent_t ev = nullptr;
    bool live = false;
};

class Transport {
  public:
    virtual ~Transport() = default;
    virtual int begin(hipStream_t stream) = 0;
    virtual int send(const void *buf, size_t bytes, int peer) = 0;
    virtual int recv(void *buf, size_t bytes, int peer) = 0;
    virtual int end() = 0;
    virtual int send_detached(const void *buf, size_t bytes, int peer, hipStream_t stream, SendTicket *t) = 0;
    virtual int ticket_wait(SendTicket *t) = 0;
    // One receive, enqueued on `stream` (the caller synchronises).  Like
    // send_detached, safe to call from several host threads at once.
    virtual int recv_now(void *buf, size_t bytes, int peer, hipStream_t stream) = 0;
    // A new transport over the same ranks with matching spaces of its own
    // (smi_comm_dup).  Collective: every rank dups its transports in the same
    // order.
    virtual std::unique_ptr<Transport> dup(int *rc) = 0;
};

// One transport group, closed on every path: begin() takes the transport's
// bulk lock (two host threads never interleave groups on one communicator)
// and end() -- or the destructor, on an early error return -- releases it.
class Group {
  public:
    explicit Group(Transport *t) : t_(t) {}
    Group(const Group &) = delete;
    Group &operator=(const Group &) = delete;
    int begin(hipStream_t s) {
        const int rc = t_->begin(s);
        open_ = rc == SMI_SUCCESS;
        return rc;
    }
    int end() {
        open_ = false;
        return t_->end();
    }
    ~Group() {
        if (open_) t_->end();
    }

  private:
    Transport *t_;
    bool open_ = false;
};

std::unique_ptr<Transport> make_rccl_transport(int rank, int size,
                                               const void *unique_id,
                                               int id_bytes, int *rc);
// device: the rank's device; every rank of a group must use the same one
std::unique_ptr<Transport> make_local_transport(int group_id, int rank, int device,
                                                int *rc);
int local_group_size(int group_id);

// ------------------------------------------------------------ communicator --
struct Comm {
    int rank = 0;
    int size = 1;
    int device = 0;
    std::unique_ptr<Transport> transport;
    hipStream_t comm_stream = nullptr;  // dedicated halo / collective stream
    // the multi-rank stencil's interior stream when the caller's stream is not
    // at the highest priority (stencil_run.cpp interior_stream), made on demand
    hipStream_t interior_stream = nullptr;
    // device workspace (grown on demand, never shrunk)
    void *work = nullptr;
    size_t work_bytes = 0;
    // halo staging for the stencil: [top, bottom, left, right] in + send L/R
    float *halo = nullptr;
    size_t halo_elems = 0;
    std::vector<hipEvent_t> events;  // reusable sync events
    std::shared_ptr<void> chan_engine;  // element-granular channels (channels.cpp)
};

Comm *lookup_comm(SMI_Comm c);
int comm_workspace(Comm *c, size_t bytes, void **ptr);
int comm_event(Comm *c, int idx, hipEvent_t *ev);

// Wait until every detached channel send of `c` has been received (finalize).
int channels_drain(Comm *c);

// ------------------------------------------------------------ profiling --
bool prof_enabled();
// Bracket one launch: call before (returns a token) and after the launch.
// tag distinguishes variants of one kernel (the K of a K-step sweep); units
// is the launch's algorithmic work (cell-steps for the stencil kernels).
int prof_begin(int kernel, hipStream_t stream, int *token, int tag = 0, double units = 0.0, bool chain = false);
int prof_end(int token, hipStream_t stream);
void prof_break_chain();
// A record timed by the launch's own dispatch: pass *start / *stop to
// hipExtLaunchKernelGGL (no marker packets around the kernel).
int prof_launch(int kernel, int *token, int tag, double units, hipEvent_t *start, hipEvent_t *stop);

size_t type_size(int type);

// Device-to-device copies in one kernel launch (copy.hip); segments that are
// not 16-byte aligned multiples go through hipMemcpyAsync.
int launch_copies(const void *const *src, void *const *dst, const size_t *bytes, int n, hipStream_t s);
#ifdef SMI_LOOPBACK_REHEARSAL
int launch_heavy_copies(const void *const *src, void *const *dst, const size_t *bytes, int n, int blocks,
                        hipStream_t s);
#endif

}  // namespace smi
