// collectives.hip -- SMI_Reduce and SMI_Bcast on whole device buffers.
//
// Reference replaced (ryutakashino/SMI):
//   SMI_Reduce + smi_kernel_reduce_<p>   codegen/templates/reduce.cl:3-245
//     root-gathering reduce, one element per 32-B packet, 16-deep credit
//     window, per-slot rotating fold (SHIFT_REG, codegen/ops.py:110-141)
//   SMI_Bcast + smi_kernel_bcast_<p>     codegen/templates/bcast.cl:3-149
//     root packs 7 elements per packet, linear fan-out to every rank
// MI355X design: on a fully connected xGMI node the root's links are the
// bottleneck of a rooted collective, so both are split over all ranks:
//   reduce = owner-chunk exchange (rank r sends chunk c of its buffer to
//            owner c) -> canonical rank-order fold on each owner (HIP kernel,
//            bit-identical to the reference fold with arrival = rank order)
//            -> owners send their reduced chunk to the root (messages up
//            to 256 KiB: direct fan-in to the root and one fold there);
//   bcast  = scatter of the root's chunks -> all-gather between the ranks
//            (small messages: direct fan-out from the root).
// Every step is a transport group of point-to-point transfers on the
// caller's stream (RCCL over xGMI in production).
#include <algorithm>
#include <cstdlib>

#include "fold.h"
#include "smi_internal.h"

namespace smi {

constexpr int kMaxFoldRanks = 64;

struct FoldRows {
    const void *row[kMaxFoldRanks];
};

// Fold of reduce.cl:65-69,100-105,120-125 (fold.h's fold_one, vectorised):
// contributions in rank order, S slots (4 for float/double, 1 for the
// integer types).
// Each thread folds E = VPT*VEC consecutive elements, loaded as VPT 16-byte
// vectors per contribution row.  The rows are streamed exactly once, so the
// default launch uses nontemporal loads/stores and one E-group per thread.
template <typename T, int S, int OP, bool NT, int VPT>
__global__ __launch_bounds__(256) void fold_kernel(FoldRows rows, T *__restrict__ out, int n,
                                                   size_t count, int vec_ok) {
    using V4 = unsigned __attribute__((ext_vector_type(4)));
    constexpr int VEC = 16 / sizeof(T);
    constexpr int E = VEC * VPT;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < (count + E - 1) / E; v += stride) {
        const size_t base = v * E;
        const bool full = vec_ok && base + E <= count;
        T q[E][S];
#pragma unroll
        for (int e = 0; e < E; ++e)
#pragma unroll
            for (int j = 0; j < S; ++j) q[e][j] = op_init<T, OP>();
        // contributions in batches of KB: all loads of a batch are in flight
        // before the (strictly ordered) fold consumes them
        constexpr int KB = 8;
        for (int k0 = 0; k0 < n; k0 += KB) {
            T d[KB][E];
#pragma unroll
            for (int i = 0; i < KB; ++i) {
                const int k = min(k0 + i, n - 1);  // past n: a valid row, never folded
                const T *src = (const T *)rows.row[k] + base;
                if (full) {
#pragma unroll
                    for (int u = 0; u < VPT; ++u) {
                        const V4 *p = reinterpret_cast<const V4 *>(src) + u;
                        if constexpr (NT)  // streamed once: do not keep the rows in L2
                            *reinterpret_cast<V4 *>(&d[i][u * VEC]) = __builtin_nontemporal_load(p);
                        else
                            *reinterpret_cast<V4 *>(&d[i][u * VEC]) = *p;
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < E; ++e) {  // clamped index: safe if the load is speculated
                        const T v = src[base + e < count ? e : (count - 1 - base)];
                        d[i][e] = (base + e < count) ? v : T(0);
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < KB; ++i) {
                if (k0 + i >= n) break;  // uniform
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const T nv = op_apply<T, OP>(d[i][e], q[e][0]);
#pragma unroll
                    for (int j = 0; j < S - 1; ++j) q[e][j] = q[e][j + 1];
                    q[e][S - 1] = nv;
                }
            }
        }
        T r[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            T res = op_init<T, OP>();
#pragma unroll
            for (int j = 0; j < S; ++j) res = op_apply<T, OP>(res, q[e][j]);
            r[e] = res;
        }
        if (full) {
#pragma unroll
            for (int u = 0; u < VPT; ++u) {
                const V4 w = *reinterpret_cast<const V4 *>(&r[u * VEC]);
                V4 *p = reinterpret_cast<V4 *>(out + base) + u;
                if constexpr (NT)
                    __builtin_nontemporal_store(w, p);
                else
                    *p = w;
            }
        } else {
#pragma unroll
            for (int e = 0; e < E; ++e)
                if (base + e < count) out[base + e] = r[e];
        }
    }
}

// Launch variant, SMI_FOLD_VARIANT (experiment build only; the library: 0, the
// tuned default): bit 0 = cached loads/stores instead of nontemporal, bit 1 = grid
// capped at 4096 blocks (grid-stride loop), bit 2 = two vectors per thread.
// 8 x 64 Mi fp32 on one MI355X: cached+capped 4.56 TB/s, default 5.75 TB/s.
static int fold_variant() {
#ifdef SMI_EXPERIMENTS  // experiment build only (smi_amd/build.py --experiments)
    static int v = [] {
        const char *e = getenv("SMI_FOLD_VARIANT");
        return e ? atoi(e) : 0;
    }();
    return v;
#else
    return 0;
#endif
}

template <typename T, int S, int OP, int VPT>
static void launch_fold_v(const FoldRows &rows, void *out, int n, size_t count, int vec_ok, int var,
                          hipStream_t s) {
    constexpr int E = VPT * 16 / (int)sizeof(T);
    const size_t work = (count + E - 1) / E;
    const size_t cap = (var & 2) ? 4096 : (size_t)1 << 30;
    const int blocks = (int)std::max<size_t>(1, std::min<size_t>((work + 255) / 256, cap));
    if (var & 1)
        hipLaunchKernelGGL((fold_kernel<T, S, OP, false, VPT>), dim3(blocks), dim3(256), 0, s, rows, (T *)out,
                           n, count, vec_ok);
    else
        hipLaunchKernelGGL((fold_kernel<T, S, OP, true, VPT>), dim3(blocks), dim3(256), 0, s, rows, (T *)out,
                           n, count, vec_ok);
}

template <typename T, int S, int OP>
static void launch_fold_t(const FoldRows &rows, void *out, int n, size_t count, int vec_ok,
                          hipStream_t s) {
    const int var = fold_variant();
    if (var & 4) launch_fold_v<T, S, OP, 2>(rows, out, n, count, vec_ok, var, s);
    else launch_fold_v<T, S, OP, 1>(rows, out, n, count, vec_ok, var, s);
}

template <typename T, int S>
static int launch_fold_op(const FoldRows &rows, void *out, int n, size_t count, int vec_ok, int op,
                          hipStream_t s) {
    switch (op) {
    case SMI_ADD: launch_fold_t<T, S, SMI_ADD>(rows, out, n, count, vec_ok, s); break;
    case SMI_MAX: launch_fold_t<T, S, SMI_MAX>(rows, out, n, count, vec_ok, s); break;
    case SMI_MIN: launch_fold_t<T, S, SMI_MIN>(rows, out, n, count, vec_ok, s); break;
    default: set_error("unsupported reduce op"); return SMI_ERR_UNSUPPORTED;
    }
    return SMI_SUCCESS;
}

static int launch_fold(const FoldRows &rows, void *out, int n, size_t count, int type, int op,
                       hipStream_t s) {
    SMI_ARG_CHECK(n >= 1 && n <= kMaxFoldRanks, "fold supports 1..64 contributions");
    if (count == 0) return SMI_SUCCESS;
    int vec_ok = ((uintptr_t)out & 15u) == 0;
    for (int k = 0; k < n; ++k) vec_ok &= ((uintptr_t)rows.row[k] & 15u) == 0;
    int tok = -1;
    if (prof_enabled()) SMI_TRY(prof_begin(SMI_PROF_REDUCE_FOLD, s, &tok));
    int rc;
    switch (type) {  // SHIFT_REG: codegen/ops.py:110-116
    case SMI_FLOAT: rc = launch_fold_op<float, 4>(rows, out, n, count, vec_ok, op, s); break;
    case SMI_DOUBLE: rc = launch_fold_op<double, 4>(rows, out, n, count, vec_ok, op, s); break;
    case SMI_INT: rc = launch_fold_op<int32_t, 1>(rows, out, n, count, vec_ok, op, s); break;
    case SMI_SHORT: rc = launch_fold_op<int16_t, 1>(rows, out, n, count, vec_ok, op, s); break;
    case SMI_CHAR: rc = launch_fold_op<int8_t, 1>(rows, out, n, count, vec_ok, op, s); break;
    default: set_error("unsupported data type"); return SMI_ERR_UNSUPPORTED;
    }
    SMI_TRY(rc);
    SMI_HIP_CHECK(hipGetLastError());
    if (tok >= 0) SMI_TRY(prof_end(tok, s));
    return SMI_SUCCESS;
}

// Owner chunk c covers elements [c*cs, min((c+1)*cs, count)); cs is a
// multiple of 16 bytes so every chunk of an aligned buffer stays aligned.
static size_t chunk_elems(size_t count, int n, size_t esz) {
    const size_t per16 = 16 / std::min<size_t>(16, esz);
    size_t cs = (count + n - 1) / n;
    cs = (cs + per16 - 1) / per16 * per16;
    return std::max<size_t>(cs, per16);
}
static size_t chunk_len(size_t count, size_t cs, int c) {
    const size_t b = (size_t)c * cs;
    return b >= count ? 0 : std::min(cs, count - b);
}

// Pipelining of smi_reduce / smi_bcast: every owner chunk is cut into n
// pieces of ps elements (a multiple of 16 bytes, so pieces of an aligned
// buffer stay aligned).  g_piece_bytes = 0: one piece (no pipelining).
size_t g_piece_bytes = (size_t)4 << 20;

// smi_reduce messages up to this size take the direct fan-in (as smi_bcast's
// direct fan-out, below): latency, not link bandwidth, bounds them
constexpr size_t kReduceFanInBytes = (size_t)256 * 1024;
struct Pieces {
    size_t ps;  // elements per piece
    int n;      // pieces per chunk
};
static Pieces pieces_of(size_t cs, size_t esz) {
    const size_t per16 = 16 / std::min<size_t>(16, esz);
    size_t want = g_piece_bytes ? std::max<size_t>(g_piece_bytes / esz, 1) : cs;
    want = (want + per16 - 1) / per16 * per16;
    const size_t n = (cs + want - 1) / want;
    size_t ps = (cs + n - 1) / n;  // balanced pieces
    ps = (ps + per16 - 1) / per16 * per16;
    return {ps, (int)((cs + ps - 1) / ps)};
}
static size_t sub_len(size_t len, size_t ps, int i) {
    const size_t b = (size_t)i * ps;
    return b >= len ? 0 : std::min(ps, len - b);
}

}  // namespace smi

using namespace smi;

extern "C" {

int smi_reduce_fold(const void *contribs, void *out, int nranks, size_t count, size_t ld,
                    SMI_Datatype type, SMI_Op op, SMI_Stream stream) {
    SMI_ARG_CHECK(out && (contribs || count == 0), "NULL buffer");
    SMI_ARG_CHECK(nranks >= 1 && nranks <= kMaxFoldRanks, "nranks out of range");
    SMI_ARG_CHECK(ld >= count, "ld < count");
    const size_t esz = type_size(type);
    if (esz == 0) {
        set_error("unsupported data type");
        return SMI_ERR_UNSUPPORTED;
    }
    FoldRows rows{};
    for (int k = 0; k < nranks; ++k) rows.row[k] = (const char *)contribs + (size_t)k * ld * esz;
    return launch_fold(rows, out, nranks, count, type, op, (hipStream_t)stream);
}

int smi_reduce(SMI_Comm comm, const void *sendbuf, void *recvbuf, size_t count, SMI_Datatype type,
               SMI_Op op, int root, int port, SMI_Stream stream_) {
    (void)port;  // ports only order operations in the reference; one stream orders them here
    Comm *c = lookup_comm(comm);
    if (!c) {
        set_error("unknown communicator");
        return SMI_ERR_BAD_COMM;
    }
    const int n = c->size, me = c->rank;
    SMI_ARG_CHECK(root >= 0 && root < n, "root out of range");
    SMI_ARG_CHECK(n <= kMaxFoldRanks, "reduce supports up to 64 ranks");
    SMI_ARG_CHECK(op >= SMI_ADD && op <= SMI_MIN, "bad op");
    const size_t esz = type_size(type);
    if (esz == 0) {
        set_error("unsupported data type");
        return SMI_ERR_UNSUPPORTED;
    }
    if (count == 0) return SMI_SUCCESS;
    SMI_ARG_CHECK(sendbuf, "NULL sendbuf");
    SMI_ARG_CHECK(me != root || recvbuf, "NULL recvbuf on root");
    hipStream_t s = (hipStream_t)stream_;

    if (n == 1) {
        FoldRows rows{};
        rows.row[0] = sendbuf;
        return launch_fold(rows, recvbuf, 1, count, type, op, s);
    }
    if (count * esz <= kReduceFanInBytes) {
        // Latency-bound: a direct fan-in, all on the caller's stream -- every
        // rank's whole buffer to the root in one transport group, then one
        // canonical rank-order fold there: one round instead of the owner
        // chunks' two (exchange, then gather), and the same fold over the
        // same rows, so the same bits.
        if (me != root) {
            Group grp(c->transport.get());
            SMI_TRY(grp.begin(s));
            SMI_TRY(c->transport->send(sendbuf, count * esz, root));
            return grp.end();
        }
        const size_t rst = (count * esz + 15) / 16 * 16;  // staging row stride (16-byte aligned rows)
        void *ws = nullptr;
        SMI_TRY(comm_workspace(c, (size_t)n * rst, &ws));
        FoldRows rows{};
        Group grp(c->transport.get());
        SMI_TRY(grp.begin(s));
        for (int k = 0; k < n; ++k) {
            rows.row[k] = k == me ? sendbuf : (const void *)((char *)ws + (size_t)k * rst);
            if (k != me) SMI_TRY(c->transport->recv((char *)ws + (size_t)k * rst, count * esz, k));
        }
        SMI_TRY(grp.end());
        return launch_fold(rows, recvbuf, n, count, type, op, s);
    }
    const size_t cs = chunk_elems(count, n, esz);
    const Pieces pc = pieces_of(cs, esz);
    // workspace: two exchange slots of n staging rows, plus the reduced
    // chunk of a non-root owner (cs elements).  Rows sit kStagePad bytes
    // further apart than a piece: with power-of-two row strides the fold's
    // n concurrent row streams collide in the same HBM channels (8 x 64 Mi
    // fp32 fold: 0.72 of HBM peak at a 256 MiB row stride, 0.80 with 4 KiB
    // more, profiles/r02/fold_stride.jsonl).
    constexpr size_t kStagePad = 4096;
    const size_t pst = pc.ps + kStagePad / esz;  // staging row stride in elements
    void *ws = nullptr;
    SMI_TRY(comm_workspace(c, (2 * (size_t)n * pst + cs) * esz, &ws));
    char *stage = (char *)ws;
    char *mine = stage + 2 * (size_t)n * pst * esz;
    const char *sb = (const char *)sendbuf;
    char *dst = (me == root) ? (char *)recvbuf + (size_t)me * cs * esz : mine;
    Transport *tp = c->transport.get();
    hipStream_t cs_ = c->comm_stream;
    auto slot = [&](int i, int k) { return stage + ((size_t)(i & 1) * n + k) * pst * esz; };
    auto sub = [&](int owner, int i) { return sub_len(chunk_len(count, cs, owner), pc.ps, i); };

    // Pipelined over P pieces (every owner chunk split into P sub-chunks of
    // ps elements), three stages on two streams:
    //   comm stream: X(0), X(1), [wait F(0)] {G(0) + X(2)}, [wait F(1)] {G(1) + X(3)} ...
    //   main stream: [wait X(i)] F(i)
    // X(i) = owner-chunk exchange of piece i (my sub-chunk i of chunk k ->
    // owner k) into staging slot i mod 2; F(i) = canonical rank-order fold of
    // my sub-chunk i (reduce.cl:65-125 with arrival = rank order); G(i) =
    // the folded piece to the root.  The fold of piece i overlaps the
    // exchange of piece i+1 (the reference streams its reduce element by
    // element under a credit window, reduce.cl:13-24,130-179); slot i mod 2
    // is rewritten by X(i+2) only after F(i), which that group waits for.
    hipEvent_t ev_s, ev_f, ev_x[3];
    SMI_TRY(comm_event(c, 2, &ev_s));
    SMI_TRY(comm_event(c, 3, &ev_f));
    for (int k = 0; k < 3; ++k) SMI_TRY(comm_event(c, 4 + k, &ev_x[k]));
    SMI_HIP_CHECK(hipEventRecord(ev_s, s));  // sendbuf is ready on the caller's stream
    SMI_HIP_CHECK(hipStreamWaitEvent(cs_, ev_s, 0));
    auto group = [&](int xi, int gi) -> int {  // {X(xi)} + {G(gi)}, either may be -1
        Group grp(tp);
        SMI_TRY(grp.begin(cs_));
        if (xi >= 0)
            for (int k = 0; k < n; ++k) {
                if (k == me) continue;
                SMI_TRY(tp->send(sb + ((size_t)k * cs + (size_t)xi * pc.ps) * esz, sub(k, xi) * esz, k));
                SMI_TRY(tp->recv(slot(xi, k), sub(me, xi) * esz, k));
            }
        if (gi >= 0) {
            const size_t off = (size_t)gi * pc.ps;
            if (me == root) {
                for (int k = 0; k < n; ++k)
                    if (k != root)
                        SMI_TRY(tp->recv((char *)recvbuf + ((size_t)k * cs + off) * esz, sub(k, gi) * esz, k));
            } else {
                SMI_TRY(tp->send(mine + off * esz, sub(me, gi) * esz, root));
            }
        }
        SMI_TRY(grp.end());
        if (xi >= 0) SMI_HIP_CHECK(hipEventRecord(ev_x[xi % 3], cs_));
        return SMI_SUCCESS;
    };
    SMI_TRY(group(0, -1));
    if (pc.n > 1) SMI_TRY(group(1, -1));
    for (int i = 0; i < pc.n; ++i) {
        SMI_HIP_CHECK(hipStreamWaitEvent(s, ev_x[i % 3], 0));
        const size_t len = sub(me, i);
        if (len) {
            FoldRows rows{};
            for (int k = 0; k < n; ++k)
                rows.row[k] = (k == me) ? (const void *)(sb + ((size_t)me * cs + (size_t)i * pc.ps) * esz)
                                        : (const void *)slot(i, k);
            SMI_TRY(launch_fold(rows, dst + (size_t)i * pc.ps * esz, n, len, type, op, s));
        }
        SMI_HIP_CHECK(hipEventRecord(ev_f, s));
        SMI_HIP_CHECK(hipStreamWaitEvent(cs_, ev_f, 0));
        SMI_TRY(group(i + 2 < pc.n ? i + 2 : -1, i));
    }
    // the caller's stream owns the result
    SMI_HIP_CHECK(hipEventRecord(ev_s, cs_));
    SMI_HIP_CHECK(hipStreamWaitEvent(s, ev_s, 0));
    return SMI_SUCCESS;
}

int smi_bcast(SMI_Comm comm, void *buf, size_t count, SMI_Datatype type, int root, int port,
              SMI_Stream stream_) {
    (void)port;
    Comm *c = lookup_comm(comm);
    if (!c) {
        set_error("unknown communicator");
        return SMI_ERR_BAD_COMM;
    }
    const int n = c->size, me = c->rank;
    SMI_ARG_CHECK(root >= 0 && root < n, "root out of range");
    const size_t esz = type_size(type);
    if (esz == 0) {
        set_error("unsupported data type");
        return SMI_ERR_UNSUPPORTED;
    }
    if (count == 0 || n == 1) return SMI_SUCCESS;
    SMI_ARG_CHECK(buf, "NULL buffer");
    hipStream_t s = (hipStream_t)stream_;
    Transport *tp = c->transport.get();
    char *b = (char *)buf;
    const size_t bytes = count * esz;

    if (bytes <= (size_t)256 * 1024 || n == 2) {  // latency-bound: direct fan-out
        Group grp(tp);
        SMI_TRY(grp.begin(s));
        if (me == root) {
            for (int k = 0; k < n; ++k)
                if (k != root) SMI_TRY(tp->send(b, bytes, k));
        } else {
            SMI_TRY(tp->recv(b, bytes, root));
        }
        return grp.end();
    }
    // Scatter + all-gather, pipelined over P pieces: group i carries the
    // scatter of piece i (the root's sub-chunk i of chunk k -> rank k, into
    // its own position) and the all-gather of piece i-1 (every rank's
    // sub-chunk to every other rank; the root only sends), so the root's
    // links scatter while the others exchange -- the reference streams its
    // broadcast packet by packet (bcast.cl:3-48).
    const size_t cs = chunk_elems(count, n, esz);
    const Pieces pc = pieces_of(cs, esz);
    auto sub = [&](int owner, int i) { return sub_len(chunk_len(count, cs, owner), pc.ps, i); };
    auto at = [&](int owner, int i) { return b + ((size_t)owner * cs + (size_t)i * pc.ps) * esz; };
    for (int i = 0; i <= pc.n; ++i) {
        Group grp(tp);
        SMI_TRY(grp.begin(s));
        if (i < pc.n) {  // scatter of piece i
            if (me == root) {
                for (int k = 0; k < n; ++k)
                    if (k != root) SMI_TRY(tp->send(at(k, i), sub(k, i) * esz, k));
            } else {
                SMI_TRY(tp->recv(at(me, i), sub(me, i) * esz, root));
            }
        }
        if (i > 0) {  // all-gather of piece i-1
            const int g = i - 1;
            for (int k = 0; k < n; ++k) {
                if (k == me) continue;
                if (k != root) SMI_TRY(tp->send(at(me, g), sub(me, g) * esz, k));
                if (me != root) SMI_TRY(tp->recv(at(k, g), sub(k, g) * esz, k));
            }
        }
        SMI_TRY(grp.end());
    }
    return SMI_SUCCESS;
}

int smi_set_pipeline_bytes(size_t piece_bytes) {
    SMI_ARG_CHECK(piece_bytes == 0 || piece_bytes >= 16, "piece_bytes must be 0 (no pipelining) or >= 16");
    g_piece_bytes = piece_bytes;
    return SMI_SUCCESS;
}

int smi_get_pipeline_bytes(size_t *piece_bytes) {
    SMI_ARG_CHECK(piece_bytes, "NULL output");
    *piece_bytes = g_piece_bytes;
    return SMI_SUCCESS;
}

}  // extern "C"
