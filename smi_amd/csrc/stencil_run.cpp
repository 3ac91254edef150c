// stencil_run.cpp -- the stencil_smi program on one rank's tile.
//
// Reference host + Convert kernels replaced: examples/host/stencil_smi.cpp
// (rank map :133-134, ping-pong half :344) and the eight
// Convert{Send,Receive}{Top,Bottom,Left,Right} kernels of
// examples/kernels/stencil_smi.cl:236-386, whose per-element SMI_Push/SMI_Pop
// streams become one transport group of bulk sends/receives per exchange.
#include "stencil_common.h"

namespace smi {

struct Neighbours {
    int top = -1, bottom = -1, left = -1, right = -1;   // stencil_smi.cl:242,257,269,293
    int tl = -1, tr = -1, bl = -1, br = -1;             // diagonals (depth-2 corners only)
};

// Depth-1 exchange: new first/last row -> rank above/below, packed first/last
// column -> left/right rank; the four halo vectors come back from them.
static int exchange1(Comm *c, const Neighbours &nb, const float *tile, int rows, int cols, float *h_top,
                     float *h_bot, float *h_left, float *h_right, const float *s_left, const float *s_right,
                     hipStream_t s) {
    Transport *tp = c->transport.get();
    const size_t rb = (size_t)cols * sizeof(float), cb = (size_t)rows * sizeof(float);
    SMI_TRY(tp->begin(s));
    if (nb.top >= 0) {
        SMI_TRY(tp->send(tile, rb, nb.top));
        SMI_TRY(tp->recv(h_top, rb, nb.top));
    }
    if (nb.bottom >= 0) {
        SMI_TRY(tp->send(tile + (size_t)(rows - 1) * cols, rb, nb.bottom));
        SMI_TRY(tp->recv(h_bot, rb, nb.bottom));
    }
    if (nb.left >= 0) {
        SMI_TRY(tp->send(s_left, cb, nb.left));
        SMI_TRY(tp->recv(h_left, cb, nb.left));
    }
    if (nb.right >= 0) {
        SMI_TRY(tp->send(s_right, cb, nb.right));
        SMI_TRY(tp->recv(h_right, cb, nb.right));
    }
    return tp->end();
}

// Depth-2 exchange (once per pair of steps): two rows / two columns per
// side neighbour, one corner cell per diagonal neighbour.
struct Halo2Buf {
    float *top2, *bot2, *left2, *right2, *corner, *send_left2, *send_right2, *send_corner;
    // Every pointer is a valid allocation, also for sides without a
    // neighbour (their values are never used; the kernels rely on it).
    Halo2 view() const {
        Halo2 h;
        h.top2 = top2;
        h.bot2 = bot2;
        h.left2 = left2;
        h.right2 = right2;
        h.corner = corner;
        h.send_left2 = send_left2;
        h.send_right2 = send_right2;
        h.send_corner = send_corner;
        return h;
    }
};

static int exchange2(Comm *c, const Neighbours &nb, const float *tile, int rows, int cols, const Halo2Buf &h,
                     hipStream_t s) {
    Transport *tp = c->transport.get();
    const size_t rb = 2 * (size_t)cols * sizeof(float), cb = 2 * (size_t)rows * sizeof(float);
    SMI_TRY(tp->begin(s));
    if (nb.top >= 0) {
        SMI_TRY(tp->send(tile, rb, nb.top));
        SMI_TRY(tp->recv(h.top2, rb, nb.top));
    }
    if (nb.bottom >= 0) {
        SMI_TRY(tp->send(tile + (size_t)(rows - 2) * cols, rb, nb.bottom));
        SMI_TRY(tp->recv(h.bot2, rb, nb.bottom));
    }
    if (nb.left >= 0) {
        SMI_TRY(tp->send(h.send_left2, cb, nb.left));
        SMI_TRY(tp->recv(h.left2, cb, nb.left));
    }
    if (nb.right >= 0) {
        SMI_TRY(tp->send(h.send_right2, cb, nb.right));
        SMI_TRY(tp->recv(h.right2, cb, nb.right));
    }
    const int diag[4] = {nb.tl, nb.tr, nb.bl, nb.br};
    for (int k = 0; k < 4; ++k) {
        if (diag[k] < 0) continue;
        SMI_TRY(tp->send(h.send_corner + k, sizeof(float), diag[k]));
        SMI_TRY(tp->recv(h.corner + k, sizeof(float), diag[k]));
    }
    return tp->end();
}

static int ensure_halo(Comm *c, size_t elems) {
    if (c->halo_elems < elems) {
        if (c->halo) SMI_HIP_CHECK(hipFree(c->halo));
        c->halo = nullptr;
        SMI_HIP_CHECK(hipMalloc(&c->halo, elems * sizeof(float)));
        c->halo_elems = elems;
    }
    return SMI_SUCCESS;
}

}  // namespace smi

using namespace smi;

extern "C" {

int smi_stencil_set_fusion(int steps_per_pass, int rows_per_wave, int rows_in_flight) {
    if (steps_per_pass > 0) {
        SMI_ARG_CHECK(steps_per_pass == 1 || steps_per_pass == 2, "steps_per_pass must be 1 or 2");
        g_tune.fuse = steps_per_pass;
    }
    if (rows_per_wave > 0) g_tune.ht2 = rows_per_wave;
    if (rows_in_flight > 0) {
        SMI_ARG_CHECK(rows_in_flight == 1 || rows_in_flight == 2 || rows_in_flight == 4 || rows_in_flight == 8,
                      "rows_in_flight must be 1, 2, 4 or 8");
        g_tune.u2 = rows_in_flight;
    }
    return SMI_SUCCESS;
}

int smi_stencil_get_fusion(int *steps_per_pass, int *rows_per_wave, int *rows_in_flight) {
    if (steps_per_pass) *steps_per_pass = g_tune.fuse;
    if (rows_per_wave) *rows_per_wave = g_tune.ht2;
    if (rows_in_flight) *rows_in_flight = g_tune.u2;
    return SMI_SUCCESS;
}

int smi_stencil_run(SMI_Comm comm, float *buf0, float *buf1, int x_local, int y_local, int px, int py,
                    int timesteps, SMI_Stream stream_, int *result_index) {
    Comm *c = lookup_comm(comm);
    if (!c) {
        set_error("unknown communicator");
        return SMI_ERR_BAD_COMM;
    }
    SMI_TRY(check_tile(buf0, buf1, x_local, y_local));
    SMI_ARG_CHECK(px >= 1 && py >= 1 && px * py == c->size, "px*py must equal the communicator size");
    SMI_ARG_CHECK(timesteps >= 0, "timesteps < 0");
    SMI_ARG_CHECK(result_index, "NULL result_index");
    hipStream_t s = (hipStream_t)stream_;
    hipStream_t cs = c->comm_stream;
    const int rows = x_local, cols = y_local;
    // rank -> (i_px, i_py), examples/host/stencil_smi.cpp:133-134
    const int ipx = c->rank / py, ipy = c->rank % py;
    Neighbours nb;
    if (ipx > 0) nb.top = (ipx - 1) * py + ipy;
    if (ipx < px - 1) nb.bottom = (ipx + 1) * py + ipy;
    if (ipy > 0) nb.left = ipx * py + ipy - 1;
    if (ipy < py - 1) nb.right = ipx * py + ipy + 1;
    if (nb.top >= 0 && nb.left >= 0) nb.tl = (ipx - 1) * py + ipy - 1;
    if (nb.top >= 0 && nb.right >= 0) nb.tr = (ipx - 1) * py + ipy + 1;
    if (nb.bottom >= 0 && nb.left >= 0) nb.bl = (ipx + 1) * py + ipy - 1;
    if (nb.bottom >= 0 && nb.right >= 0) nb.br = (ipx + 1) * py + ipy + 1;
    const int side_nb[4] = {nb.top, nb.bottom, nb.left, nb.right};
    int side_mask = 0;
    for (int k = 0; k < 4; ++k)
        if (side_nb[k] >= 0) side_mask |= 1 << k;

    const bool fused = g_tune.fuse == 2 && rows >= 4 && cols >= 8;
    const int pairs = fused ? timesteps / 2 : 0;
    const int singles = timesteps - 2 * pairs;
    *result_index = (pairs + singles) & 1;
    if (timesteps == 0) return SMI_SUCCESS;

    // single-step arguments (modes / halo views set below)
    SweepArgs a{};
    a.rows = rows;
    a.cols = cols;
    for (int k = 0; k < 4; ++k) a.mode[k] = side_nb[k] >= 0 ? SMI_SIDE_HALO : SMI_SIDE_COPY;
    Sweep2Args a2{};
    a2.rows = rows;
    a2.cols = cols;
    for (int k = 0; k < 4; ++k) a2.skip[k] = side_nb[k] >= 0;

    int cur = 0;  // index of the buffer holding the current state
    auto bufp = [&](int i) { return i ? buf1 : buf0; };

    if (side_mask == 0) {  // single tile: no halos, no exchange
        for (int p = 0; p < pairs; ++p, cur ^= 1) {
            a2.in = bufp(cur);
            a2.out = bufp(cur ^ 1);
            SMI_TRY(launch_sweep2(a2, s));
        }
        for (int t = 0; t < singles; ++t, cur ^= 1) {
            a.in = bufp(cur);
            a.out = bufp(cur ^ 1);
            SMI_TRY(launch_sweep(a, s));
        }
        return SMI_SUCCESS;
    }

    // Halo staging.  Depth 2 (used by both modes; the depth-1 views are its
    // inner row/column): top2 | bot2 | left2 | right2 | corner(4) |
    // send_left2 | send_right2 | send_corner(4).
    const size_t need = 4 * (size_t)cols + 8 * (size_t)rows + 8;
    SMI_TRY(ensure_halo(c, need));
    Halo2Buf hb;
    hb.top2 = c->halo;
    hb.bot2 = hb.top2 + 2 * (size_t)cols;
    hb.left2 = hb.bot2 + 2 * (size_t)cols;
    hb.right2 = hb.left2 + 2 * (size_t)rows;
    hb.corner = hb.right2 + 2 * (size_t)rows;
    hb.send_left2 = hb.corner + 4;
    hb.send_right2 = hb.send_left2 + 2 * (size_t)rows;
    hb.send_corner = hb.send_right2 + 2 * (size_t)rows;
    const Halo2 h2 = hb.view();
    // depth-1 views: row -1, row X, col -1, col Y; packed depth-1 sends
    a.halo[0] = hb.top2 + cols;
    a.halo[1] = hb.bot2;
    a.halo[2] = hb.left2 + rows;
    a.halo[3] = hb.right2;
    float *s_left = hb.send_left2 + rows;  // depth-1 packed sends (staging only)
    float *s_right = hb.send_right2;
    a.send_left = nb.left >= 0 ? s_left : nullptr;
    a.send_right = nb.right >= 0 ? s_right : nullptr;
    auto xchg1 = [&](const float *tile, hipStream_t st) {
        return exchange1(c, nb, tile, rows, cols, const_cast<float *>(a.halo[0]), const_cast<float *>(a.halo[1]),
                         const_cast<float *>(a.halo[2]), const_cast<float *>(a.halo[3]), s_left, s_right, st);
    };
    auto xchg2 = [&](const float *tile, hipStream_t st) { return exchange2(c, nb, tile, rows, cols, hb, st); };

    hipEvent_t ev_edge, ev_int;
    SMI_TRY(comm_event(c, 0, &ev_edge));
    SMI_TRY(comm_event(c, 1, &ev_int));

    // Schedule (two streams, no host synchronisation between steps):
    //   comm stream : [wait interior(t-1)] edge/ring(t) -> rec E_edge(t) -> exchange(t)
    //   main stream : [wait E_edge(t-1)] interior(t)    -> rec E_int(t)
    // The edge/ring kernel reads in(t) (interior cells from interior(t-1),
    // halo-facing cells from its own predecessor) and the halos of
    // exchange(t-1); the interior reads only in(t), never a halo vector, so
    // neither the halo-facing cells nor the xGMI exchange sit on its path.
    SMI_HIP_CHECK(hipEventRecord(ev_int, s));
    SMI_HIP_CHECK(hipStreamWaitEvent(cs, ev_int, 0));
    // initial halos = the neighbours' initial edges (the reference's
    // artificial timestep t=0, stencil_smi.cl:26-29,183-224)
    if (fused) {
        SMI_TRY(launch_pack2(buf0, rows, cols, h2, cs));
        SMI_TRY(xchg2(buf0, cs));
    } else {
        SMI_TRY(launch_pack_cols(buf0, rows, cols, a.send_left, a.send_right, cs));
        SMI_TRY(xchg1(buf0, cs));
    }

    const bool overlap = g_tune.overlap != 0;
    // ---- pairs of steps (depth-2 halos)
    for (int p = 0; p < pairs; ++p, cur ^= 1) {
        a2.in = bufp(cur);
        a2.out = bufp(cur ^ 1);
        const bool need_xchg = p < pairs - 1 || singles > 0;
        if (overlap) {
            SMI_TRY(launch_ring2(a2, h2, cs));
            SMI_HIP_CHECK(hipEventRecord(ev_edge, cs));
            if (need_xchg) SMI_TRY(xchg2(a2.out, cs));
            SMI_TRY(launch_sweep2(a2, s));
            SMI_HIP_CHECK(hipEventRecord(ev_int, s));
            SMI_HIP_CHECK(hipStreamWaitEvent(s, ev_edge, 0));
            SMI_HIP_CHECK(hipStreamWaitEvent(cs, ev_int, 0));
        } else {
            SMI_HIP_CHECK(hipEventRecord(ev_edge, cs));
            SMI_HIP_CHECK(hipStreamWaitEvent(s, ev_edge, 0));
            SMI_TRY(launch_ring2(a2, h2, s));
            SMI_TRY(launch_sweep2(a2, s));
            SMI_HIP_CHECK(hipEventRecord(ev_int, s));
            SMI_HIP_CHECK(hipStreamWaitEvent(cs, ev_int, 0));
            if (need_xchg) SMI_TRY(xchg2(a2.out, cs));
        }
    }
    if (pairs > 0 && singles > 0) {
        // the remaining single step reads depth-1 views of the last exchange
        SMI_HIP_CHECK(hipEventRecord(ev_edge, cs));
        SMI_HIP_CHECK(hipStreamWaitEvent(s, ev_edge, 0));
        a.in = bufp(cur);
        a.out = bufp(cur ^ 1);
        a.send_left = a.send_right = nullptr;
        SMI_TRY(launch_sweep(a, s));
        cur ^= 1;
        return SMI_SUCCESS;
    }

    // ---- single steps (depth-1 halos)
    SweepArgs inner = a;  // interior launch: halo-facing sides left to the edge kernel
    for (int k = 0; k < 4; ++k)
        if (inner.mode[k] == SMI_SIDE_HALO) inner.mode[k] = SMI_SIDE_SKIP;
    inner.send_left = inner.send_right = nullptr;
    if (!overlap) {  // the full sweep reads the halos on the main stream
        SMI_HIP_CHECK(hipEventRecord(ev_edge, cs));
        SMI_HIP_CHECK(hipStreamWaitEvent(s, ev_edge, 0));
    }
    for (int t = 0; t < singles; ++t, cur ^= 1) {
        const float *in = bufp(cur);
        float *out = bufp(cur ^ 1);
        const bool last = t == singles - 1;
        a.in = inner.in = in;
        a.out = inner.out = out;
        if (overlap) {
            SMI_TRY(launch_edge(a, side_mask, cs));
            SMI_HIP_CHECK(hipEventRecord(ev_edge, cs));
            if (!last) SMI_TRY(xchg1(out, cs));
            SMI_TRY(launch_sweep(inner, s));
            SMI_HIP_CHECK(hipEventRecord(ev_int, s));
            SMI_HIP_CHECK(hipStreamWaitEvent(s, ev_edge, 0));
            SMI_HIP_CHECK(hipStreamWaitEvent(cs, ev_int, 0));
        } else {
            SMI_TRY(launch_sweep(a, s));
            SMI_HIP_CHECK(hipEventRecord(ev_int, s));
            if (!last) {
                SMI_HIP_CHECK(hipStreamWaitEvent(cs, ev_int, 0));
                SMI_TRY(xchg1(out, cs));
                SMI_HIP_CHECK(hipEventRecord(ev_edge, cs));
                SMI_HIP_CHECK(hipStreamWaitEvent(s, ev_edge, 0));
            }
        }
    }
    // the caller's stream owns the result: join the comm stream
    SMI_HIP_CHECK(hipEventRecord(ev_edge, cs));
    SMI_HIP_CHECK(hipStreamWaitEvent(s, ev_edge, 0));
    return SMI_SUCCESS;
}

}  // extern "C"
