// stencil_run.cpp -- the stencil_smi program on one rank's tile.
//
// Reference host + Convert kernels replaced: examples/host/stencil_smi.cpp
// (rank map :133-134, ping-pong half :344) and the eight
// Convert{Send,Receive}{Top,Bottom,Left,Right} kernels of
// examples/kernels/stencil_smi.cl:236-386, whose per-element SMI_Push/SMI_Pop
// streams become one transport group of bulk sends/receives per exchange.
#include <sched.h>

#include <chrono>
#include <cstdlib>

#include "stencil_common.h"

namespace smi {

struct Neighbours {
    int top = -1, bottom = -1, left = -1, right = -1;   // stencil_smi.cl:242,257,269,293
    int tl = -1, tr = -1, bl = -1, br = -1;             // diagonals (depth-2 corners only)
};

// The pass-boundary join of the K-step passes.  interior(t) reads the bands
// band(t-1) wrote on the comm stream.  A stream wait on its event costs a
// barrier packet on the main stream -- ~7-10 us between two interiors even
// when band(t-1) finished long before (tools/streambench).
// band(t-1) runs beside interior(t-1) and normally ends well inside it, so the
// host watches it instead: once hipEventQuery reports it complete (its
// end-of-kernel release done), interior(t) is enqueued behind interior(t-1)
// with no wait packet, and its own dispatch acquire makes the bands visible.
// Should interior(t-1) finish first, the host still waits for band(t-1): a
// wait packet on the library's own interior stream measured far worse than
// the host's few microseconds (0.70 vs 0.91 of a lone tile).
// The host only waits for work already enqueued, so no rank's host can block
// another's (every exchange up to t-1 was posted before).
static bool host_join_enabled() {
#ifdef SMI_LOOPBACK_REHEARSAL
    if (const char *v = getenv("SMI_HOST_JOIN")) return atoi(v) != 0;  // rehearsal A/B
#endif
    return g_tune.host_join != 0;
}

#ifdef SMI_LOOPBACK_REHEARSAL
// rehearsal: a host thread that falls behind -- SMI_REH_STALL_US of busy
// host time before every SMI_REH_STALL_EVERY-th pass's interior is enqueued
// (the same point under either join), to price what a descheduled host costs
static void rehearsal_stall(int kpass) {
    static const long us = getenv("SMI_REH_STALL_US") ? atol(getenv("SMI_REH_STALL_US")) : 0;
    static const int every = getenv("SMI_REH_STALL_EVERY") ? std::max(1, atoi(getenv("SMI_REH_STALL_EVERY"))) : 10;
    if (us <= 0 || kpass % every != every / 2) return;
    const auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(us)) {
    }
}
#else
static void rehearsal_stall(int) {}
#endif

// The wait: a short spin (the band normally ended long before, and a wake-up
// after a sleep would cost the pass more than it saves), then the core is
// yielded between polls, so that rank threads sharing the job's cores (the
// in-process groups, the C++ hosts) reach their own transport rendezvous --
// which band(t-1)'s exchange may be waiting for.  A band that never finishes
// (a peer that failed, so exchange(t-2) never completes) is an error after
// kJoinTimeout rather than a spin forever.
static constexpr int kJoinSpinPolls = 64;
static constexpr std::chrono::seconds kJoinTimeout{300};

static int join_band(hipEvent_t band_prev) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned polls = 0;; ++polls) {
        const hipError_t q = hipEventQuery(band_prev);
        if (q == hipSuccess) return SMI_SUCCESS;
        if (q != hipErrorNotReady) SMI_HIP_CHECK(q);
        if (polls < kJoinSpinPolls) continue;
        if ((polls & 1023) == 0 && std::chrono::steady_clock::now() - t0 > kJoinTimeout) {
            set_error("smi_stencil_run: the band kernel of the previous pass did not finish within 300 s "
                      "(a peer rank stopped exchanging halos?)");
            return SMI_ERR_COMM;
        }
        sched_yield();
    }
}

// The stream the multi-rank interior runs on.  HIP maps streams onto
// GPU_MAX_HW_QUEUES (default 4) hardware queues per priority and shares a
// queue between streams beyond that; RCCL makes streams of its own.  A
// caller's stream at normal priority created after the communicator landed
// on a queue RCCL's work also uses, and the interior then serialised with the
// exchange: 0.70-0.79 of a lone tile instead of 0.92-0.94 in the interior-rank
// rehearsal (profiles/r05/rehearsal/queues/).  The comm stream is at the
// highest priority; an interior stream there as well gets a queue of its own.
// So a caller's stream at the highest priority is used as it is; any other
// is joined to an interior stream of the communicator at that priority (a
// wait only when the caller's stream still has work pending) and joins it
// back at the end of the run.
static int interior_stream(Comm *c, hipStream_t user, hipStream_t *out, bool *own) {
    int least = 0, greatest = 0, prio = 0;
    SMI_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    SMI_HIP_CHECK(hipStreamGetPriority(user, &prio));
    *out = user;
    *own = false;
    if (prio == greatest) return SMI_SUCCESS;
    if (!c->interior_stream) {
        // made on the communicator's device whatever the calling thread's
        // current device is (the stream lives as long as the communicator)
        int cur = 0;
        SMI_HIP_CHECK(hipGetDevice(&cur));
        if (cur != c->device) SMI_HIP_CHECK(hipSetDevice(c->device));
        const hipError_t e = hipStreamCreateWithPriority(&c->interior_stream, hipStreamNonBlocking, greatest);
        if (cur != c->device) SMI_HIP_CHECK(hipSetDevice(cur));
        SMI_HIP_CHECK(e);
    }
    const hipError_t q = hipStreamQuery(user);
    if (q == hipErrorNotReady) {
        hipEvent_t ev;
        SMI_TRY(comm_event(c, 3, &ev));
        SMI_HIP_CHECK(hipEventRecord(ev, user));
        SMI_HIP_CHECK(hipStreamWaitEvent(c->interior_stream, ev, 0));
    } else if (q != hipSuccess) {
        SMI_HIP_CHECK(q);
    }
    *out = c->interior_stream;
    *own = true;
    return SMI_SUCCESS;
}

// Depth-1 exchange: new first/last row -> rank above/below, packed first/last
// column -> left/right rank; the four halo vectors come back from them.
static int exchange1(Comm *c, const Neighbours &nb, const float *tile, int rows, int cols, float *h_top,
                     float *h_bot, float *h_left, float *h_right, const float *s_left, const float *s_right,
                     hipStream_t s) {
    Transport *tp = c->transport.get();
    const size_t rb = (size_t)cols * sizeof(float), cb = (size_t)rows * sizeof(float);
    Group grp(tp);
    SMI_TRY(grp.begin(s));
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
    return grp.end();
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
    Group grp(tp);
    SMI_TRY(grp.begin(s));
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
    return grp.end();
}

// Depth-K exchange (once per K steps): K rows / KC = kc_of(K) columns per
// side neighbour, one K x KC block per diagonal neighbour.
struct HaloKBuf {
    float *top, *bot, *left, *right, *send_left, *send_right;
    float *corner[4], *send_corner[4];
    HaloK view() const {
        HaloK h;
        h.top = top;
        h.bot = bot;
        h.left = left;
        h.right = right;
        h.send_left = send_left;
        h.send_right = send_right;
        for (int k = 0; k < 4; ++k) {
            h.corner[k] = corner[k];
            h.send_corner[k] = send_corner[k];
        }
        return h;
    }
};

static int exchangek(Comm *c, const Neighbours &nb, const float *tile, int rows, int cols, int K, const HaloKBuf &h,
                     hipStream_t s) {
    Transport *tp = c->transport.get();
#ifdef SMI_LOOPBACK_REHEARSAL
    if (getenv("SMI_LOOPBACK_NOXCHG")) return SMI_SUCCESS;  // rehearsal: price bands + interior alone
#endif
    const int KC = kc_of(K);
    const size_t rb = (size_t)K * cols * sizeof(float), cb = (size_t)rows * KC * sizeof(float);
    const size_t kb = (size_t)K * KC * sizeof(float);
#ifdef SMI_LOOPBACK_REHEARSAL
    if (getenv("SMI_LOOPBACK_FUSED") && nb.top == 0 && nb.left == 0 && nb.tl == 0) {
        // rehearsal: the same 8 messages as one copy kernel (like one RCCL group)
        const void *src[8] = {tile, tile + (size_t)(rows - K) * cols, h.send_left, h.send_right,
                              h.send_corner[0], h.send_corner[1], h.send_corner[2], h.send_corner[3]};
        void *dst[8] = {h.bot, h.top, h.right, h.left, h.corner[3], h.corner[2], h.corner[1], h.corner[0]};
        const size_t by[8] = {rb, rb, cb, cb, kb, kb, kb, kb};
        return launch_copies(src, dst, by, 8, s);
    }
    if (const char *hv = getenv("SMI_LOOPBACK_HEAVY")) {
        if (nb.top == 0 && nb.left == 0 && nb.tl == 0) {
            // rehearsal: one copy kernel with rcclGenericKernel's footprint,
            // SMI_LOOPBACK_HEAVY workgroups (RCCL's channels)
            const void *src[8] = {tile, tile + (size_t)(rows - K) * cols, h.send_left, h.send_right,
                                  h.send_corner[0], h.send_corner[1], h.send_corner[2], h.send_corner[3]};
            void *dst[8] = {h.bot, h.top, h.right, h.left, h.corner[3], h.corner[2], h.corner[1], h.corner[0]};
            const size_t by[8] = {rb, rb, cb, cb, kb, kb, kb, kb};
            return launch_heavy_copies(src, dst, by, 8, atoi(hv), s);
        }
    }
#endif
    Group grp(tp);
    SMI_TRY(grp.begin(s));
    if (nb.top >= 0) {
        SMI_TRY(tp->send(tile, rb, nb.top));
        SMI_TRY(tp->recv(h.top, rb, nb.top));
    }
    if (nb.bottom >= 0) {
        SMI_TRY(tp->send(tile + (size_t)(rows - K) * cols, rb, nb.bottom));
        SMI_TRY(tp->recv(h.bot, rb, nb.bottom));
    }
    if (nb.left >= 0) {
        SMI_TRY(tp->send(h.send_left, cb, nb.left));
        SMI_TRY(tp->recv(h.left, cb, nb.left));
    }
    if (nb.right >= 0) {
        SMI_TRY(tp->send(h.send_right, cb, nb.right));
        SMI_TRY(tp->recv(h.right, cb, nb.right));
    }
    const int diag[4] = {nb.tl, nb.tr, nb.bl, nb.br};
    for (int k = 0; k < 4; ++k) {
        if (diag[k] < 0) continue;
        SMI_TRY(tp->send(h.send_corner[k], kb, diag[k]));
        SMI_TRY(tp->recv(h.corner[k], kb, diag[k]));
    }
    return grp.end();
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

static Neighbours neighbours_of(int rank, int px, int py) {
    // rank -> (i_px, i_py), examples/host/stencil_smi.cpp:133-134
    const int ipx = rank / py, ipy = rank % py;
    Neighbours nb;
    if (ipx > 0) nb.top = (ipx - 1) * py + ipy;
    if (ipx < px - 1) nb.bottom = (ipx + 1) * py + ipy;
    if (ipy > 0) nb.left = ipx * py + ipy - 1;
    if (ipy < py - 1) nb.right = ipx * py + ipy + 1;
    if (nb.top >= 0 && nb.left >= 0) nb.tl = (ipx - 1) * py + ipy - 1;
    if (nb.top >= 0 && nb.right >= 0) nb.tr = (ipx - 1) * py + ipy + 1;
    if (nb.bottom >= 0 && nb.left >= 0) nb.bl = (ipx + 1) * py + ipy - 1;
    if (nb.bottom >= 0 && nb.right >= 0) nb.br = (ipx + 1) * py + ipy + 1;
    return nb;
}

// The phases of a run: K-step passes of the configured K (clipped to what the
// tile holds: a multi-rank tile needs 2K x 2K).  A remainder of 3 or more
// steps is spread over the passes instead -- the same number of passes,
// balanced to within one step (T = 20 at K = 12: 10 + 10, not 12 + 8; a pass
// costs about one HBM sweep whatever its depth, and the deeper one of an
// unbalanced split pays for its extra levels: 8192^2 T = 20 0.2308 -> 0.2245
// ms, T = 30 0.3247 -> 0.3178 ms, profiles/r02/plan_split.jsonl); a remainder
// of 1 or 2 steps stays a pair and/or a single step (12 + 1 beats 7 + 6).
// Every phase starts from halos of the current state, so the split changes
// scheduling only, never a bit of the result.
struct Plan {
    int nph = 0;
    int k[4] = {0, 0, 0, 0};  // steps per pass
    int n[4] = {0, 0, 0, 0};  // passes
    int passes() const { return n[0] + n[1] + n[2] + n[3]; }
};

static Plan make_plan(int rows, int cols, int timesteps, bool multi) {
    Plan p;
    auto add = [&](int k, int n) {
        if (n > 0) {
            p.k[p.nph] = k;
            p.n[p.nph] = n;
            ++p.nph;
        }
    };
    const int fuse = g_tune.fuse;
    int K = fuse >= SWEEPK_MIN ? fuse : 0;
    if (K && multi) {
        // a multi-rank tile holds the K-row bands and the float4-aligned
        // K-column bands (4 * ceil(K / 4) wide) of both sides
        K = std::min(K, rows / 2);
        while (K > 0 && 8 * ((K + 3) / 4) > cols) --K;
    }
    if (K > SWEEPK_MAX) {
        // deep passes (stencild.h) need a tall enough sweep rectangle (a
        // multi-rank interior loses K rows per side with a neighbour)
        SweepKArgs probe{};
        probe.rows = rows;
        probe.cols = cols;
        probe.row_hi = multi ? rows - 2 * K : rows;
        probe.col_hi = cols;
        if (!sweepd_fits(K, probe)) K = SWEEPK_MAX;
    }
    if (cols < 8 || K < SWEEPK_MIN) K = 0;
    int rest = timesteps;
    if (K) {
        const int passes = rest / K + 1, base = rest / passes, extra = rest % passes;
        if (rest % K >= SWEEPK_MIN && base >= SWEEPK_MIN) {
            add(base + 1, extra);
            add(base, passes - extra);
            rest = 0;
        } else {
            add(K, rest / K);
            rest %= K;
        }
    }
    if (fuse >= 2 && rows >= 4 && cols >= 8) {
        add(2, rest / 2);
        rest %= 2;
    }
    add(1, rest);
    return p;
}

}  // namespace smi

using namespace smi;

extern "C" {

int smi_stencil_set_fusion(int steps_per_pass, int rows_per_wave, int rows_in_flight) {
    if (steps_per_pass > 0) {
        SMI_ARG_CHECK(steps_per_pass <= SWEEPD_MAX, "steps_per_pass must be 1..20");
        g_tune.fuse = steps_per_pass;
    }
    // rows_per_wave / rows_in_flight tune the kernel of the current setting
    const bool deep = g_tune.fuse >= SWEEPK_MIN;
    if (rows_per_wave > 0) (deep ? g_tune.htk : g_tune.ht2) = rows_per_wave;
    if (rows_per_wave < 0 && deep) g_tune.htk = 0;  // automatic: one round of resident waves
    if (rows_in_flight > 0 && !deep) {
        SMI_ARG_CHECK(rows_in_flight == 1 || rows_in_flight == 2 || rows_in_flight == 4 || rows_in_flight == 8,
                      "rows_in_flight must be 1, 2, 4 or 8");
        g_tune.u2 = rows_in_flight;
    }
    // the K-step sweep's pipeline depth is fixed at build time;
    // rows_in_flight is accepted and ignored there
    return SMI_SUCCESS;
}

int smi_stencil_get_fusion(int *steps_per_pass, int *rows_per_wave, int *rows_in_flight) {
    const bool deep = g_tune.fuse >= SWEEPK_MIN;
    if (steps_per_pass) *steps_per_pass = g_tune.fuse;
    if (rows_per_wave) *rows_per_wave = deep ? g_tune.htk : g_tune.ht2;
    if (rows_in_flight) *rows_in_flight = deep ? g_tune.uk : g_tune.u2;
    return SMI_SUCCESS;
}

int smi_stencil_set_bands(int reserve_waves, int interior_rounds) {
    SMI_ARG_CHECK(reserve_waves <= 65536 && interior_rounds <= 64, "reserve_waves / interior_rounds out of range");
    if (reserve_waves >= 0) g_tune.band_reserve = reserve_waves;
    if (interior_rounds >= 0) g_tune.rounds_multi = std::max(1, interior_rounds);
    return SMI_SUCCESS;
}

int smi_stencil_get_bands(int *reserve_waves, int *interior_rounds) {
    if (reserve_waves) *reserve_waves = g_tune.band_reserve;
    if (interior_rounds) *interior_rounds = g_tune.rounds_multi;
    return SMI_SUCCESS;
}

int smi_stencil_set_band_kernel(int lean) {
    SMI_ARG_CHECK(lean <= 1, "band kernel: 0 (one wave per segment) or 1 (lean, beside the interior)");
    if (lean >= 0) g_tune.band_lean = lean;
    return SMI_SUCCESS;
}

int smi_stencil_get_band_kernel(int *lean) {
    if (lean) *lean = g_tune.band_lean;
    return SMI_SUCCESS;
}

int smi_stencil_set_join(int host_join) {
    SMI_ARG_CHECK(host_join <= 1, "pass join: 0 (device-side wait) or 1 (host-observed)");
    if (host_join >= 0) g_tune.host_join = host_join;
    return SMI_SUCCESS;
}

int smi_stencil_get_join(int *host_join) {
    if (host_join) *host_join = g_tune.host_join;
    return SMI_SUCCESS;
}

int smi_stencil_set_deep(int ce16, int rev16, int waves) {
    SMI_ARG_CHECK(ce16 <= 256 && rev16 <= 256 && waves <= (1 << 20), "deep sweep settings out of range");
    if (ce16 >= 0) g_tune.deep_ce16 = ce16;
    if (rev16 >= 0) g_tune.deep_rev16 = rev16;
    if (waves >= 0) g_tune.deep_waves = waves;
    return SMI_SUCCESS;
}

int smi_stencil_get_deep(int *ce16, int *rev16, int *waves) {
    if (ce16) *ce16 = g_tune.deep_ce16;
    if (rev16) *rev16 = g_tune.deep_rev16;
    if (waves) *waves = g_tune.deep_waves;
    return SMI_SUCCESS;
}

int smi_stencil_deep_geometry(int rows, int cols, int K, int side_mask, int *waves, int *strips, int *row_blocks,
                              int *row_blocks_edge, int *min_block_rows) {
    SMI_ARG_CHECK(rows >= 1 && cols >= 4 && cols % 4 == 0, "tile must be >= 1 x 4, cols % 4 == 0");
    SMI_ARG_CHECK(side_mask >= 0 && side_mask < 16, "side_mask: bits 0..3");
    SweepKArgs a{};
    a.rows = rows;
    a.cols = cols;
    const int kc = kc_of(K);
    a.row_lo = (side_mask & 1) ? K : 0;
    a.row_hi = (side_mask & 2) ? rows - K : rows;
    a.col_lo = (side_mask & 4) ? kc : 0;
    a.col_hi = (side_mask & 8) ? cols - kc : cols;
    a.gT = !(side_mask & 1);
    a.gB = !(side_mask & 2);
    a.gL = !(side_mask & 4);
    a.gR = !(side_mask & 8);
    SMI_ARG_CHECK(sweepd_fits(K, a), "K outside 13..20 or sweep rectangle shorter than 4K rows");
    SweepDGeom g;
    SMI_TRY(sweepd_geometry(K, a, 0, &g));
    int hmin = rows;
    for (int pass = 0; pass < 2; ++pass) {
        const int nb = pass ? g.nrb_ce : g.nrb;
        if (pass ? (g.tasks == g.n_int * g.nrb) : g.n_int == 0) continue;
        for (int rb = 0; rb < nb; ++rb) {
            int o0, o1;
            sweepd_block_rows(a, rb, nb, g.wlast, &o0, &o1);
            hmin = std::min(hmin, o1 - o0);
        }
    }
    if (waves) *waves = g.tasks;
    if (strips) *strips = g.nstrips;
    if (row_blocks) *row_blocks = g.nrb;
    if (row_blocks_edge) *row_blocks_edge = g.tasks == g.n_int * g.nrb ? 0 : g.nrb_ce;
    if (min_block_rows) *min_block_rows = hmin;
    return SMI_SUCCESS;
}

int smi_stencil_plan(int x_local, int y_local, int px, int py, int rank, int timesteps, SMI_StencilPhase *phases,
                     int max_phases, int *nphases, int *neighbours, int *result_index) {
    SMI_ARG_CHECK(x_local >= 1 && y_local >= 4 && y_local % 4 == 0, "tile must be >= 1 x 4, y_local % 4 == 0");
    SMI_ARG_CHECK(px >= 1 && py >= 1 && rank >= 0 && rank < px * py, "rank outside the px x py grid");
    SMI_ARG_CHECK(timesteps >= 0, "timesteps < 0");
    SMI_ARG_CHECK(nphases && (phases || max_phases == 0), "NULL output");
    const Neighbours nb = neighbours_of(rank, px, py);
    const bool multi = nb.top >= 0 || nb.bottom >= 0 || nb.left >= 0 || nb.right >= 0;
    const Plan p = make_plan(x_local, y_local, timesteps, multi);
    SMI_ARG_CHECK(max_phases >= p.nph, "max_phases too small (4 always suffice)");
    for (int i = 0; i < p.nph; ++i) {
        phases[i].steps_per_pass = p.k[i];
        phases[i].passes = p.n[i];
    }
    *nphases = p.nph;
    if (neighbours) {
        const int v[8] = {nb.top, nb.bottom, nb.left, nb.right, nb.tl, nb.tr, nb.bl, nb.br};
        for (int i = 0; i < 8; ++i) neighbours[i] = v[i];
    }
    if (result_index) *result_index = p.passes() & 1;
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
    Neighbours nb = neighbours_of(c->rank, px, py);
#ifdef SMI_LOOPBACK_REHEARSAL
    // Timing-rehearsal build only (never the product library; built by
    // `smi_amd/build.py --rehearsal`, driven by tools/rehearsal.py): with
    // SMI_LOOPBACK=1 a 1x1 run is its own neighbour on every side and
    // diagonal, so one GPU replays the full per-pass work of an interior rank
    // of a large decomposition (band kernel, 8-way exchange through the
    // transport, interior sweep) with the same stream schedule.  The halos
    // then wrap around, so the numbers differ from the stencil's.
    if (px == 1 && py == 1 && c->size == 1 && getenv("SMI_LOOPBACK"))
        nb.top = nb.bottom = nb.left = nb.right = nb.tl = nb.tr = nb.bl = nb.br = 0;
#endif
    const int side_nb[4] = {nb.top, nb.bottom, nb.left, nb.right};
    int side_mask = 0;
    for (int k = 0; k < 4; ++k)
        if (side_nb[k] >= 0) side_mask |= 1 << k;

    const Plan plan = make_plan(rows, cols, timesteps, side_mask != 0);
    *result_index = plan.passes() & 1;
    prof_break_chain();  // markers chain only between this run's own passes
    if (timesteps == 0) return SMI_SUCCESS;
    int kmax = 0;  // deepest K-step phase (sizes the depth-K staging)
    for (int i = 0; i < plan.nph; ++i) kmax = std::max(kmax, plan.k[i] >= SWEEPK_MIN ? plan.k[i] : 0);

    // single-step arguments (modes / halo views set below)
    SweepArgs a{};
    a.rows = rows;
    a.cols = cols;
    for (int k = 0; k < 4; ++k) a.mode[k] = side_nb[k] >= 0 ? SMI_SIDE_HALO : SMI_SIDE_COPY;
    Sweep2Args a2{};
    a2.rows = rows;
    a2.cols = cols;
    for (int k = 0; k < 4; ++k) a2.skip[k] = side_nb[k] >= 0;
    // K-step passes: the interior sweep stays K rows / 4*ceil(K/4) columns
    // clear of every halo-facing side (the band kernel computes those bands
    // beside it); global edges are handled inside the sweep (stencilk.h).
    auto interior_args = [&](int K) {
        SweepKArgs ak{};
        ak.rows = rows;
        ak.cols = cols;
        const int kc = kc_of(K);
        ak.row_lo = nb.top >= 0 ? K : 0;
        ak.row_hi = nb.bottom >= 0 ? rows - K : rows;
        ak.col_lo = nb.left >= 0 ? kc : 0;
        ak.col_hi = nb.right >= 0 ? cols - kc : cols;
        ak.gT = nb.top < 0;
        ak.gB = nb.bottom < 0;
        ak.gL = nb.left < 0;
        ak.gR = nb.right < 0;
        return ak;
    };
    auto band_args = [&]() {
        BandKArgs bk{};
        bk.rows = rows;
        bk.cols = cols;
        for (int k = 0; k < 4; ++k) bk.has[k] = side_nb[k] >= 0;
        bk.pack = side_mask != 0;
        return bk;
    };

    int cur = 0;  // index of the buffer holding the current state
    auto bufp = [&](int i) { return i ? buf1 : buf0; };

    if (side_mask == 0) {  // single tile: no halos, no exchange, no events
        for (int ph = 0; ph < plan.nph; ++ph) {
            const int K = plan.k[ph];
            SweepKArgs ak = interior_args(K);
            for (int p = 0; p < plan.n[ph]; ++p, cur ^= 1) {
                if (K >= SWEEPK_MIN) {
                    ak.in = bufp(cur);
                    ak.out = bufp(cur ^ 1);
                    SMI_TRY(launch_sweepk(K, ak, s));
                } else if (K == 2) {
                    a2.in = bufp(cur);
                    a2.out = bufp(cur ^ 1);
                    SMI_TRY(launch_sweep2(a2, s));
                } else {
                    a.in = bufp(cur);
                    a.out = bufp(cur ^ 1);
                    SMI_TRY(launch_sweep(a, s));
                }
            }
        }
        return SMI_SUCCESS;
    }

    hipEvent_t ev_edge, ev_int, ev_edge_alt, ev_fin;
    SMI_TRY(comm_event(c, 0, &ev_edge));
    SMI_TRY(comm_event(c, 1, &ev_int));
    SMI_TRY(comm_event(c, 2, &ev_edge_alt));
    SMI_TRY(comm_event(c, 4, &ev_fin));
    const bool overlap = g_tune.overlap != 0;
    const hipStream_t user = s;
    bool own_stream = false;
    if (overlap) SMI_TRY(interior_stream(c, user, &s, &own_stream));

    // Halo staging.  Depth 2 (its inner row/column doubles as the depth-1
    // halo): top2 | bot2 | left2 | right2 | corner(4) | send_left2 |
    // send_right2 | send_corner(4); then depth K (16-byte aligned): top | bot
    // (K x cols) | left | right | send_left | send_right (rows x KC, [row][k])
    // | 4 + 4 K x KC corners.  The regions are sized for the deepest phase; a
    // shallower phase (the remainder pass) lays its depth out densely from
    // the start of each region.
    const size_t need2 = (4 * (size_t)cols + 8 * (size_t)rows + 8 + 3) / 4 * 4;
    const size_t kcmax = kc_of(kmax);
    const size_t needk = kmax ? 2 * (size_t)kmax * cols + 4 * (size_t)rows * kcmax + 8 * (size_t)kmax * kcmax : 0;
    SMI_TRY(ensure_halo(c, need2 + needk));
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
    auto halok = [&]() {
        HaloKBuf hk{};
        float *p = c->halo + need2;
        hk.top = p;
        hk.bot = hk.top + (size_t)kmax * cols;
        hk.left = hk.bot + (size_t)kmax * cols;
        hk.right = hk.left + (size_t)rows * kcmax;
        hk.send_left = hk.right + (size_t)rows * kcmax;
        hk.send_right = hk.send_left + (size_t)rows * kcmax;
        float *q = hk.send_right + (size_t)rows * kcmax;
        for (int k = 0; k < 4; ++k) {
            hk.corner[k] = q + (size_t)k * kmax * kcmax;
            hk.send_corner[k] = q + (size_t)(4 + k) * kmax * kcmax;
        }
        return hk;
    };
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

    int kpass = 0;                 // K-step passes of the current phase
    hipEvent_t last_band = nullptr;  // completion of the phase's last band kernel (host join)

    // Schedule (two streams, no host synchronisation between passes):
    //   comm stream : [wait interior(t-1)] band(t) -> rec E_edge(t) -> exchange(t)
    //   main stream : [wait E_edge(t-1)] interior(t)    -> rec E_int(t)
    // The band kernel (the depth-K bands; the depth-2 / depth-1 phases use
    // their ring / edge kernels) reads in(t) (interior cells from interior(t-1),
    // halo-facing cells from its own predecessor) and the halos of
    // exchange(t-1); the interior reads only in(t), never a halo vector, so
    // neither the halo-facing cells nor the xGMI exchange sit on its path.
    // Each phase (K-step passes, the remainder pass, pairs, singles) starts
    // from halos of the current state: the neighbours' current edges (for
    // the first phase the reference's artificial timestep t=0,
    // stencil_smi.cl:26-29,183-224).
    const bool host_join = overlap && host_join_enabled();
    auto phase_start = [&]() -> int {
        SMI_HIP_CHECK(hipEventRecord(ev_int, s));
        SMI_HIP_CHECK(hipStreamWaitEvent(cs, ev_int, 0));
        return SMI_SUCCESS;
    };
    // one pass of a phase: bands (comm stream) + interior (main stream)
    // ring(st, stop) / interior(st, stop): stop (nullable) = an event the
    // launch records by its own dispatch (K-step passes: no marker packets
    // between kernels; ~4 us per pass, tools/streambench); the other phases'
    // kernels ignore it and it is recorded after them here.
    auto pass = [&](auto ring, auto interior, auto xchg, bool need_xchg, const float *out, bool carries) -> int {
        if (overlap && carries && host_join) {
            // K-step passes, host-observed join (see join_band above):
            // band(t) carries ev_band[t & 1]; interior(t) follows band(t-1)
            // with no wait packet when the host has seen band(t-1) finish
            hipEvent_t ev_cur = (kpass & 1) ? ev_edge_alt : ev_edge, ev_prev = (kpass & 1) ? ev_edge : ev_edge_alt;
            SMI_TRY(ring(cs, ev_cur));
            rehearsal_stall(kpass);
            if (kpass > 0) SMI_TRY(join_band(ev_prev));
            SMI_TRY(interior(s, ev_int));
            if (need_xchg) SMI_TRY(xchg(out, cs));
            SMI_HIP_CHECK(hipStreamWaitEvent(cs, ev_int, 0));
            last_band = ev_cur;
            ++kpass;
        } else if (overlap) {
            // The interior is enqueued before the exchange: posting the
            // transport's sends/receives costs host time (RCCL group, or
            // event + copy per message in-process) that must not delay the
            // interior's launch -- the trace of an interior rank showed the
            // main stream idle ~100 us per pass behind the exchange calls.
            SMI_TRY(ring(cs, carries ? ev_edge : nullptr));
            if (!carries) SMI_HIP_CHECK(hipEventRecord(ev_edge, cs));
            if (carries) rehearsal_stall(kpass++);
            SMI_TRY(interior(s, carries ? ev_int : nullptr));
            if (!carries) SMI_HIP_CHECK(hipEventRecord(ev_int, s));
            SMI_HIP_CHECK(hipStreamWaitEvent(s, ev_edge, 0));
            if (need_xchg) SMI_TRY(xchg(out, cs));
            SMI_HIP_CHECK(hipStreamWaitEvent(cs, ev_int, 0));
        } else {
            SMI_HIP_CHECK(hipEventRecord(ev_edge, cs));
            SMI_HIP_CHECK(hipStreamWaitEvent(s, ev_edge, 0));
            SMI_TRY(ring(s, nullptr));
            SMI_TRY(interior(s, nullptr));
            SMI_HIP_CHECK(hipEventRecord(ev_int, s));
            SMI_HIP_CHECK(hipStreamWaitEvent(cs, ev_int, 0));
            if (need_xchg) SMI_TRY(xchg(out, cs));
        }
        return SMI_SUCCESS;
    };

    for (int ph = 0; ph < plan.nph; ++ph) {
        const int K = plan.k[ph], npass = plan.n[ph];
        SMI_TRY(phase_start());
        if (K >= SWEEPK_MIN) {
            // ---- K steps per pass (depth-K halos)
            const HaloKBuf hk = halok();
            const HaloK hkv = hk.view();
            SweepKArgs ak = interior_args(K);
            BandKArgs bk = band_args();
            bk.h = hkv;
            auto xchgk = [&](const float *tile, hipStream_t st) {
                return exchangek(c, nb, tile, rows, cols, K, hk, st);
            };
            SMI_TRY(launch_packk(bufp(cur), rows, cols, K, hkv, cs));
            SMI_TRY(xchgk(bufp(cur), cs));
            kpass = 0;
            for (int p = 0; p < npass; ++p, cur ^= 1) {
                bk.in = ak.in = bufp(cur);
                bk.out = ak.out = bufp(cur ^ 1);
                SMI_TRY(pass([&](hipStream_t st, hipEvent_t stop) {
                                 return launch_bandk(K, bk, g_tune.band_reserve, st, stop);
                             },
                             [&](hipStream_t st, hipEvent_t stop) {
                                 return launch_sweepk_ex(K, ak, 0, g_tune.band_reserve, true, st, stop);
                             },
                             xchgk, p < npass - 1, ak.out, true));
            }
            // whatever runs next on the main stream reads the last bands:
            // joined on the host as well (no wait packet on the interior
            // stream, see join_band)
            if (host_join && last_band) SMI_TRY(join_band(last_band));
        } else if (K == 2) {
            // ---- pairs of steps (depth-2 halos)
            SMI_TRY(launch_pack2(bufp(cur), rows, cols, h2, cs));
            SMI_TRY(xchg2(bufp(cur), cs));
            for (int p = 0; p < npass; ++p, cur ^= 1) {
                a2.in = bufp(cur);
                a2.out = bufp(cur ^ 1);
                SMI_TRY(pass([&](hipStream_t st, hipEvent_t) { return launch_ring2(a2, h2, st); },
                             [&](hipStream_t st, hipEvent_t) { return launch_sweep2(a2, st); }, xchg2, p < npass - 1,
                             a2.out, false));
            }
        } else {
            // ---- single steps (depth-1 halos)
            SMI_TRY(launch_pack_cols(bufp(cur), rows, cols, a.send_left, a.send_right, cs));
            SMI_TRY(xchg1(bufp(cur), cs));
            SweepArgs inner = a;  // interior launch: halo-facing sides left to the edge kernel
            for (int k = 0; k < 4; ++k)
                if (inner.mode[k] == SMI_SIDE_HALO) inner.mode[k] = SMI_SIDE_SKIP;
            inner.send_left = inner.send_right = nullptr;
            for (int t = 0; t < npass; ++t, cur ^= 1) {
                a.in = inner.in = bufp(cur);
                a.out = inner.out = bufp(cur ^ 1);
                if (overlap) {
                    SMI_TRY(pass([&](hipStream_t st, hipEvent_t) { return launch_edge(a, side_mask, st); },
                                 [&](hipStream_t st, hipEvent_t) { return launch_sweep(inner, st); }, xchg1,
                                 t < npass - 1, a.out, false));
                } else {
                    // the full sweep reads the halos itself
                    SMI_TRY(pass([&](hipStream_t, hipEvent_t) { return (int)SMI_SUCCESS; },
                                 [&](hipStream_t st, hipEvent_t) { return launch_sweep(a, st); }, xchg1,
                                 t < npass - 1, a.out, false));
                }
            }
        }
    }
    // the caller's stream owns the result: join the comm stream (and the
    // interior stream when the run had one)
    SMI_HIP_CHECK(hipEventRecord(ev_edge, cs));
    SMI_HIP_CHECK(hipStreamWaitEvent(user, ev_edge, 0));
    if (own_stream) {
        SMI_HIP_CHECK(hipEventRecord(ev_fin, s));
        SMI_HIP_CHECK(hipStreamWaitEvent(user, ev_fin, 0));
    }
    return SMI_SUCCESS;
}

}  // extern "C"
