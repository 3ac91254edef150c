// stencilk.hip -- host side of the K-step sweep (kernel: stencilk.h, one
// instantiation per K in stencilk_k<K>.hip).
#include <cstdlib>

#include "stencil_common.h"

namespace smi {

#define SMI_SWEEPK_DECL(K)                                                                           \
    int sweepk_launch_k##K(const SweepKArgs &a, int nstrips, int nrb, int blocks, hipStream_t s,         \
                           hipEvent_t start, hipEvent_t stop);                                           \
    int sweepk_resident_k##K();
SMI_SWEEPK_DECL(3)
SMI_SWEEPK_DECL(4)
SMI_SWEEPK_DECL(5)
SMI_SWEEPK_DECL(6)
SMI_SWEEPK_DECL(7)
SMI_SWEEPK_DECL(8)
SMI_SWEEPK_DECL(9)
SMI_SWEEPK_DECL(10)
SMI_SWEEPK_DECL(11)
SMI_SWEEPK_DECL(12)

static int resident_waves(int K) {
    switch (K) {
    case 3: return sweepk_resident_k3();
    case 4: return sweepk_resident_k4();
    case 5: return sweepk_resident_k5();
    case 6: return sweepk_resident_k6();
    case 7: return sweepk_resident_k7();
    case 8: return sweepk_resident_k8();
    case 9: return sweepk_resident_k9();
    case 10: return sweepk_resident_k10();
    case 11: return sweepk_resident_k11();
    default: return sweepk_resident_k12();
    }
}

int sweepk_window_cols(int K) { return 256 - 8 * sweepk_apron_lanes(K); }

int launch_sweepk(int K, const SweepKArgs &a, hipStream_t s) { return launch_sweepk_ex(K, a, 0, 0, true, s); }

// Strips and row blocks of a K-step sweep over a's output rectangle.
// ht > 0: rows per wave as given; else automatic (g_tune.htk, or one round
// of resident waves -- minus `reserve` waves left to the comm stream's
// kernels in a multi-rank run, smi_stencil_set_bands).
static void sweepk_geometry(int K, const SweepKArgs &a, int ht_req, int reserve, int *nstrips_, int *nrb_) {
    const int sw = sweepk_window_cols(K);
    const int nstrips = (a.col_hi - (a.col_lo & ~31) + sw - 1) / sw;  // line-aligned strips (stencilk.h)
    const int out_rows = a.row_hi - a.row_lo;
    int ht = ht_req > 0 ? ht_req : g_tune.htk;
    if (ht <= 0) {
        // auto: one round of resident waves, each a tall row block of its
        // strip.  Multi-rank interior: either leave `reserve` waves to the
        // comm stream's kernels (one round of the rest), or cut the interior
        // into several rounds so that workgroups retire during the pass and
        // the comm stream's kernels are dispatched then.
        int waves = resident_waves(K);
        const bool single = a.gT && a.gB && a.gL && a.gR;
        int rounds = single ? 1 : std::max(1, g_tune.rounds_multi);
        if (!single && reserve > 0) {
            waves = std::max(64, waves - reserve);
            rounds = 1;
        }
        const int per_strip = std::max(1, waves * rounds / nstrips);
        ht = std::max(2 * K, (out_rows + per_strip - 1) / per_strip);
    }
    *nstrips_ = nstrips;
    *nrb_ = (out_rows + ht - 1) / ht;
}

static int check_sweepk(int K, const SweepKArgs &a) {
    SMI_ARG_CHECK(K >= SWEEPK_MIN && K <= SWEEPK_MAX, "sweepk: steps per pass must be 3..12");
    SMI_ARG_CHECK(a.cols % 4 == 0 && a.col_lo % 4 == 0 && a.col_hi % 4 == 0, "sweepk: columns not float4 aligned");
    SMI_ARG_CHECK(a.row_lo >= 0 && a.row_hi <= a.rows && a.col_lo >= 0 && a.col_hi <= a.cols,
                  "sweepk: output rectangle outside the tile");
    return SMI_SUCCESS;
}

// prof: record the launch under SMI_PROF_STENCIL_SWEEPK.  stop (nullable):
// an event the launch's dispatch records when the kernel completes (or an
// ordinary record when there is nothing to launch).
int launch_sweepk_ex(int K, const SweepKArgs &a, int ht_req, int reserve, bool prof, hipStream_t s,
                     hipEvent_t stop) {
    if (a.row_hi <= a.row_lo || a.col_hi <= a.col_lo) {
        if (stop) SMI_HIP_CHECK(hipEventRecord(stop, s));
        return SMI_SUCCESS;
    }
    if (K > SWEEPK_MAX) {
        // deeper passes: the rotating-ring sweep (stencild.h); its geometry
        // has no row-block override, and wave slots reserved for the band
        // kernel (smi_stencil_set_bands) come off its one round of waves
        SMI_ARG_CHECK(ht_req <= 0, "sweepk: K > 12 has no row-block override");
        hipEvent_t start = nullptr, kstop = stop, after = nullptr;
        int tok = -1;
        bool marker = false;
        if (prof && prof_enabled()) {
            const double units = (double)(a.row_hi - a.row_lo) * (a.col_hi - a.col_lo) * K;
            if (stop) {
                SMI_TRY(prof_launch(SMI_PROF_STENCIL_SWEEPK, &tok, K, units, &start, &kstop));
                after = stop;
            } else {
                SMI_TRY(prof_begin(SMI_PROF_STENCIL_SWEEPK, s, &tok, K, units, true));
                marker = true;
            }
        }
        SMI_TRY(launch_sweepd(K, a, reserve, s, start, kstop));
        if (after) SMI_HIP_CHECK(hipEventRecord(after, s));
        if (marker) SMI_TRY(prof_end(tok, s));
        return SMI_SUCCESS;
    }
    SMI_TRY(check_sweepk(K, a));
    int nstrips = 0, nrb = 0;
    sweepk_geometry(K, a, ht_req, reserve, &nstrips, &nrb);
    const int out_rows = a.row_hi - a.row_lo;
    const long tasks = (long)nstrips * nrb;
    const int blocks = (int)((tasks + 3) / 4);
    // Timing (profiling on).  Back-to-back single-tile passes: one chained
    // marker per pass (the end marker of pass i is the begin of pass i+1):
    // the least host time per launch -- dispatch-carried start / stop events
    // cost ~5 us more host time per launch, which a short timed run (the
    // driver's 20 steps = 2 passes) sees (tools/exp/timed_overhead.py).  A
    // multi-rank pass (`stop` given: the comm stream waits for the interior)
    // is timed by its dispatch (start / stop handed to the launch; the
    // caller's ordering event is recorded right after it).
    hipEvent_t start = nullptr, kstop = stop, after = nullptr;
    int tok = -1;
    const double units = (double)out_rows * (a.col_hi - a.col_lo) * K;
    bool marker = false;
    if (prof && prof_enabled()) {
        if (stop) {
            SMI_TRY(prof_launch(SMI_PROF_STENCIL_SWEEPK, &tok, K, units, &start, &kstop));
            after = stop;
        } else {
            SMI_TRY(prof_begin(SMI_PROF_STENCIL_SWEEPK, s, &tok, K, units, true));
            marker = true;
        }
    }
    int rc = SMI_SUCCESS;
    switch (K) {
    case 3: rc = sweepk_launch_k3(a, nstrips, nrb, blocks, s, start, kstop); break;
    case 4: rc = sweepk_launch_k4(a, nstrips, nrb, blocks, s, start, kstop); break;
    case 5: rc = sweepk_launch_k5(a, nstrips, nrb, blocks, s, start, kstop); break;
    case 6: rc = sweepk_launch_k6(a, nstrips, nrb, blocks, s, start, kstop); break;
    case 7: rc = sweepk_launch_k7(a, nstrips, nrb, blocks, s, start, kstop); break;
    case 8: rc = sweepk_launch_k8(a, nstrips, nrb, blocks, s, start, kstop); break;
    case 9: rc = sweepk_launch_k9(a, nstrips, nrb, blocks, s, start, kstop); break;
    case 10: rc = sweepk_launch_k10(a, nstrips, nrb, blocks, s, start, kstop); break;
    case 11: rc = sweepk_launch_k11(a, nstrips, nrb, blocks, s, start, kstop); break;
    default: rc = sweepk_launch_k12(a, nstrips, nrb, blocks, s, start, kstop); break;
    }
    SMI_TRY(rc);
    if (after) SMI_HIP_CHECK(hipEventRecord(after, s));
    if (marker) SMI_TRY(prof_end(tok, s));
    return SMI_SUCCESS;
}

}  // namespace smi
