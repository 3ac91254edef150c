// stencild.hip -- host side of the deep K-step sweep (kernel: stencild.h,
// one instantiation per K in stencild_k<K>.hip, SWEEPD_MIN <= K <= SWEEPD_MAX).
#include "stencil_common.h"

namespace smi {

#define SMI_SWEEPD_DECL(K)                                                                            \
    int sweepd_launch_k##K(const SweepKArgs &a, const SweepDGeom &g, int blocks, hipStream_t s,          \
                           hipEvent_t start, hipEvent_t stop);                                        \
    int sweepd_resident_k##K();
SMI_SWEEPD_DECL(13)
SMI_SWEEPD_DECL(14)
SMI_SWEEPD_DECL(15)
SMI_SWEEPD_DECL(16)
SMI_SWEEPD_DECL(17)
SMI_SWEEPD_DECL(18)
SMI_SWEEPD_DECL(19)
SMI_SWEEPD_DECL(20)

static int resident_waves(int K) {
    switch (K) {
    case 13: return sweepd_resident_k13();
    case 14: return sweepd_resident_k14();
    case 15: return sweepd_resident_k15();
    case 16: return sweepd_resident_k16();
    case 17: return sweepd_resident_k17();
    case 18: return sweepd_resident_k18();
    case 19: return sweepd_resident_k19();
    default: return sweepd_resident_k20();
    }
}

int sweepd_window_cols(int K) { return 256 - 8 * ((K + 3) / 4); }

bool sweepd_fits(int K, const SweepKArgs &a) {
    // two row blocks of at least K rows each even for a lone strip
    return K >= SWEEPD_MIN && K <= SWEEPD_MAX && a.row_hi - a.row_lo >= 4 * K && a.cols >= 8;
}

// Strips and row blocks (stencild.h, SweepDGeom).  One round of resident
// waves (or g_tune.deep_waves), the edge-column strips and the bottom
// blocks shortened by their measured extra cost (g_tune.deep_ce16 /
// deep_rev16, in 16ths of a block's work).
int sweepd_geometry(int K, const SweepKArgs &a, int reserve, SweepDGeom *g) {
    const int KC = 4 * ((K + 3) / 4), SW = sweepd_window_cols(K);
    const int cs0 = a.col_lo & ~31;
    SweepDGeom r{};
    r.nstrips = (a.col_hi - cs0 + SW - 1) / SW;
    r.ce[0] = r.ce[1] = r.ce[2] = r.ce[3] = -1;
    int nce = 0;
    r.int0 = -1;
    for (int s = 0; s < r.nstrips; ++s) {
        const int cs = cs0 + s * SW;
        const bool ce = (a.gL && cs - KC <= 0) || (a.gR && cs - KC + 256 >= a.cols);
        if (ce) {
            SMI_ARG_CHECK(nce < 4, "sweepd: more than four edge-column strips");
            r.ce[nce++] = s;
        } else {
            if (r.int0 < 0) r.int0 = s;
            ++r.n_int;
        }
    }
    if (r.int0 < 0) r.int0 = 0;
    // interior strips are one contiguous range (edge-column strips sit at the ends)
    for (int k = 0; k < nce; ++k)
        SMI_ARG_CHECK(r.ce[k] < r.int0 || r.ce[k] >= r.int0 + r.n_int, "sweepd: edge-column strip inside the interior");
    const int out_rows = a.row_hi - a.row_lo;
    const int ce16 = 16 + std::max(0, g_tune.deep_ce16);
    r.wlast = std::max(4, std::min(16, 256 / (16 + std::max(0, g_tune.deep_rev16))));
    int waves = g_tune.deep_waves > 0 ? g_tune.deep_waves : resident_waves(K);
    SMI_ARG_CHECK(waves > 0, "sweepd: occupancy query failed");
    if (reserve > 0) waves = std::max(64, waves - reserve);
    int nrb = std::max(1, (int)((long)waves * 16 / ((long)r.n_int * 16 + (long)nce * ce16)));
    const bool both = a.gT && a.gB;
    // every block at least K rows (the shortest is a weighted bottom block)
    auto shortest = [&](const SweepDGeom &q) {
        const int nbmax = nce ? q.nrb_ce : q.nrb;
        const long den = (long)(nbmax - 1) * 16 + (a.gB ? q.wlast : 16);
        return (long)out_rows * std::min(16, a.gB ? q.wlast : 16) / den;
    };
    for (;; --nrb) {
        r.nrb = std::max(nrb, both ? 2 : 1);
        r.nrb_ce = std::max(r.nrb, r.nrb * ce16 / 16);
        if (shortest(r) - 1 >= K) break;
        if (nrb <= (both ? 2 : 1)) {
            // a short tile (down to 4K rows, sweepd_fits): no balancing
            // weights, every strip in the same equal blocks
            r.nrb_ce = r.nrb;
            r.wlast = 16;
            SMI_ARG_CHECK(shortest(r) - 1 >= K, "sweepd: tile too short for this K");
            break;
        }
    }
    r.tasks = r.n_int * r.nrb + nce * r.nrb_ce;
    *g = r;
    return SMI_SUCCESS;
}

int launch_sweepd(int K, const SweepKArgs &a, int reserve, hipStream_t s, hipEvent_t start, hipEvent_t stop) {
    SMI_ARG_CHECK(sweepd_fits(K, a), "sweepd: K out of range or tile too short");
    SMI_ARG_CHECK(a.cols % 4 == 0 && a.col_lo % 4 == 0 && a.col_hi % 4 == 0, "sweepd: columns not float4 aligned");
    SMI_ARG_CHECK(a.row_lo >= 0 && a.row_hi <= a.rows && a.col_lo >= 0 && a.col_hi <= a.cols,
                  "sweepd: output rectangle outside the tile");
    SweepDGeom g;
    SMI_TRY(sweepd_geometry(K, a, reserve, &g));
    const int blocks = (g.tasks + 3) / 4;
    switch (K) {
    case 13: return sweepd_launch_k13(a, g, blocks, s, start, stop);
    case 14: return sweepd_launch_k14(a, g, blocks, s, start, stop);
    case 15: return sweepd_launch_k15(a, g, blocks, s, start, stop);
    case 16: return sweepd_launch_k16(a, g, blocks, s, start, stop);
    case 17: return sweepd_launch_k17(a, g, blocks, s, start, stop);
    case 18: return sweepd_launch_k18(a, g, blocks, s, start, stop);
    case 19: return sweepd_launch_k19(a, g, blocks, s, start, stop);
    default: return sweepd_launch_k20(a, g, blocks, s, start, stop);
    }
}

}  // namespace smi
