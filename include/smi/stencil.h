/*
 * stencil.h -- the stencil_smi hot path: 4-point Jacobi with streamed halos.
 *
 * Replaces the stencil_smi application's device pipeline
 *   Read / Stencil / Write            examples/kernels/stencil_smi.cl:20-234
 *   Convert{Send,Receive}{Top,Bottom,Left,Right}
 *                                     examples/kernels/stencil_smi.cl:236-386
 * and the host decomposition (rank = i_px*PY + i_py, tile rows
 * [i_px*X_LOCAL, ..), cols [i_py*Y_LOCAL, ..))
 *                                     examples/host/stencil_smi.cpp:48-62,133-134
 * Arithmetic contract (bit-exact): interior cell
 *   out = 0.25f * (((S + W) + E) + N)    S=x[i+1][j] W=x[i][j-1] E=x[i][j+1] N=x[i-1][j]
 * in IEEE fp32 round-to-nearest with no contraction (stencil_smi.cl:153-156);
 * cells on the global edge are copied unchanged (stencil_smi.cl:143-151).
 *
 * Layout: a rank's tile is x_local rows of y_local fp32, row-major, dense
 * (row pitch = y_local), 16-byte aligned; y_local must be a multiple of 4.
 */
#ifndef SMI_STENCIL_H
#define SMI_STENCIL_H

#include "communicator.h"

#ifdef __cplusplus
extern "C" {
#endif

/* How a tile side is treated by one sweep. */
typedef enum {
    SMI_SIDE_COPY = 0,  /* side lies on the global edge: copy its cells      */
    SMI_SIDE_HALO = 1,  /* neighbour values come from the halo vector        */
    SMI_SIDE_SKIP = 2   /* leave the side's cells unwritten (computed apart) */
} SMI_SideMode;

/* Side order in the arrays below. */
enum { SMI_TOP = 0, SMI_BOTTOM = 1, SMI_LEFT = 2, SMI_RIGHT = 3 };

/* One Jacobi step of one tile, enqueued on `stream`.
 *   halo[SMI_TOP] / halo[SMI_BOTTOM]: y_local values of the row above / below
 *   halo[SMI_LEFT] / halo[SMI_RIGHT]: x_local values of the column left/right
 * (required, i.e. non-NULL, exactly for sides in SMI_SIDE_HALO mode).
 * send_left / send_right (nullable) receive the tile's new first / last
 * column, packed -- the fused equivalent of Write's tee into send_left /
 * send_right (stencil_smi.cl:201-224).  `in` and `out` must not overlap. */
int smi_stencil_step(const float *in, float *out, int x_local, int y_local,
                     const int mode[4], const float *const halo[4],
                     float *send_left, float *send_right, SMI_Stream stream);

/* Full run of the stencil_smi program on this rank's tile: `timesteps`
 * Jacobi steps over the PX x PY decomposition of `comm` (PX*PY == size),
 * halos exchanged every step with the four neighbours through RCCL on a
 * dedicated stream, overlapped with the interior sweep.  buf0 holds the
 * initial tile; buf1 is scratch of the same size.  On return *result_index
 * (0 or 1) names the buffer holding the final tile (like the reference's
 * half timesteps%2, stencil_smi.cpp:344; with fusion the index is
 * (K-step passes + pairs + remaining single steps) % 2).  Asynchronous w.r.t. the host
 * except for transport rendezvous and, with neighbours, the K-step passes'
 * pass-boundary join: before enqueueing interior(t) the host waits for the
 * band kernel of pass t-1 (it ends inside interior(t-1)), so the call returns
 * about one pass before the GPU finishes.  With neighbours the interior runs
 * on `stream` if that is at the highest stream priority, else on a
 * highest-priority stream of the communicator joined to `stream` at the start
 * and end of the call (a normal-priority stream can share a hardware queue
 * with RCCL's streams).  Results are identical either way. */
int smi_stencil_run(SMI_Comm comm, float *buf0, float *buf1, int x_local,
                    int y_local, int px, int py, int timesteps,
                    SMI_Stream stream, int *result_index);

/* Tuning knobs of the sweep kernel (row-block height, rows in flight per
 * wave, non-temporal stores, 1 = overlap halo exchange with the interior).
 * Pass <= 0 / < 0 to keep a value.  Bit-exact results for every setting. */
int smi_stencil_set_tuning(int rows_per_wave, int rows_in_flight,
                           int nontemporal_stores, int overlap);
int smi_stencil_get_tuning(int *rows_per_wave, int *rows_in_flight,
                           int *nontemporal_stores, int *overlap);

/* Temporal blocking: steps_per_pass = K in 1..20 fuses up to K Jacobi steps
 * into one pass over HBM (same per-cell arithmetic, bit-identical result).
 * K = 13..20 runs the rotating-ring sweep, which needs a sweep rectangle
 * of at least 4K rows (the tile, or a multi-rank interior: the tile minus K
 * rows per side with a neighbour); K is clipped to 12 otherwise.
 * Multi-rank runs then exchange depth-K halos -- K rows / KC = 4 ceil(K/4)
 * columns per side neighbour and a K x KC corner block per diagonal
 * neighbour -- once per K steps; a band kernel computes the halo-facing bands
 * (K rows / KC columns deep) while the interior sweep runs.  A run is planned as K-step passes;
 * a remainder r = timesteps % K >= 3 is spread over ceil(timesteps / K)
 * passes balanced to within one step (20 = 10 + 10), r = 1 or 2 adds a pair
 * and/or a single step (smi_stencil_plan).  In a multi-rank run K is
 * clipped to half the smaller tile side; tiles smaller than 4 x 8 run single
 * steps only.
 * rows_per_wave: rows per wave of the active fused kernel (K >= 3: -1 =
 * automatic, one round of resident waves); rows_in_flight (1, 2, 4 or 8)
 * tunes the two-step kernel and is ignored for K >= 3.  Pass 0 to keep. */
int smi_stencil_set_fusion(int steps_per_pass, int rows_per_wave, int rows_in_flight);
int smi_stencil_get_fusion(int *steps_per_pass, int *rows_per_wave, int *rows_in_flight);

/* Multi-rank K-step passes: the interior sweep runs beside the band kernel
 * (the halo-facing bands, on the comm stream) and the exchange.
 * reserve_waves = wave slots the interior sweep leaves free for them, and
 * the band kernel then runs as that many waves looping over its segments
 * (0 = none reserved: one band wave per segment, run in the interior's
 * tail), interior_rounds =
 * rounds of resident waves the interior sweep is cut into (default 1).  Pass
 * < 0 to keep.  Scheduling only: bit-identical results for every setting. */
int smi_stencil_set_bands(int reserve_waves, int interior_rounds);
int smi_stencil_get_bands(int *reserve_waves, int *interior_rounds);

/* Multi-rank K-step passes with K >= 13 (scheduling only, bit-neutral): the
 * kernel that computes the halo-facing bands.  1 (default) = the lean kernel
 * (<= 64 VGPRs, one workgroup per CU, its levels staged through LDS) that
 * runs beside the interior sweep; 0 = one wave per band segment, which only
 * finds wave slots in the interior's tail.  lean = -1 keeps the setting. */
int smi_stencil_set_band_kernel(int lean);
int smi_stencil_get_band_kernel(int *lean);

/* Multi-rank K-step passes (scheduling only, bit-neutral): how interior(t)
 * is ordered after the band kernel of pass t-1.  1 (default) = on the host:
 * smi_stencil_run waits for band(t-1) to finish (it ends inside
 * interior(t-1)) and then enqueues interior(t) with no wait packet between
 * two interiors (~5 us per pass less than a device-side wait); the host is
 * then about one pass ahead of the GPU, so a host thread held up for longer
 * than one pass (~150 us at 8192^2, K = 20) idles the GPU for the excess.
 * 0 = on the device: a stream wait per pass; the host enqueues the whole
 * run without waiting and absorbs host stalls of any length behind the
 * queued passes, at ~3 % more GPU time per pass.
 * host_join = -1 keeps the setting. */
int smi_stencil_set_join(int host_join);
int smi_stencil_get_join(int *host_join);

/* The rotating-ring sweep (K = 13..20) launches one round of waves whose
 * row blocks are shortened where a wave has more work per row: ce16 / rev16
 * = the extra work of a wave holding a global-edge column / of the
 * upward-walking bottom block, in 16ths of a plain wave's; waves = the
 * launch's waves (0 = every resident wave slot).  Pass < 0 to keep.
 * Scheduling only: bit-identical results for every setting. */
int smi_stencil_set_deep(int ce16, int rev16, int waves);
int smi_stencil_get_deep(int *ce16, int *rev16, int *waves);

/* The rotating-ring sweep's work split for one K-step pass (K = 13..20) of a
 * rows x cols tile whose sides with a neighbour are set in side_mask (bit 0
 * top, 1 bottom, 2 left, 3 right; the sweep then covers the tile minus K rows
 * / KC columns there, as in smi_stencil_run): waves launched, column strips,
 * row blocks per interior strip and per edge-column strip, and the output
 * rows of the shortest block (every block must exceed K).  Host only; with
 * no device, set the launch's waves first (smi_stencil_set_deep). */
int smi_stencil_deep_geometry(int rows, int cols, int K, int side_mask, int *waves, int *strips, int *row_blocks,
                              int *row_blocks_edge, int *min_block_rows);

/* One phase of a planned run: `passes` launches of `steps_per_pass` steps. */
typedef struct {
    int steps_per_pass;
    int passes;
} SMI_StencilPhase;

/* The schedule smi_stencil_run follows on `rank` of a px x py decomposition
 * of x_local x y_local tiles under the current fusion setting, computed on
 * the host (no device needed): the phases in order (4 always suffice), the
 * neighbour ranks top, bottom, left, right, top-left, top-right,
 * bottom-left, bottom-right (-1 on the global edge; nullable; the rank map
 * of stencil_smi.cpp:133-134) and the index of the buffer that will hold
 * the result (nullable). */
int smi_stencil_plan(int x_local, int y_local, int px, int py, int rank, int timesteps,
                     SMI_StencilPhase *phases, int max_phases, int *nphases, int neighbours[8],
                     int *result_index);

#ifdef __cplusplus
}
#endif
#endif /* SMI_STENCIL_H */
