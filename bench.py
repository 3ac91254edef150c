#!/usr/bin/env python3
"""bench.py -- stencil_smi Jacobi GCell/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--fake-host]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

With N > 1 and no WORLD_SIZE in the environment, bench.py launches its own
ranks (the reference runs `mpirun -np 8 ./stencil_smi_host`, README.md:96):
the parent starts N child processes of itself with subprocess before anything
touches the GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in
their environment; it never execs), forwards rank 0's result line, and exits
non-zero if a child fails or outlives --launch-timeout.  --fake-host (implied
when fewer GPUs than ranks are visible) puts every rank on GPU 0 with its own
NCCL_HOSTID, so RCCL moves the halos over its socket transport: a functional
rehearsal of the multi-process path on a one-GPU box, timings meaningless.

A "step" is one Jacobi timestep over the whole job's grid.  N=1 runs
BASELINE config 2 (8192x8192 fp32 on one GPU, no halo exchange).  N>1 runs
weak scaling with an 8192x8192 tile per GPU on the stencil_smi decomposition
(1x2, 2x2, 2x4; rank = i_px*PY + i_py), halos exchanged every step through
RCCL over xGMI, overlapped with the interior sweep.  Inputs are resident in
HBM before the timed region; the timed region is exactly K steps bracketed by
a barrier + device synchronize on both sides; the time is the max over ranks.

A run of T steps is planned as ceil(T / 20) sweep passes of at most 20 steps
(passes of more than 12 steps run the rotating-ring sweep, stencild.h, on
single tiles and on multi-rank interiors alike; a tile too small for a deep
pass -- fewer than 4K rows in its sweep rectangle -- clips K to 12), balanced to within one step
when T % 20 >= 3 (config.plan; the driver's 20 steps are one pass).  Before the timed
region every kernel of that plan launches once and untimed runs of the same
plan repeat for at least --warmup-ms (GPU clock settling; with N > 1 every rank
runs the same number of them).

The JSON line also carries:
  roofline      -- the stencil kernel with the largest measured time in the
                   timed region (HIP events on the launch stream: one marker
                   between back-to-back single-tile passes, so each launch is
                   timed from the end of the previous one; a multi-rank pass
                   is timed by its own dispatch) and every kernel's share of the
                   region.  achieved = the pass's compulsory bytes (every
                   stored cell read once and written once, 8 B) / its average
                   duration, frac = achieved / the 8 TB/s HBM3E peak;
                   `traffic` = the HBM bytes per launch from the rocprofv3 PMC
                   passes committed under profiles/ and hbm_frac = traffic /
                   launch time / peak (over-fetch included); cell_step_GBs =
                   8 B per cell-STEP x K steps per launch / launch time
                   (temporal blocking, not a fraction of peak);
                   kernel_avg_ms is cross-checked against the rocprofv3
                   --kernel-trace --stats summary of the driver's own command
                   (profiles/rocprof_driver_cmd.json)
  cpu_baseline  -- the oracle's C restatement of the reference stencil
                   (OpenMP, every thread of this job's CPU share) timed on
                   this host on a bounded sample (rank 0, N=1 only), with the
                   CPU model / nproc and the serial Reference()-order and
                   rank-decomposed (emulator) legs; aux.cpu: reduce and
                   gesummv CPU legs
  halo          -- (N>1) xGMI bytes per step of the halo exchange and the
                   per-link rate the measured step time demands
  aux           -- measured after the timed stencil region (skip: --no-aux):
                   gesummv 32768^2 row-sharded over the N GPUs (BASELINE
                   config 5) and, for N>1, SMI_Reduce int32/fp32 and SMI_Bcast
                   at 4 KiB-256 MiB (config 4) with algbw vs the xGMI bound,
                   and the p2p bandwidth/latency microbenchmarks on one link,
                   each with mean / stddev / 99 % CI over its runs (the
                   reference harness's statistics);
                   bounded by a watchdog so the stencil line always prints
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
VALU_PEAK_TADDS = 78.6         # MI355X_MICROARCH.md: FP32 vector 157.3 TFLOPS spec (FMA = 2) -> adds/s
BYTES_PER_CELL = 8             # one fp32 read + one fp32 write per cell per step
TILE = 8192                    # per-GPU tile edge (BASELINE config 2 / weak scaling)
DECOMP = {1: (1, 1), 2: (1, 2), 4: (2, 2), 8: (2, 4), 16: (4, 4)}
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_stencil_sweep.json")
# rocprofv3 --kernel-trace --stats of the driver's own command, summarised by
# tools/rocprof_summary.py (kernel -> avg duration), cited next to the line's
# own HIP-event timing of the same kernel
ROCPROF_FILE = os.path.join(ROOT, "profiles", "rocprof_driver_cmd.json")
XGMI_LINK_GBS = 153.6          # MI355X Infinity Fabric: 7 links x 153.6 GB/s per GPU
GESUMMV_N = 32768              # BASELINE config 5
COLL_BYTES = (4 << 10, 1 << 20, 64 << 20, 256 << 20)   # BASELINE config 4 span
AUX_BUDGET_S = 120.0           # watchdog on the auxiliary measurements
WARMUP_MS = 50.0               # untimed warm-up floor (GPU clock settling)
PARITY_MAX_STEPS = 64          # timed runs up to this many steps are re-run and checked whole
PARITY_BOUNDED_STEPS = 48      # longer runs: the first 48 steps of the same pass structure


def kernel_label(kind: int, tag: int) -> str:
    from smi_amd import profiling
    if kind == profiling.SWEEPK and tag > 12:
        return f"sweepd_kernel<{tag}> (smi_amd/csrc/stencild.h, rotating-ring sweep, {tag} Jacobi steps per launch)"
    if kind == profiling.SWEEPK:
        return f"sweepk_kernel<{tag}> (smi_amd/csrc/stencilk.h, {tag} Jacobi steps per launch)"
    if kind == profiling.SWEEP and tag == 2:
        return "sweep2_kernel (smi_amd/csrc/stencil2.hip, two Jacobi steps per launch)"
    if kind == profiling.SWEEP:
        return "sweep_kernel (smi_amd/csrc/stencil.hip, one Jacobi step per launch)"
    return "halo-band kernels (bandk_kernel<K> in smi_amd/csrc/stencil_bandk.h, ring2, edge)"


def decomposition(n: int) -> tuple[int, int]:
    if n in DECOMP:
        return DECOMP[n]
    px = int(np.sqrt(n))
    while n % px:
        px -= 1
    return px, n // px


def host_cpu() -> dict:
    """The host's processor: model (/proc/cpuinfo), nproc, the CPUs this
    process may run on, and the thread count the CPU legs use (the box's
    OMP_NUM_THREADS share when set, else every CPU of the affinity mask)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    threads = int(omp) if omp.isdigit() and int(omp) > 0 else affinity
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": affinity, "threads": threads}


def _time_loop(fn, budget_s: float, min_reps: int = 1):
    """Repeat fn until budget_s of wall time (at least min_reps); returns
    (reps, seconds)."""
    fn()  # warm: page faults, thread pool
    reps, dt = 0, 0.0
    while dt < budget_s or reps < min_reps:
        t0 = time.perf_counter()
        fn()
        dt += time.perf_counter() - t0
        reps += 1
    return reps, dt


def cpu_baseline(budget_s: float = 2.0) -> dict:
    """CPU baselines of SURVEY §8(d) / BASELINE.md §3, all on the oracle's C
    restatement (the reference's own CPU path -- Intel FPGA emulator + MPI --
    cannot be built here or on the box):
      value       -- the stencil on every host thread this job may use
                     (OpenMP), 8192^2 tile stepped in place between two
                     preallocated buffers for ~budget_s (no allocation in
                     the timed calls), on the job's CPU quota;
      legs.serial_reference_order -- the host Reference() loop order
                     (examples/host/stencil_smi.cpp:33-46) on 1 core;
      legs.emulator_config1 / emulator_2x4 -- the rank-decomposed program
                     (Read/Stencil/Write per rank, halo queues) run
                     threads-as-ranks, one thread per rank (the reference runs
                     one MPI process per rank, README.md:84-97): config 1
                     (256^2, 2x2, T=32, 4 threads) and a 2x4 grid of 1024^2
                     tiles (8 threads); the same program on 1 core beside
                     each."""
    import oracle
    cpu = host_cpu()
    threads = cpu["threads"]
    g = oracle.init_uniform(TILE, TILE, seed=42)
    # two preallocated, first-touched buffers stepped in place: the timed
    # calls allocate nothing (round 4 timed a malloc + first touch of 768 MiB
    # per 4-step chunk and understated the CPU by ~3.7x)
    bufs = (g, np.empty_like(g))

    def rate(thr: int, budget: float) -> tuple[float, int, float]:
        oracle.stencil_steps(bufs[0], bufs[1], 2, threads=thr)  # warm: pages, thread pool
        chunk, steps, dt = 4, 0, 0.0
        while dt < budget:
            t0 = time.perf_counter()
            oracle.stencil_steps(bufs[0], bufs[1], chunk, threads=thr)  # even: result back in bufs[0]
            dt += time.perf_counter() - t0
            steps += chunk
            chunk = min(chunk * 2, 64)
        return TILE * TILE * steps / dt / 1e9, steps, dt

    value, steps, dt = rate(threads, budget_s)
    out = {
        "value": round(value, 3),
        "unit": "GCell/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{TILE}x{TILE} fp32 Jacobi, {steps} steps, OpenMP C restatement "
                  f"(oracle/smi_oracle.c oracle_stencil_steps: two preallocated buffers stepped in place) "
                  f"of stencil_smi.cl:117-165, {dt:.1f} s wall on {threads} threads "
                  f"(this job's CPU quota, OMP_NUM_THREADS; the affinity mask spans {cpu['affinity_cpus']} CPUs "
                  f"shared with other jobs)",
        **cpu,
    }
    # no leg on every CPU of the affinity mask: the box's mask spans the whole
    # machine (256 CPUs) while the job's CPU quota is OMP_NUM_THREADS (16), so
    # such a leg measures oversubscription, not the CPU (round 5 read 0.47
    # GCell/s on 256 threads against 48 on 16)
    legs = {}
    del bufs
    gs = g[:2048, :2048].copy()
    reps, dt = _time_loop(lambda: oracle.stencil(gs, 2, order="host", threads=1), 1.5)
    legs["serial_reference_order"] = {
        "GCells": round(2048 * 2048 * 2 * reps / dt / 1e9, 4), "cores": 1,
        "sample": f"2048x2048, {2 * reps} steps in {dt:.2f} s, host Reference() order (stencil_smi.cpp:33-46)"}
    for name, (X, Y, PX, PY) in (("emulator_config1", (256, 256, 2, 2)), ("emulator_2x4", (2048, 4096, 2, 4))):
        ge = oracle.init_uniform(X, Y, seed=5)
        leg = {"sample": f"{X}x{Y} as {PX}x{PY} ranks of {X // PX}x{Y // PY}, 32 steps", "ranks": PX * PY}
        for thr in (PX * PY, 1):
            reps, dt = _time_loop(lambda: oracle.stencil_decomposed(ge, 32, PX, PY, threads=thr), 0.5, 3)
            key = "threads_as_ranks" if thr > 1 else "one_core"
            leg[key] = {"GCells": round(X * Y * 32 * reps / dt / 1e9, 4), "ms_per_program": round(dt / reps * 1e3, 3),
                        "threads": thr, "programs": reps}
        legs[name] = leg
    out["legs"] = legs
    return out


def cpu_aux_legs(budget_s: float = 1.0) -> dict:
    """CPU legs of the auxiliary configs on the oracle, threads-as-ranks
    (SURVEY §8(d)): the canonical reduce fold (reduce.cl:42-148) of 8
    contributions folded as 8 owner chunks on 8 threads, the broadcast
    (bcast.cl:3-111) of one rank's buffer into 7 others packet by packet on 8
    threads, and one 8-way gesummv row shard (4096 x 32768,
    gesummv_rank0.cl:53-203) on every host thread."""
    import oracle
    cpu = host_cpu()
    n, count = 8, 16 << 20
    c = np.random.default_rng(3).random((n, count), dtype=np.float32)
    reps, dt = _time_loop(lambda: oracle.reduce(c, 2, 0, threads=n), budget_s)
    red = {"GBs": round(4 * (n + 1) * count * reps / dt / 1e9, 3), "cores": n, "threads_as_ranks": n,
           "sample": f"{n} x {count} fp32 add as {n} owner chunks, {reps} folds in {dt:.2f} s "
                     f"(algorithmic bytes 4(n+1) per element)"}
    reps, dt = _time_loop(lambda: oracle.bcast(c, n - 1, threads=n), budget_s)
    bc = {"GBs": round(4 * count * reps / dt / 1e9, 3), "cores": n, "threads_as_ranks": n,
          "sample": f"{4 * count >> 20} MiB fp32 from rank {n - 1} to {n - 1} ranks in 28-byte packets, "
                    f"{reps} broadcasts in {dt:.2f} s (algbw: message bytes / time)"}
    del c
    rows, m = GESUMMV_N // 8, GESUMMV_N
    rng = np.random.default_rng(4)
    A = rng.random((rows, m), dtype=np.float32)
    B = rng.random((rows, m), dtype=np.float32)
    x = rng.random(m, dtype=np.float32)
    reps, dt = _time_loop(lambda: oracle.gesummv(A, B, x, 1.5, 0.5, threads=cpu["threads"]), budget_s)
    gem = {"GBs": round(4 * (2 * rows * m + m + rows) * reps / dt / 1e9, 3), "cores": cpu["threads"],
           "ms": round(dt / reps * 1e3, 3), "sample": f"{rows}x{m} row shard (A and B), {reps} runs"}
    return {"reduce_fold_f32": red, "bcast_f32": bc, "gesummv_shard": gem, "kind": "port", **cpu}


def pmc_traffic(cells: int, steps_per_launch: int) -> float | None:
    """HBM bytes per sweep launch from the committed rocprofv3 PMC summary,
    if it was measured on this same per-GPU tile and kernel."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
        for e in d.get("entries", [d]):
            if int(e.get("cells", -1)) == cells and int(e.get("steps_per_launch", 1)) == steps_per_launch:
                return float(e["hbm_bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        pass
    return None


def rocprof_avg(kernel_symbol: str) -> dict | None:
    """The committed rocprofv3 summary's average duration of this kernel (the
    driver's bench command under --kernel-trace --stats), if present."""
    try:
        with open(ROCPROF_FILE) as f:
            d = json.load(f)
        k = d["kernels"].get(kernel_symbol)
        if k:
            return {"avg_ms": k["avg_ms"], "calls": k["calls"], "command": d.get("command"),
                    "source": d.get("source")}
    except (OSError, ValueError, KeyError):
        pass
    return None


def halo_report(PX: int, PY: int, X: int, Y: int, K: int, ms_per_step: float) -> dict:
    """xGMI traffic of the halo exchange for the busiest rank: per K-step pass
    a rank sends K rows of Y fp32 to each vertical neighbour, K columns of X
    fp32 to each horizontal neighbour and a KxK block to each diagonal
    neighbour (stencil_smi.cl:183-224 streams the same rows/columns one step
    at a time).  Every neighbour is its own xGMI link, so the per-link rate
    is the largest single-neighbour payload over the step time."""
    best = None
    for ipx in range(PX):
        for ipy in range(PY):
            nv = (ipx > 0) + (ipx < PX - 1)
            nh = (ipy > 0) + (ipy < PY - 1)
            nd = sum(1 for dx in (-1, 1) for dy in (-1, 1)
                     if 0 <= ipx + dx < PX and 0 <= ipy + dy < PY)
            b = 4 * (nv * Y + nh * X) + 4 * nd * K  # per step (KxK block / K steps)
            if best is None or b > best[0]:
                best = (b, nv, nh, nd)
    b, nv, nh, nd = best
    link_b = 4 * max(Y if nv else 0, X if nh else 0)
    link_rate = link_b / (ms_per_step * 1e-3) / 1e9
    return {
        "bytes_per_step_busiest_rank": b,
        "neighbours": {"vertical": nv, "horizontal": nh, "diagonal": nd},
        "link_GBs_needed": round(link_rate, 2),
        "link_peak_GBs": XGMI_LINK_GBS,
        "link_frac": round(link_rate / XGMI_LINK_GBS, 4),
        "note": "per-link halo rate the measured step time demands; the exchange is latency-bound "
                "(K rows/columns per pass), hidden behind the interior sweep",
    }


def _timed(fn, iters: int, barrier, world: int) -> float:
    """Seconds per call: one untimed call, then `iters` calls bracketed by a
    barrier + device sync; max over ranks."""
    import torch
    import torch.distributed as dist
    fn()
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    barrier()
    dt = (time.perf_counter() - t0) / iters
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t[0])
    return dt


def _timed_runs(fn, runs: int, barrier, world: int) -> dict:
    """The reference harness's statistics (microbenchmarks/host/
    reduce_benchmark.cpp:120-155): `runs` runs, each bracketed by a barrier +
    device sync and timed as the max over ranks; mean, population stddev and
    the 99 % confidence half-width 2.58 * stddev / sqrt(runs), in us."""
    import torch
    import torch.distributed as dist
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(runs):
        barrier()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    if world > 1:
        t = torch.tensor(ts, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ts = [float(v) for v in t]
    us = np.array(ts) * 1e6
    mean = float(us.mean())
    sd = float(np.sqrt(((us - mean) ** 2).mean()))
    ci = 2.58 * sd / np.sqrt(len(us))
    return {"us": round(mean, 2), "stddev_us": round(sd, 2), "ci99_us": round(ci, 2),
            "ci99_pct_of_mean": round(100 * ci / mean, 2), "runs": len(us), "mean_s": mean * 1e-6}


def seeded_tile(rank: int, X: int, Y: int) -> np.ndarray:
    """The synthetic input of `rank`'s tile (uniform [0,1) fp32, seed 1000+rank)."""
    return np.random.default_rng(1000 + rank).random((X, Y), dtype=np.float32)


def light_cone(rank: int, PX: int, PY: int, X: int, Y: int, T: int, own: np.ndarray):
    """`rank`'s tile extended by T cells on every side that has a neighbour
    (clipped at the global edges), assembled from the seeded tiles of the
    ranks it overlaps, and the slice of it that is the tile itself.  T steps
    of the global stencil on this region are exact on the tile: whatever the
    region's artificial boundary does travels at most one cell per step
    (examples/host/stencil_smi.cpp:391-405 checks the whole grid; this is the
    same check, one rank's share at a time)."""
    ipx, ipy = rank // PY, rank % PY
    r0, r1 = max(0, ipx * X - T), min(PX * X, (ipx + 1) * X + T)
    c0, c1 = max(0, ipy * Y - T), min(PY * Y, (ipy + 1) * Y + T)
    ext = np.empty((r1 - r0, c1 - c0), dtype=np.float32)
    for qx in range(r0 // X, (r1 - 1) // X + 1):
        for qy in range(c0 // Y, (c1 - 1) // Y + 1):
            q = qx * PY + qy
            src = own if q == rank else seeded_tile(q, X, Y)
            gr0, gr1 = max(r0, qx * X), min(r1, (qx + 1) * X)
            gc0, gc1 = max(c0, qy * Y), min(c1, (qy + 1) * Y)
            ext[gr0 - r0:gr1 - r0, gc0 - c0:gc1 - c0] = src[gr0 - qx * X:gr1 - qx * X, gc0 - qy * Y:gc1 - qy * Y]
            del src
    return ext, (slice(ipx * X - r0, ipx * X - r0 + X), slice(ipy * Y - c0, ipy * Y - c0 + Y))


def verify_timed_plan(comm, tile, scratch, g_host: np.ndarray, steps: int, PX: int, PY: int, rank: int,
                      world: int) -> dict:
    """Re-run the timed plan (same stencil.run, same T, same decomposition)
    from a kept copy of the seeded input, outside the timed region, and check
    every cell bit for bit against the oracle's C restatement of
    stencil_smi.cl:153-156 (the reference checks every run it times,
    examples/host/stencil_smi.cpp:391-405).  N > 1: each rank checks its own
    tile on its light cone; the ranks agree the verdict over gloo.  Runs of
    more than PARITY_MAX_STEPS steps are checked on the first
    PARITY_BOUNDED_STEPS steps of the same pass structure (same kernels), so
    the check stays within a few seconds of CPU."""
    import torch
    import oracle
    from smi_amd import stencil
    X, Y = g_host.shape
    T = steps if steps <= PARITY_MAX_STEPS else PARITY_BOUNDED_STEPS
    tile.copy_(torch.from_numpy(g_host))
    torch.cuda.synchronize()
    res = stencil.run(comm, tile, T, PX, PY, scratch)
    torch.cuda.synchronize()
    got = res.cpu().numpy()
    t0 = time.perf_counter()
    ext, sl = light_cone(rank, PX, PY, X, Y, T, g_host)
    want = oracle.stencil(ext, T, threads=host_cpu()["threads"])[sl]
    del ext
    oracle_s = time.perf_counter() - t0
    bad = int(np.count_nonzero(got.view(np.uint32) != want.view(np.uint32)))
    cells = got.size
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([bad, cells], dtype=torch.float64)
        dist.all_reduce(t)
        bad, cells = int(t[0]), int(t[1])
    return {"checked": True, "bit_exact": bad == 0, "mismatches": bad, "cells": cells, "steps": T,
            "same_plan_as_timed": T == steps,
            "plan": [{"steps_per_pass": k, "passes": n} for k, n in stencil.plan(X, Y, PX, PY, rank, T)["phases"]],
            "oracle": "oracle/smi_oracle.c (stencil_smi.cl:153-156 order), each rank's tile on its light cone",
            "oracle_s": round(oracle_s, 2)}


def _all_ok(ok: bool, world: int) -> bool:
    """A check made on one rank, agreed by every rank (rank 0 prints)."""
    if world == 1:
        return ok
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if ok else 0])
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def aux_gesummv(comm, world: int, rank: int, stream, barrier) -> dict:
    """BASELINE config 5: y = alpha*A*x + beta*B*x, 32768^2 fp32, rows sharded
    over the ranks (strong scaling), y chunks gathered on rank 0
    (gesummv_rank0.cl:53-203).  Algorithmic bytes 4*(2*N*M + M + N)."""
    import torch
    from smi_amd import gesummv
    n = m = GESUMMV_N
    r0, r1 = gesummv.row_range(n, world, rank)
    gen = torch.Generator(device="cuda").manual_seed(77 + rank)
    A = torch.rand((r1 - r0, m), generator=gen, device="cuda") * 2 - 1
    B = torch.rand((r1 - r0, m), generator=gen, device="cuda") * 2 - 1
    x = torch.ones(m, device="cuda")
    y = torch.empty(n, device="cuda") if rank == 0 else None
    torch.cuda.synchronize()

    def call():
        gesummv.gesummv(comm, A, B, x, n, 1.5, 0.5, y=y, root=0, stream=stream)

    with torch.cuda.stream(stream):
        dt = _timed(call, 10, barrier, world)
    del A, B
    algo = 4 * (2 * n * m + m + n)
    gbs = algo / dt / 1e9
    return {"workload": f"gesummv {n}x{m} fp32, {world}-way row shard, y gathered on rank 0",
            "ms": round(dt * 1e3, 4), "GBs": round(gbs, 1),
            "hbm_frac": round(gbs / (HBM_PEAK_GBS * world), 4)}


def aux_kernels_1gpu() -> dict:
    """N = 1 only: the per-GPU kernels of the 8-GPU configs on one GPU --
    the config-5 row shard (4096 x 32768 A and B through gemv_rows) and the
    smi_reduce owner fold of config 4 (8 contributions of 8 Mi fp32 in
    staging rows 4 KiB apart, as smi_reduce lays them out).  HIP events on
    the launch stream (include/smi/profiling.h)."""
    import torch
    from smi_amd import collectives, gesummv, profiling

    def timed(fn, kern, reps=20):
        fn()
        torch.cuda.synchronize()
        profiling.reset()
        profiling.enable(True)
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        profiling.enable(False)
        ms, n = profiling.read(kern)
        return ms / max(n, 1)

    out = {}
    n, m = GESUMMV_N // 8, GESUMMV_N
    gen = torch.Generator(device="cuda").manual_seed(5)
    A = torch.rand((n, m), generator=gen, device="cuda")
    B = torch.rand((n, m), generator=gen, device="cuda")
    x = torch.rand(m, generator=gen, device="cuda")
    y = torch.empty(n, device="cuda")
    ms = timed(lambda: gesummv.gemv_rows(A, B, x, 1.5, 0.5, y), profiling.GEMV)
    byts = 4 * (2 * n * m + m + n)
    out["gemv_shard8"] = {"kernel": "gemv_split_kernel (smi_amd/csrc/gesummv.hip)", "rows": n, "cols": m,
                          "avg_ms": round(ms, 4), "GBs": round(byts / ms / 1e6, 1),
                          "hbm_frac": round(byts / ms / 1e6 / HBM_PEAK_GBS, 4)}
    del A, B
    cnt, nr, pad = 1 << 23, 8, 1024
    c = torch.rand((nr, cnt + pad), generator=gen, device="cuda")[:, :cnt]
    o = torch.empty(cnt, device="cuda")
    ms = timed(lambda: collectives.reduce_fold(c, "add", o), profiling.REDUCE_FOLD)
    byts = 4 * cnt * (nr + 1)
    out["reduce_fold8"] = {"kernel": "fold_kernel<float,4,ADD> (smi_amd/csrc/collectives.hip)",
                           "contributions": nr, "count": cnt, "row_stride_bytes": 4 * (cnt + pad),
                           "avg_ms": round(ms, 4), "GBs": round(byts / ms / 1e6, 1),
                           "hbm_frac": round(byts / ms / 1e6 / HBM_PEAK_GBS, 4)}
    return out


def aux_p2p(comm, world: int, rank: int, stream, barrier) -> dict:
    """p2p microbenchmarks (microbenchmarks/kernels/bandwidth_*.cl,
    latency_*.cl) over one xGMI link, rank 0 -> rank 1 through smi_send /
    smi_recv: bandwidth at 4 KiB - 256 MiB of doubles 0.1f + i (checked on
    rank 1), and the one-int ping-pong latency (round trip / 2)."""
    import torch
    from smi_amd import collectives
    bw = []
    start = float(np.float32(0.1))
    for nbytes in COLL_BYTES:
        n = nbytes // 8
        if rank == 0:
            buf = start + torch.arange(n, dtype=torch.float64, device="cuda")
        else:
            buf = torch.zeros(n, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()

        def call():
            if rank == 0:
                collectives.send(comm, buf, 1, stream=stream)
            elif rank == 1:
                collectives.recv(comm, buf, 0, stream=stream)

        with torch.cuda.stream(stream):
            st = _timed_runs(call, 30 if nbytes <= (1 << 20) else 10, barrier, world)
        ok = True
        if rank == 1:
            ok = bool((buf == start + torch.arange(n, dtype=torch.float64, device="cuda")).all().item())
        gbs = nbytes / st.pop("mean_s") / 1e9
        row = {"bytes": nbytes, **st, "GBs": round(gbs, 2), "link_frac": round(gbs / XGMI_LINK_GBS, 4)}
        if not _all_ok(ok, world):
            row["error"] = "KAT mismatch on rank 1"
        bw.append(row)
        del buf
    v = torch.zeros(1, dtype=torch.int32, device="cuda")
    trips = 100

    def pingpong():
        for _ in range(trips):
            if rank == 0:
                collectives.send(comm, v, 1, stream=stream)
                collectives.recv(comm, v, 1, stream=stream)
            elif rank == 1:
                collectives.recv(comm, v, 0, stream=stream)
                v.add_(1)
                collectives.send(comm, v, 0, stream=stream)

    with torch.cuda.stream(stream):
        st = _timed_runs(pingpong, 10, barrier, world)
    st.pop("mean_s")
    lat = {k: (round(v / (2 * trips), 3) if k.endswith("_us") or k == "us" else v) for k, v in st.items()}
    return {"pair": [0, 1], "bandwidth": bw, "latency_us": lat["us"], "latency": lat,
            "note": "latency = ping-pong round trip / 2 of one int32 (runs of 100 round trips), stream-ordered "
                    "smi_send/smi_recv; stats per the reference harness (mean, population stddev, 99 % CI)"}


def aux_collectives(comm, world: int, rank: int, stream, barrier) -> list:
    """BASELINE config 4: SMI_Reduce (int32 + fp32 add) and SMI_Bcast, 4 KiB -
    256 MiB per rank.  algbw = message bytes / time; the xGMI bound for the
    owner-chunk reduce (and scatter + all-gather bcast) is n*B_link/2: each
    link carries 2*N/n bytes per direction."""
    import torch
    from smi_amd import collectives
    out = []
    root = world - 1
    for nbytes in COLL_BYTES:
        count = nbytes // 4
        iters = 30 if nbytes <= (1 << 20) else 10
        snd_i = torch.full((count,), rank + 1, dtype=torch.int32, device="cuda")
        snd_f = torch.rand(count, device="cuda")
        rcv = torch.empty(count, dtype=torch.float32, device="cuda") if rank == root else None
        rcv_i = torch.empty(count, dtype=torch.int32, device="cuda") if rank == root else None
        buf = torch.rand(count, device="cuda")
        torch.cuda.synchronize()
        with torch.cuda.stream(stream):
            t_ri = _timed_runs(lambda: collectives.reduce(comm, snd_i, rcv_i, "add", root=root, stream=stream),
                               iters, barrier, world)
            t_rf = _timed_runs(lambda: collectives.reduce(comm, snd_f, rcv, "add", root=root, stream=stream),
                               iters, barrier, world)
            t_b = _timed_runs(lambda: collectives.bcast(comm, buf, root=0, stream=stream), iters, barrier, world)
        sys.stderr.write(f"[bench rank {rank}] aux collectives {nbytes} B done\n")
        ok = True
        if rank == root:  # KAT: sum of (rank + 1) = n(n+1)/2 (microbenchmarks/kernels/reduce.cl:13-24)
            ok = bool((rcv_i == world * (world + 1) // 2).all().item())
        bound = world * XGMI_LINK_GBS / 2
        for op, st in (("reduce_i32_add", t_ri), ("reduce_f32_add", t_rf), ("bcast_f32", t_b)):
            gbs = nbytes / st.pop("mean_s") / 1e9
            out.append({"op": op, "bytes": nbytes, **st, "algbw_GBs": round(gbs, 2),
                        "xgmi_bound_GBs": bound, "xgmi_frac": round(gbs / bound, 4)})
        if not _all_ok(ok, world):
            out.append({"op": "reduce_i32_add", "bytes": nbytes, "error": "KAT mismatch on the root"})
        del snd_i, snd_f, rcv, rcv_i, buf
    return out


def visible_gpus() -> int:
    """GPUs this process may use, counted without initialising HIP: the
    visibility variables when set, else the GPU nodes of the KFD topology."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() not in ("", "-1")])
    base = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for node in os.listdir(base):
            try:
                with open(os.path.join(base, node, "gpu_id")) as f:
                    n += int(f.read().strip() or 0) != 0
            except (OSError, ValueError):
                pass
    except OSError:
        return 0
    return n


def launch_ranks(args, argv: list[str]) -> int:
    """Start `args.gpus` ranks of this script as child processes (never an
    exec: the parent has not touched the GPU and does not), forward rank 0's
    JSON line to stdout, return the first failing child's exit code (0 if
    all succeed).  The children inherit stderr, so their progress lines keep
    the job visibly alive."""
    import signal
    import socket
    import subprocess
    n = args.gpus
    fake = args.fake_host
    if not fake:
        ngpu = visible_gpus()  # without HIP: the parent never touches the GPU
        if ngpu < n:
            fake = True
            sys.stderr.write(f"[bench] {ngpu} GPU(s) visible for {n} ranks: --fake-host\n")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK="0" if fake else str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0",
                   SMI_BENCH_SELF_LAUNCH="1")
        if fake:
            env.update(NCCL_HOSTID=f"smi-bench-host-{r}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1",
                       SMI_BENCH_FAKE_HOST="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                      start_new_session=True))
    deadline = time.monotonic() + args.launch_timeout
    rc = 0
    # rank 0's line is read on a thread (a full pipe must never block it);
    # the children are polled together: the first one to fail takes the
    # others down at once (survivors would sit in RCCL until the deadline)
    out = {}
    reader = threading.Thread(target=lambda: out.setdefault("0", procs[0].stdout.read()), daemon=True)
    reader.start()
    while True:
        codes = [p.poll() for p in procs]
        bad = next((c for c in codes if c not in (None, 0)), None)
        if bad is not None:
            sys.stderr.write(f"[bench] a rank exited with {bad}: stopping the others\n")
            rc = bad
            break
        if all(c == 0 for c in codes):
            break
        if time.monotonic() > deadline:
            sys.stderr.write(f"[bench] ranks outlived --launch-timeout {args.launch_timeout:.0f} s: killed\n")
            rc = 124
            break
        time.sleep(0.2)
    for p in procs:  # each child leads its own process group (start_new_session)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except OSError:
                pass
            p.wait()
    if rc == 0:
        rc = next((p.returncode for p in procs if p.returncode != 0), 0)
    reader.join(timeout=10)
    out0 = out.get("0") or b""
    line = next((ln for ln in out0.decode(errors="replace").splitlines() if ln.startswith("{")), None)
    if line:
        sys.stdout.write(line + "\n")
        sys.stdout.flush()
    elif rc == 0:
        sys.stderr.write("[bench] rank 0 printed no result line\n")
        rc = 1
    return rc


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # ~25 ms of untimed warm-up: the GPU clock needs >10 ms of load to reach
    # its steady state (120 steps after 10 warm-up steps measured ~11 % low,
    # profiles/r01f/bench_warmup_sweep.log); 2400 timed steps = 200 K-step passes
    ap.add_argument("--steps", type=int, default=2400)
    ap.add_argument("--warmup", type=int, default=2400)
    ap.add_argument("--tile", type=int, default=TILE)
    ap.add_argument("--warmup-ms", type=float, default=WARMUP_MS,
                    help="untimed warm-up floor in ms (repeated runs of the timed plan) after the --warmup steps")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip re-running the timed plan from the seeded input and checking it against the oracle")
    ap.add_argument("--no-aux", action="store_true",
                    help="skip the gesummv / reduce / bcast lines measured after the timed stencil region")
    ap.add_argument("--fake-host", action="store_true",
                    help="self-launched ranks all on GPU 0, one NCCL_HOSTID each (RCCL over sockets)")
    ap.add_argument("--launch-timeout", type=float, default=1500.0,
                    help="self-launch: kill every rank after this many seconds")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(args, sys.argv[1:]))

    # stdout carries exactly one line, the result: anything the libraries
    # underneath write there (RCCL's version banner, gloo's connection notes,
    # from C as well as Python) goes to stderr instead
    result_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    import smi_amd
    from smi_amd import profiling, stencil

    t_start = time.perf_counter()

    def log(what):  # progress on stderr (stdout carries only the result line)
        sys.stderr.write(f"[bench rank {os.environ.get('RANK', '0')} +{time.perf_counter() - t_start:.1f}s] {what}\n")
        sys.stderr.flush()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    smi_amd.load()

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        comm = smi_amd.Comm.from_env(device=local)
        log("RCCL communicator up")
    else:
        comm = smi_amd.LocalGroup(1, device=local).comm(0)

    def barrier():
        if world > 1:
            dist.barrier()

    PX, PY = decomposition(world)
    X = Y = args.tile
    g = seeded_tile(rank, X, Y)
    tile = torch.from_numpy(g).cuda()
    scratch = torch.empty_like(tile)
    # the highest priority, like the communicator's comm stream: a stream at
    # normal priority can share a hardware queue with RCCL's own streams, and
    # the library then runs the interior on a stream of its own, joined to
    # this one at the start and end of each run (stencil_run.cpp
    # interior_stream); at the highest priority the interior runs right here
    stream = torch.cuda.Stream(priority=-1)

    fusion = stencil.get_fusion()
    K = fusion["steps_per_pass"]
    plan = stencil.plan(X, Y, PX, PY, rank, args.steps)
    warm_ms = 0.0
    with torch.cuda.stream(stream):
        if args.warmup:
            stencil.run(comm, tile, args.warmup, PX, PY, scratch)
            torch.cuda.synchronize()
            log(f"{args.warmup} warm-up steps done")
        # HIP loads a kernel's code object at its first launch: every kernel
        # of the timed plan (the K-step passes and the remainder pass) runs
        # once outside the timed region ...
        # (with profiling on, so the HIP events the timed region records come
        # from the pool instead of being created inside it)
        profiling.enable(True)
        for k, _ in plan["phases"]:
            stencil.run(comm, tile, k, PX, PY, scratch)
        torch.cuda.synchronize()
        log("every kernel of the plan launched once")
        profiling.enable(False)
        profiling.reset()
        # ... and the GPU clock needs tens of ms of load to settle (120 steps
        # after 10 warm-up steps read ~11 % low, profiles/r01f/
        # bench_warmup_sweep.log): untimed runs until at least --warmup-ms of
        # warm-up has run.  Every rank must run the same number of warm-up runs (each carries
        # halo exchanges that pair up across ranks): with N > 1 the ranks
        # agree after every run whether any of them still needs warm-up.
        # The warm-up runs the timed plan itself, so the kernels the timed
        # region launches are the ones warmed up (code and clocks).
        t_w = time.perf_counter()
        while True:
            more = (time.perf_counter() - t_w) * 1e3 < args.warmup_ms
            if world > 1:
                flag = torch.tensor([1 if more else 0])
                dist.all_reduce(flag, op=dist.ReduceOp.MAX)
                more = bool(flag.item())
            if not more:
                break
            stencil.run(comm, tile, args.steps if args.steps > 0 else max(K, 1) * 4, PX, PY, scratch)
            torch.cuda.synchronize()
        warm_ms = (time.perf_counter() - t_w) * 1e3
        log(f"warm-up floor done ({warm_ms:.1f} ms)")
        # The timed region: exactly --steps steps, profiling off (no marker
        # or event in it), bracketed by a barrier + device sync.
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        stencil.run(comm, tile, args.steps, PX, PY, scratch)
        torch.cuda.synchronize()
        barrier()
        t1 = time.perf_counter()
        # Per-kernel times: an identical repetition of the timed plan right
        # after it, with HIP events on each launch's stream (its wall time is
        # reported beside the timed one, never used for `value`).
        profiling.reset()
        profiling.enable(True)
        torch.cuda.synchronize()
        barrier()
        t2 = time.perf_counter()
        stencil.run(comm, tile, args.steps, PX, PY, scratch)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        profiling.enable(False)
        # Repetition statistics for the headline (never used for `value`):
        # more identical timed regions, each bracketed like the timed one,
        # ~2 s of them at most, 30 at most, 5 at least.
        rep_s = []
        n_rep = max(5, min(30, int(2.0 / max(t1 - t0, 1e-6))))
        if world > 1:
            # every rank must run the same count (each run carries halo
            # exchanges that pair up across ranks): the ranks' own wall times
            # can straddle an integer boundary, so agree on the largest
            flag = torch.tensor([n_rep])
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            n_rep = int(flag.item())
        for _ in range(n_rep):
            barrier()
            torch.cuda.synchronize()
            ta = time.perf_counter()
            stencil.run(comm, tile, args.steps, PX, PY, scratch)
            torch.cuda.synchronize()
            barrier()
            rep_s.append(time.perf_counter() - ta)
    elapsed = t1 - t0
    if world > 1:  # per repetition, the slowest rank's time
        t = torch.tensor(rep_s, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        rep_s = [float(v) for v in t]
    prof_rep_ms = (t3 - t2) * 1e3
    log(f"timed region done: {args.steps} steps in {elapsed * 1e3:.3f} ms (profiled repetition {prof_rep_ms:.3f} ms)")
    # Every stencil kernel launched in the profiled repetition, with its
    # measured time (HIP events around each launch on its own stream); the
    # roofline prices the one that took the most time.
    keys = [(kern, tag) for kern, tag in profiling.entries()
            if kern in (profiling.SWEEP, profiling.SWEEPK, profiling.EDGE)]
    if world > 1:
        # ranks can record different kernels (a tile with neighbours on both
        # sides and no interior left records no sweep): reduce over the union
        every = [None] * world
        dist.all_gather_object(every, keys)
        keys = sorted({tuple(k) for ks in every for k in ks})
    kernels = []
    for kern, tag in keys:
        ms, n, units = profiling.read_tag(kern, tag)
        kernels.append({"kernel": kernel_label(kern, tag), "kind": kern, "tag": tag, "launches": n,
                        "total_ms": ms, "cell_steps": units})
    if world > 1:  # the slowest rank's times, kernel by kernel (0 where a rank has none)
        t = torch.tensor([elapsed] + [k["total_ms"] for k in kernels] + [k["launches"] for k in kernels]
                         + [k["cell_steps"] for k in kernels], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
        nk = len(kernels)
        for i, k in enumerate(kernels):
            k["total_ms"] = float(t[1 + i])
            k["launches"] = int(t[1 + nk + i])
            k["cell_steps"] = float(t[1 + 2 * nk + i])
    timed_ms = elapsed * 1e3
    for k in kernels:
        k["avg_ms"] = k["total_ms"] / max(k["launches"], 1)
        k["share_of_timed_region"] = k["total_ms"] / timed_ms
        # 8 B per cell-STEP: with K steps per pass this is K x the bytes the
        # pass moves (temporal blocking) -- a rate, not a fraction of peak
        k["cell_step_GBs"] = (BYTES_PER_CELL * k["cell_steps"] / (k["total_ms"] * 1e-3) / 1e9
                              if k["total_ms"] > 0 and k["cell_steps"] else None)
    sweeps = [k for k in kernels if k["kind"] != profiling.EDGE]
    dom = max(sweeps, key=lambda k: k["total_ms"]) if sweeps else None

    cells_per_gpu = X * Y
    total_cells = cells_per_gpu * world
    value = total_cells * args.steps / elapsed / 1e9
    rep = np.array([total_cells * args.steps / t / 1e9 for t in rep_s])
    rep_mean = float(rep.mean())
    rep_sd = float(np.sqrt(((rep - rep_mean) ** 2).mean()))
    repeats = {"runs": len(rep), "mean": round(rep_mean, 1), "stddev": round(rep_sd, 1),
               "ci99": round(2.58 * rep_sd / np.sqrt(len(rep)), 1), "min": round(float(rep.min()), 1),
               "median": round(float(np.median(rep)), 1), "max": round(float(rep.max()), 1), "unit": "GCell/s",
               "note": "the timed plan re-run after the timed region, each run bracketed by a barrier + device "
                       "sync, max over ranks; statistics as microbenchmarks/host/reduce_benchmark.cpp:120-155 "
                       "(population stddev, 2.58 sigma / sqrt(runs)); value is the single timed region"}
    if dom:
        spl = dom["tag"]  # steps per launch
        cells_launch = int(round(dom["cell_steps"] / max(dom["launches"], 1) / spl))
        # compulsory bytes of one pass: every cell it stores read once and
        # written once (8 B), whatever the steps per pass
        bytes_launch = BYTES_PER_CELL * cells_launch
        sweep_avg_ms = dom["avg_ms"]
        achieved = bytes_launch / (sweep_avg_ms * 1e-3) / 1e9
        step_gbs = achieved * spl
        kernel_name = dom["kernel"]
    else:
        spl, cells_launch, bytes_launch, sweep_avg_ms, achieved, step_gbs, kernel_name = 0, 0, 0, 0.0, 0.0, 0.0, None
    traffic = pmc_traffic(cells_per_gpu, spl) if dom else None
    traffic_basis = "measured (rocprofv3 PMC, this tile and kernel)" if traffic else None
    if traffic and world > 1 and cells_launch:
        # the multi-rank interior sweep covers the tile minus K-wide halo
        # bands: the 1x1 pass's measured bytes scaled by the cells it stores
        traffic *= cells_launch / cells_per_gpu
        traffic_basis = "1x1 PMC pass scaled by the interior's cells per launch (estimate)"
    out = {
        "metric": "Jacobi stencil GCell/s (8192^2 fp32 per GPU)",
        "value": round(value, 2),
        "unit": "GCell/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (uniform [0,1) fp32 grid, seed 1000+rank)",
        "config": {
            "workload": f"stencil_smi 4-point Jacobi, {X}x{Y} fp32 tile per GPU, "
                        f"{PX}x{PY} decomposition ({PX * X}x{PY * Y} global)"
                        + (", halo exchange over RCCL/xGMI overlapped with the interior" if world > 1
                           else ", no halo exchange (BASELINE config 2)"),
            "grid": [PX * X, PY * Y],
            "tile": [X, Y],
            "decomposition": [PX, PY],
            "plan": [{"steps_per_pass": k, "passes": n} for k, n in plan["phases"]],
            "tuning": stencil.get_tuning(),
            "fusion": fusion,
            "launch": "self (bench.py started the ranks)" if os.environ.get("SMI_BENCH_SELF_LAUNCH")
                      else "external" if world > 1 else "single process",
            "fake_host": bool(os.environ.get("SMI_BENCH_FAKE_HOST")),
            "warmup_ms_floor": args.warmup_ms,
            "warmup_ms_run": round(warm_ms, 1),
            # the library's recorded source hash; load() refuses a library whose
            # hash differs from this tree's (smi_amd.build._src_hash())
            "lib_srchash": smi_amd._lib.recorded_srchash(),
        },
        "repeats": repeats,
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_basis": traffic_basis,
            "kernel": kernel_name,
            "kernel_avg_ms": round(sweep_avg_ms, 5),
            "launches": dom["launches"] if dom else 0,
            "steps_per_launch": spl,
            "cells_per_launch": cells_launch,
            "bytes_per_launch": int(bytes_launch),
            "cell_step_GBs": round(step_gbs, 1),
            "share_of_timed_region": round(dom["share_of_timed_region"], 4) if dom else None,
            "kernels_share_of_timed_region": round(sum(k["total_ms"] for k in kernels) / timed_ms, 4)
                                             if world == 1 else None,
            "timing": "value from the timed region (profiling off); kernel times from an identical profiled "
                      "repetition right after it",
            "profiled_repetition_ms": round(prof_rep_ms, 4),
            "kernels": [{"kernel": k["kernel"], "launches": k["launches"], "total_ms": round(k["total_ms"], 5),
                         "avg_ms": round(k["avg_ms"], 5), "share_of_timed_region": round(k["share_of_timed_region"], 4),
                         "cell_step_GBs": round(k["cell_step_GBs"], 1) if k["cell_step_GBs"] else None}
                        for k in kernels],
            "note": "kernel = the stencil kernel with the largest measured time in the profiled repetition of the "
                    "timed plan (HIP events on its stream, one marker between back-to-back passes). achieved = the pass's compulsory "
                    "bytes (every cell it stores read once + written once, 8 B) / its avg launch time, frac = "
                    "achieved / peak. traffic = measured HBM bytes per launch of that kernel (rocprofv3 FETCH_SIZE "
                    "x2 + WRITE_SIZE, profiles/pmc_stencil_sweep.json), hbm_frac = traffic / avg launch time / "
                    "peak (what the memory system moved, over-fetch included). cell_step_GBs = 8 B per cell-STEP "
                    "x K steps per pass / launch time: temporal blocking, not a fraction of peak",
        },
    }
    if dom:
        rp = (rocprof_avg(f"{'sweepd' if spl > 12 else 'sweepk'}_kernel<{spl}>")
              if dom["kind"] == profiling.SWEEPK else None)
        if rp and world == 1:  # the committed summary is of the N = 1 driver command
            rp["ratio_to_hip_events"] = round(rp["avg_ms"] / sweep_avg_ms, 4) if sweep_avg_ms else None
            out["roofline"]["rocprof"] = rp
    if traffic and sweep_avg_ms:
        hbm = traffic / (sweep_avg_ms * 1e-3) / 1e9
        out["roofline"]["hbm_achieved"] = round(hbm, 1)
        out["roofline"]["hbm_frac"] = round(hbm / HBM_PEAK_GBS, 4)  # per GPU
    if sweep_avg_ms and spl:
        # The VALU side of the same launch: algorithmic fp32 adds (3 per
        # cell-step, ((S+W)+E)+N; the scaled levels drop the reference's x0.25
        # per step) over the FP32 vector add rate (157.3 TFLOPS spec counts an
        # FMA as 2: 32 lanes x 1024 SIMDs x 2.4 GHz = 78.6 T adds/s).
        adds = 3.0 * cells_launch * spl / (sweep_avg_ms * 1e-3) / 1e12
        out["roofline"]["valu"] = {"achieved": round(adds, 2), "peak": VALU_PEAK_TADDS, "unit": "T fp32 adds/s",
                                   "frac": round(adds / VALU_PEAK_TADDS, 4),
                                   "note": "3 adds per cell-step x cells x K per launch / avg launch time; the issued "
                                           "VALU count (SQ_INSTS_VALU) is in profiles/r04/sq_driver.txt"}
    if world > 1:
        out["halo"] = halo_report(PX, PY, X, Y, max(spl, 1), elapsed / args.steps * 1e3)
    if not args.no_parity:
        with torch.cuda.stream(stream):
            out["parity"] = verify_timed_plan(comm, tile, scratch, g, args.steps, PX, PY, rank, world)
        log(f"parity: {out['parity']['mismatches']} mismatching cells of {out['parity']['cells']} "
            f"({out['parity']['steps']} steps)")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()

    # Auxiliary lines (BASELINE configs 4 and 5), measured after the timed
    # stencil region.  A watchdog bounds them: if they do not finish, rank 0
    # still prints the stencil line and every rank exits.
    printed = threading.Lock()

    def emit(o):
        if rank == 0 and printed.acquire(blocking=False):
            data = (json.dumps(o) + "\n").encode()
            while data:
                data = data[os.write(result_fd, data):]

    def watchdog():
        o = dict(out)
        o["aux"] = {"error": f"auxiliary measurements exceeded {AUX_BUDGET_S:.0f} s"}
        emit(o)
        os._exit(0)

    if not args.no_aux:
        timer = threading.Timer(AUX_BUDGET_S, watchdog)
        timer.daemon = True
        timer.start()
        aux = {}
        try:
            aux["gesummv"] = aux_gesummv(comm, world, rank, stream, barrier)
            log("aux gesummv done")
            if world > 1:
                aux["collectives"] = aux_collectives(comm, world, rank, stream, barrier)
                log("aux collectives done")
                aux["p2p"] = aux_p2p(comm, world, rank, stream, barrier)
                log("aux p2p done")
            else:
                aux["kernels"] = aux_kernels_1gpu()
                if not args.no_cpu_baseline:
                    aux["cpu"] = cpu_aux_legs()
        except Exception as e:  # report, never lose the stencil line
            aux["error"] = f"{type(e).__name__}: {e}"
        out["aux"] = aux
    emit(out)
    comm.finalize()
    if world > 1:
        dist.destroy_process_group()
    if not args.no_aux:
        timer.cancel()  # after teardown: a wedged finalize is bounded too


if __name__ == "__main__":
    main()
