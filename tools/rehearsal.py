#!/usr/bin/env python3
"""Per-rank timing rehearsal of the multi-GPU stencil on ONE GPU.

Loads the rehearsal build of the library (smi_amd/build.py --rehearsal,
SMI_LOOPBACK_REHEARSAL), in which a 1x1 run with SMI_LOOPBACK=1 is its own
neighbour on all four sides and four diagonals: the GPU then does exactly the
per-pass work of an interior rank of a large decomposition (band kernel on
the comm stream, 8-peer exchange through the transport, interior sweep on the
main stream)
with the production stream schedule.  The halos wrap around, so the values
are not the stencil's -- timing only.  Prints ms/step next to the plain
single-tile run, i.e. an estimate of per-GPU weak-scaling efficiency with
an exchange that costs one device-to-device copy of the halo bytes.
REHEARSAL_ROUNDS (list) sets the rounds of resident waves the multi-rank
interior sweep is cut into, REHEARSAL_RESERVE (list) the wave slots it leaves
free for the band kernel and the exchange (smi_stencil_set_bands),
REHEARSAL_LEAN (list, default 1) the band kernel for K >= 13 (1 = the lean
kernel beside the interior, 0 = one wave per segment).
REHEARSAL_PROF=0 times the runs without the library's profiling markers (the
band / interior averages are then not reported).  Python's garbage collector
is off inside each timed run (REHEARSAL_GC=1 leaves it on).  efficiency = min
over the lone-tile runs / min over the interior-rank runs, efficiency_median
the same with medians.
SMI_LOOPBACK_FUSED=1 prices the exchange as one copy kernel (like one RCCL
group), SMI_LOOPBACK_NOXCHG=1 leaves it out, SMI_LOOPBACK_HEAVY=<blocks> as
one copy kernel of that many 256-thread workgroups with rcclGenericKernel's
register and LDS footprint (280 VGPRs, 19.7 KB; tools/rccl_footprint.py).
REHEARSAL_TRANSPORT=rccl runs the exchange through the real RCCL kernel: a
one-rank RCCL communicator whose 8 sends and receives go to itself (RCCL's
self send/recv, one group per pass, the production RcclTransport).
usage: rehearsal.py [tile] [K...]
"""
import gc
import json
import os
import sys
import time

os.environ["SMI_LIB_VARIANT"] = "rehearsal"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import smi_amd  # noqa: E402
from smi_amd import profiling, stencil  # noqa: E402


LAST_CHRONO = []


def timed(comm, t, sc, steps, reps=5):
    """ms per step of `reps` runs, sorted (the in-process transport creates
    and retires HIP events per message: occasional host stalls that RCCL
    does not have, so the min is the estimate); LAST_CHRONO keeps the same
    runs in the order they ran"""
    runs = [_timed(comm, t, sc, steps) for _ in range(reps)]
    LAST_CHRONO[:] = runs
    return sorted(runs)


_STREAM = []


def _new_stream():
    # REH_STREAM_PRIO=high: the run's stream at the highest priority (the
    # library then runs the interior on it); by default at normal priority,
    # created after the communicator, as a caller would (the library then
    # moves the interior to a stream of its own at the highest priority)
    return torch.cuda.Stream(priority=-1 if os.environ.get("REH_STREAM_PRIO") == "high" else 0)


def _timed(comm, t, sc, steps):
    # one stream for every run: a new torch stream per run (rounds 3-5) made
    # every few runs land on the comm stream's hardware queue (HIP maps
    # streams round-robin onto GPU_MAX_HW_QUEUES = 4 queues), serialising the
    # interior with the bands and the exchange -- the series' "slow run"
    if not _STREAM:
        _STREAM.append(_new_stream())
    s = _STREAM[0]
    with torch.cuda.stream(s):
        stencil.run(comm, t, 2 * steps, 1, 1, sc)
        s.synchronize()
        profiling.reset()
        profiling.enable(os.environ.get("REHEARSAL_PROF", "1") != "0")
        # no garbage-collector pass inside a timed run (a C/C++ host has
        # none; round 5 traced the "slow run" of every series to one)
        gc_on = os.environ.get("REHEARSAL_GC", "0") != "0"
        gc.collect()
        if not gc_on:
            gc.disable()
        try:
            t0 = time.perf_counter()
            stencil.run(comm, t, steps, 1, 1, sc)
            s.synchronize()
            dt = time.perf_counter() - t0
        finally:
            gc.enable()
        profiling.enable(False)
    return dt / steps * 1e3


def exchange_label(noxchg) -> str:
    if noxchg:
        return "none"
    if os.environ.get("SMI_LOOPBACK_FUSED"):
        return "one copy kernel"
    if os.environ.get("SMI_LOOPBACK_HEAVY"):
        return f"one copy kernel with rcclGenericKernel's footprint, {os.environ['SMI_LOOPBACK_HEAVY']} workgroups"
    if os.environ.get("REHEARSAL_TRANSPORT") == "rccl":
        return "RCCL self send/recv (one-rank communicator, rcclGenericKernel)"
    return "in-process transport"


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    ks = [int(k) for k in sys.argv[2:]] or [12]
    smi_amd.load(build_if_missing=False)
    if os.environ.get("REH_STREAM_EARLY"):  # the run's stream created before the communicator
        _STREAM.append(_new_stream())
    if os.environ.get("REHEARSAL_TRANSPORT") == "rccl":
        comm = smi_amd.Comm.create(0, 1, 0, smi_amd.Comm.unique_id())
    else:
        comm = smi_amd.LocalGroup(1).comm(0)
    t = torch.rand((n, n), device="cuda")
    sc = torch.empty_like(t)
    for k in ks:
        stencil.set_fusion(k)
        steps = int(os.environ.get("REHEARSAL_PASSES", "10")) * max(k, 2)
        os.environ.pop("SMI_LOOPBACK", None)
        alone = timed(comm, t, sc, steps)[0]
        noxchg = os.environ.get("SMI_LOOPBACK_NOXCHG")
        grid = [(r, b) for r in (int(x) for x in os.environ.get("REHEARSAL_ROUNDS", "1,2,3").split(","))
                for b in (int(x) for x in os.environ.get("REHEARSAL_RESERVE", "0").split(","))]
        grid = [(r, b, lean) for r, b in grid
                for lean in (int(x) for x in os.environ.get("REHEARSAL_LEAN", "1").split(","))]
        for rounds, reserve, lean in grid:
            stencil.set_bands(reserve, rounds)
            stencil.set_band_kernel(lean)
            for ov in [int(x) for x in os.environ.get("REHEARSAL_OVERLAP", "1,0").split(",")]:
                stencil.set_tuning(overlap=ov)
                # the lone tile right before each setting (the GPU clock
                # drifts between settings and boxes)
                os.environ.pop("SMI_LOOPBACK", None)
                alone_runs = timed(comm, t, sc, steps)
                alone = min(alone, alone_runs[0]) if os.environ.get("REHEARSAL_ALONE_MIN") else alone_runs[0]
                os.environ["SMI_LOOPBACK"] = "1"
                runs = timed(comm, t, sc, steps)
                loop = runs[0]
                band = profiling.read(profiling.EDGE)
                sweep = profiling.read(profiling.SWEEPK if k >= 4 else profiling.SWEEP)
                os.environ.pop("SMI_LOOPBACK", None)
                print(json.dumps({"K": k, "rounds": rounds, "reserve_waves": reserve, "band_kernel": "lean" if lean and k >= 13 else "wave per segment", "no_bands": bool(os.environ.get("SMI_REH_NOBANDS")), "prof": os.environ.get("REHEARSAL_PROF", "1") != "0", "overlap": ov, "tile": n, "exchange": exchange_label(noxchg),
                                  "ms_per_step_alone": round(alone, 5),
                                  "ms_per_step_interior_rank": round(loop, 5),
                                  "efficiency": round(alone / loop, 4),
                                  "runs_ms_per_step": [round(r, 5) for r in runs],
                                  "runs_chronological": [round(r, 5) for r in LAST_CHRONO],
                                  "alone_runs_ms_per_step": [round(r, 5) for r in alone_runs],
                                  # median of the lone-tile runs / median of the interior-rank runs
                                  "efficiency_median": round(alone_runs[len(alone_runs) // 2] / runs[len(runs) // 2], 4),
                                  "gc_in_timed_runs": os.environ.get("REHEARSAL_GC", "0") != "0",
                                  "run_stream_priority": "high" if os.environ.get("REH_STREAM_PRIO") == "high" else "normal",
                                  "band_avg_ms": round(band[0] / max(band[1], 1), 5),
                                  "interior_avg_ms": round(sweep[0] / max(sweep[1], 1), 5)}), flush=True)
    stencil.set_tuning(overlap=1)
    stencil.set_bands(0, 1)
    stencil.set_band_kernel(1)
    comm.finalize()


if __name__ == "__main__":
    main()
