#!/usr/bin/env python3
"""Per-rank timing rehearsal of the multi-GPU stencil on ONE GPU.

Loads the rehearsal build of the library (smi_amd/build.py --rehearsal,
SMI_LOOPBACK_REHEARSAL), in which a 1x1 run with SMI_LOOPBACK=1 is its own
neighbour on all four sides and four diagonals: the GPU then does exactly the
per-pass work of an interior rank of a large decomposition (band kernel on
the comm stream, 8-peer exchange through the transport, interior sweep on the
main stream) with the production stream schedule.  The halos wrap around, so
the values are not the stencil's -- timing only.

Cases (REHEARSAL_CASES, comma list; each timed the same way, interleaved
run by run so that clock drift hits every case alike):
  alone  -- the lone tile (no neighbours): what bench.py --gpus 1 times
  full   -- interior rank: bands + exchange + interior
  bands  -- interior rank without the exchange (SMI_LOOPBACK_NOXCHG)
  xchg   -- interior rank without the band work (SMI_REH_NOBANDS)
  bare   -- neither: the two-stream schedule and the host join only
  brows / bcols -- bands without the exchange, only the top / bottom row
           walks or only the transposed left / right column walks
  full_p0 -- full, the band kernel's waves at normal priority
The exchange is RCCL's real kernel by default (a one-rank RCCL communicator
whose 8 sends and receives per pass go to itself through the production
RcclTransport); REHEARSAL_TRANSPORT=local uses the in-process transport.

Timing: Python's garbage collector is collected once and
disabled before anything is timed (a C++ host has none); every timed run is
preceded by a load-based warm-up of that same case (REHEARSAL_WARM_MS, default
100 ms of back-to-back runs) and follows it with no host idle beyond the
synchronize that ends it -- the shape of bench.py's warm-up floor -- and
lasts REHEARSAL_PASSES K-step passes (default 400: ~60 ms at K = 20).
efficiency = alone / case (ms per step) for the min and the median over
REHEARSAL_REPS runs.  BENCH_LONE_MS_PER_STEP (bench.py's production lone tile
measured in the same session) adds efficiency_vs_bench.  REHEARSAL_PROF=1
adds one profiled run per case (band / interior averages, not timed).
usage: rehearsal.py [tile] [K]
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

CASES = {
    "alone": {},
    "full": {"SMI_LOOPBACK": "1"},
    "bands": {"SMI_LOOPBACK": "1", "SMI_LOOPBACK_NOXCHG": "1"},
    "xchg": {"SMI_LOOPBACK": "1", "SMI_REH_NOBANDS": "1"},
    "bare": {"SMI_LOOPBACK": "1", "SMI_LOOPBACK_NOXCHG": "1", "SMI_REH_NOBANDS": "1"},
    # the band kernel's two halves, no exchange
    "brows": {"SMI_LOOPBACK": "1", "SMI_LOOPBACK_NOXCHG": "1", "SMI_REH_BANDS": "rows"},
    "bcols": {"SMI_LOOPBACK": "1", "SMI_LOOPBACK_NOXCHG": "1", "SMI_REH_BANDS": "cols"},
    # the band kernel at the interior's wave priority instead of a raised one
    "full_p0": {"SMI_LOOPBACK": "1", "SMI_REH_BAND_PRIO": "0"},
}
SWITCHES = ("SMI_LOOPBACK", "SMI_LOOPBACK_NOXCHG", "SMI_REH_NOBANDS", "SMI_REH_BANDS", "SMI_REH_BAND_PRIO")


def set_case(name):
    for k in SWITCHES:
        os.environ.pop(k, None)
    os.environ.update(CASES[name])


def median(v):
    s = sorted(v)
    return s[len(s) // 2] if len(s) % 2 else 0.5 * (s[len(s) // 2 - 1] + s[len(s) // 2])


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    cases = os.environ.get("REHEARSAL_CASES", "alone,full,bands,xchg,bare").split(",")
    reps = int(os.environ.get("REHEARSAL_REPS", "5"))
    warm_ms = float(os.environ.get("REHEARSAL_WARM_MS", "100"))
    passes = int(os.environ.get("REHEARSAL_PASSES", "400"))
    prof = os.environ.get("REHEARSAL_PROF", "0") != "0"
    bench_lone = float(os.environ["BENCH_LONE_MS_PER_STEP"]) if os.environ.get("BENCH_LONE_MS_PER_STEP") else None
    smi_amd.load(build_if_missing=False)
    if os.environ.get("REHEARSAL_TRANSPORT", "rccl") == "rccl":
        comm = smi_amd.Comm.create(0, 1, 0, smi_amd.Comm.unique_id())
        exchange = "RCCL self send/recv (one-rank communicator, rcclGenericKernel)"
    else:
        comm = smi_amd.LocalGroup(1).comm(0)
        exchange = "in-process transport"
    # one stream for every run, made after the communicator as a caller would;
    # REH_STREAM_PRIO=normal puts it at normal priority (the library then runs
    # the interior on a highest-priority stream of its own)
    s = torch.cuda.Stream(priority=0 if os.environ.get("REH_STREAM_PRIO") == "normal" else -1)
    t = torch.rand((n, n), device="cuda")
    sc = torch.empty_like(t)
    stencil.set_fusion(k)
    steps = passes * k
    warm_steps = 20 * k

    gc.collect()
    gc.disable()
    runs = {c: [] for c in cases}
    warm = {c: [] for c in cases}
    order = []
    with torch.cuda.stream(s):
        for c in cases:  # every kernel of every case loaded once
            set_case(c)
            stencil.run(comm, t, 2 * k, 1, 1, sc)
        s.synchronize()
        for r in range(reps):
            for c in cases:
                set_case(c)
                # load-based warm-up of this case, then the timed run right
                # behind it (bench.py's warm-up floor: GPU clocks and the
                # timed kernels' code hot, nothing idle but the synchronize)
                tw = time.perf_counter()
                nw = 0
                while (time.perf_counter() - tw) * 1e3 < warm_ms:
                    stencil.run(comm, t, warm_steps, 1, 1, sc)
                    s.synchronize()
                    nw += 1
                warm[c].append(round((time.perf_counter() - tw) * 1e3, 1))
                t0 = time.perf_counter()
                stencil.run(comm, t, steps, 1, 1, sc)
                s.synchronize()
                dt = time.perf_counter() - t0
                runs[c].append(dt / steps * 1e3)
                order.append((c, round(dt / steps * 1e3, 6)))
        profd = {}
        if prof:
            for c in cases:
                set_case(c)
                profiling.reset()
                profiling.enable(True)
                stencil.run(comm, t, 40 * k, 1, 1, sc)
                s.synchronize()
                profiling.enable(False)
                band = profiling.read(profiling.EDGE)
                sweep = profiling.read(profiling.SWEEPK)
                profd[c] = {"band_avg_ms": round(band[0] / max(band[1], 1), 5),
                            "interior_avg_ms": round(sweep[0] / max(sweep[1], 1), 5)}
    gc.enable()
    set_case("alone")
    a_min = min(runs["alone"]) if "alone" in runs else None
    a_med = median(runs["alone"]) if "alone" in runs else None
    out = {"K": k, "tile": n, "passes_per_run": passes, "steps_per_run": steps, "reps": reps,
           "warm_ms_floor": warm_ms, "exchange": exchange,
           "run_stream_priority": "normal" if os.environ.get("REH_STREAM_PRIO") == "normal" else "high",
           "bench_lone_ms_per_step": bench_lone, "cases": {}}
    for c in cases:
        v = runs[c]
        e = {"ms_per_step_min": round(min(v), 6), "ms_per_step_median": round(median(v), 6),
             "run_ms_min": round(min(v) * steps, 2),
             "runs_ms_per_step": [round(x, 6) for x in v], "warmup_ms": warm[c]}
        if a_min and c != "alone":
            e["efficiency_min"] = round(a_min / min(v), 4)
            e["efficiency_median"] = round(a_med / median(v), 4)
            if bench_lone:
                e["efficiency_vs_bench_min"] = round(bench_lone / min(v), 4)
                e["efficiency_vs_bench_median"] = round(bench_lone / median(v), 4)
        if c == "alone" and bench_lone:
            e["vs_bench_lone"] = round(median(v) / bench_lone, 4)
        if c in profd:
            e.update(profd[c])
        out["cases"][c] = e
    out["chronological"] = order
    print(json.dumps(out), flush=True)
    comm.finalize()


if __name__ == "__main__":
    main()
