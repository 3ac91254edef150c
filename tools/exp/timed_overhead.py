#!/usr/bin/env python3
"""Where the non-kernel time of the driver's short timed region goes
(bench.py --steps 20: two 10-step passes): host time of the stencil.run call,
GPU time between a marker recorded before it and one after it, the kernels'
own durations (dispatch-timed), and the host-observed region with the
synchronize.  One JSON line per repetition."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import smi_amd  # noqa: E402
from smi_amd import profiling, stencil  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    smi_amd.load(build_if_missing=False)
    comm = smi_amd.LocalGroup(1).comm(0)
    t = torch.rand((8192, 8192), device="cuda")
    sc = torch.empty_like(t)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(30):
            stencil.run(comm, t, steps, 1, 1, sc)
        torch.cuda.synchronize()
        for rep in range(8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            profiling.reset()
            profiling.enable(os.environ.get("TO_PROF", "1") != "0")
            h0 = time.perf_counter()
            e0.record(s)
            h1 = time.perf_counter()
            stencil.run(comm, t, steps, 1, 1, sc)
            h2 = time.perf_counter()
            e1.record(s)
            torch.cuda.synchronize()
            h3 = time.perf_counter()
            profiling.enable(False)
            ms, n = profiling.read(profiling.SWEEPK)
            print(json.dumps({"steps": steps, "prof": os.environ.get("TO_PROF", "1") != "0", "host_run_call_us": round((h2 - h1) * 1e6, 1),
                              "host_region_us": round((h3 - h0) * 1e6, 1),
                              "gpu_marker_to_marker_us": round(e0.elapsed_time(e1) * 1e3, 1),
                              "kernels_us": round(ms * 1e3, 1), "launches": n}), flush=True)
    comm.finalize()


if __name__ == "__main__":
    main()
