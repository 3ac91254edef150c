"""Experiment: wall time of one stencil.run(T) at 8192^2 (sync, run, sync --
the bench's timed region) under different steps-per-pass settings, i.e.
different splits of T into passes.  Median of 40 runs after a warm-up."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import smi_amd  # noqa: E402
from smi_amd import stencil  # noqa: E402

smi_amd.load()
comm = smi_amd.LocalGroup(1).comm(0)
a = torch.rand(8192, 8192, device="cuda")
b = torch.empty_like(a)
for T, ks in ((20, (12, 10, 11, 9)), (24, (12, 8)), (25, (12, 9)), (13, (12, 7)), (30, (12, 10))):
    for k in ks:
        stencil.set_fusion(k, -1)
        plan = stencil.plan(8192, 8192, 1, 1, 0, T)["phases"]
        t_w = time.perf_counter()
        while time.perf_counter() - t_w < 0.05:
            stencil.run(comm, a, 48, 1, 1, b)
            torch.cuda.synchronize()
        ts = []
        for _ in range(40):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            stencil.run(comm, a, T, 1, 1, b)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        med = ts[len(ts) // 2]
        print(json.dumps({"T": T, "fusion": k, "plan": plan, "ms_med": round(med * 1e3, 4),
                          "GCells": round(8192 * 8192 * T / med / 1e9, 1)}), flush=True)
stencil.set_fusion(12, -1)
comm.finalize()
