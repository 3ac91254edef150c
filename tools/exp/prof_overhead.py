"""Wall time of a 2400-step run (200 K=12 passes) at 8192^2 with the HIP-event
profiling on and off: what recording two events around every launch costs."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import smi_amd  # noqa: E402
from smi_amd import profiling, stencil  # noqa: E402

smi_amd.load()
comm = smi_amd.LocalGroup(1).comm(0)
a = torch.rand(8192, 8192, device="cuda")
b = torch.empty_like(a)
for _ in range(3):
    stencil.run(comm, a, 240, 1, 1, b)
torch.cuda.synchronize()
for rep in range(3):
    for prof in (False, True):
        profiling.reset()
        profiling.enable(prof)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        stencil.run(comm, a, 2400, 1, 1, b)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        profiling.enable(False)
        ms, n = profiling.read(profiling.SWEEPK) if prof else (0.0, 0)
        print(json.dumps({"prof": prof, "wall_ms": round(dt * 1e3, 3), "kernel_ms": round(ms, 3), "launches": n,
                          "gap_us_per_pass": round((dt * 1e3 - ms) / 200 * 1e3, 2) if prof else None}), flush=True)
comm.finalize()
