#!/usr/bin/env python3
"""Host/launch overhead of a short timed stencil run (bench --steps 20):
wall time of stencil.run(T) between two device synchronisations vs the sum
of its kernels' HIP-event times, with and without per-launch profiling."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import smi_amd  # noqa: E402
from smi_amd import profiling, stencil  # noqa: E402

smi_amd.load()
comm = smi_amd.LocalGroup(1).comm(0)
a = torch.rand((8192, 8192), device="cuda")
b = torch.empty_like(a)
s = torch.cuda.Stream()
res = {}
with torch.cuda.stream(s):
    for _ in range(30):
        stencil.run(comm, a, 48, 1, 1, b)
    torch.cuda.synchronize()
    for T in (0, 12, 20, 24):
        for prof in (False, True):
            walls, kern = [], []
            for _ in range(15):
                stencil.run(comm, a, 48, 1, 1, b)  # keep the clock up
                torch.cuda.synchronize()
                profiling.reset()
                profiling.enable(prof)
                t0 = time.perf_counter()
                stencil.run(comm, a, T, 1, 1, b)
                torch.cuda.synchronize()
                walls.append((time.perf_counter() - t0) * 1e3)
                profiling.enable(False)
                if prof:
                    kern.append(sum(profiling.read_tag(k, t)[0] for k, t in profiling.entries()))
            res[f"T={T} prof={int(prof)}"] = {"wall_ms_med": round(float(np.median(walls)), 4),
                                             "kernels_ms_med": round(float(np.median(kern)), 4) if kern else None}
print(json.dumps(res, indent=1))
