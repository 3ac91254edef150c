#!/usr/bin/env python3
"""Tuning table for the multi-step sweeps on one GPU: time per Jacobi STEP
(kernel time / steps per pass, HIP events around every launch) for
steps_per_pass K in {2, 4, 8, 12} x rows per wave x rows in flight."""
import itertools
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import smi_amd  # noqa: E402
from smi_amd import profiling, stencil  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    ks = [int(k) for k in (sys.argv[3].split(",") if len(sys.argv) > 3 else ["2", "4", "8"])]
    smi_amd.load()
    comm = smi_amd.LocalGroup(1).comm(0)
    a = torch.rand((n, n), device="cuda")
    b = torch.empty_like(a)
    grid = {2: itertools.product([8, 16], [8]),
            4: itertools.product([-1, 48, 96], [3]),
            8: itertools.product([-1, 48, 96, 192], [3]),
            12: itertools.product([-1, 48, 96, 192], [3]),
            16: itertools.product([-1, 64, 128], [4, 8])}
    settings = [(k, ht, u) for k in ks for (ht, u) in grid[k]]
    res = {}
    for rnd in range(3):
        for (k, ht, u) in settings:
            stencil.set_fusion(k, ht, u)
            stencil.run(comm, a, 2 * k, 1, 1, b)
            torch.cuda.synchronize()
            profiling.reset()
            profiling.enable(True)
            stencil.run(comm, a, passes * k, 1, 1, b)
            torch.cuda.synchronize()
            profiling.enable(False)
            ms, cnt = profiling.read(profiling.SWEEPK if k >= 4 else profiling.SWEEP)
            res.setdefault((k, ht, u), []).append(ms / cnt / k)
    rows = sorted(((sorted(v)[1], s) for s, v in res.items()))
    for med, (k, ht, u) in rows:
        print(json.dumps({"K": k, "ht": ht, "u": u, "ms_per_step": round(med, 5),
                          "GCells": round(n * n / med / 1e6, 1),
                          "GBs_algorithmic": round(8 * n * n / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
