#!/usr/bin/env python3
"""Sweep-kernel tuning table on one GPU: avg kernel time and GB/s per setting
(HIP events around every launch, interleaved rounds in one process)."""
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
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    smi_amd.load()
    a = torch.rand((n, n), device="cuda")
    b = torch.empty_like(a)
    # reference point: torch's own device copy of the same bytes
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        b.copy_(a)
    e0.record()
    for _ in range(steps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    copy_ms = e0.elapsed_time(e1) / steps
    print(json.dumps({"torch_copy_ms": copy_ms, "GBs": 8 * n * n / copy_ms / 1e6}), flush=True)
    settings = list(itertools.product([8, 12, 16, 24], [8, 16], [1]))
    res = {s: [] for s in settings}
    for rnd in range(3):
        for (ht, u, nt) in settings:
            stencil.set_tuning(ht, u, nt, -1)
            for _ in range(2):
                stencil.step(a, b)
            torch.cuda.synchronize()
            profiling.reset()
            profiling.enable(True)
            for _ in range(steps):
                stencil.step(a, b)
                a, b = b, a
            torch.cuda.synchronize()
            profiling.enable(False)
            ms, cnt = profiling.read(profiling.SWEEP)
            res[(ht, u, nt)].append(ms / cnt)
    # two steps per pass: time per STEP (kernel time / 2)
    stencil.set_fusion(2)
    comm = smi_amd.LocalGroup(1).comm(0)
    res2 = {}
    for rnd in range(3):
        for (ht, u) in itertools.product([8, 16, 32, 64], [2, 4, 8]):
            stencil.set_fusion(2, ht, u)
            stencil.run(comm, a, 4, 1, 1, b)
            torch.cuda.synchronize()
            profiling.reset()
            profiling.enable(True)
            stencil.run(comm, a, 2 * steps, 1, 1, b)
            torch.cuda.synchronize()
            profiling.enable(False)
            ms, cnt = profiling.read(profiling.SWEEP)
            res2.setdefault((ht, u), []).append(ms / cnt / 2)
    for (ht, u), v in sorted(res2.items(), key=lambda kv: sorted(kv[1])[1]):
        med = sorted(v)[len(v) // 2]
        print(json.dumps({"fused": 2, "ht2": ht, "u2": u, "ms_per_step": round(med, 5),
                          "GBs_algorithmic": round(8 * n * n / med / 1e6, 1)}), flush=True)
    stencil.set_fusion(1)
    rows = []
    for s, v in res.items():
        med = sorted(v)[len(v) // 2]
        rows.append((med, s))
    rows.sort()
    for med, (ht, u, nt) in rows:
        print(json.dumps({"ht": ht, "u": u, "nt": nt, "ms": round(med, 5),
                          "GBs": round(8 * n * n / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
