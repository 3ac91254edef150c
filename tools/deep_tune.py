#!/usr/bin/env python3
"""Sweep the rotating-ring sweep's balancing weights (smi_stencil_set_deep:
edge-column and upward-bottom-block extra work in 16ths) on the driver's
config (8192^2, T = 20, one K = 20 pass) and print ms per pass for each.
Scheduling only: every setting is bit-identical (tests/test_stencil_gpu.py
test_ring_geometry_is_bit_neutral)."""
import itertools
import json
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import smi_amd  # noqa: E402
from smi_amd import stencil  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
T = 20
torch.cuda.set_device(0)
comm = smi_amd.LocalGroup(1).comm(0)
a = torch.rand((N, N), device="cuda")
b = torch.empty_like(a)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]


def timed(reps=30):
    for _ in range(10):
        stencil.run(comm, a, T, 1, 1, b)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        ev[0].record()
        stencil.run(comm, a, T, 1, 1, b)
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    ts.sort()
    return ts[len(ts) // 2], ts[0]


base = stencil.get_deep()
grid = [(ce, rev) for ce, rev in itertools.product((6, 8, 10, 12, 14, 16), (4, 6, 8, 10, 12))]
for rnd in range(2):
    for ce, rev in grid:
        stencil.set_deep(ce, rev, 0)
        med, mn = timed()
        print(json.dumps({"round": rnd, "ce16": ce, "rev16": rev, "ms_med": round(med, 5), "ms_min": round(mn, 5)}),
              flush=True)
stencil.set_deep(base["ce16"], base["rev16"], base["waves"])
comm.finalize()
