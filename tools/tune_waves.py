#!/usr/bin/env python3
"""Sweep the rotating-ring sweep's launch size (smi_stencil_set_deep waves:
0 = one round of every resident wave slot, 2 per SIMD at K = 20; 1024 = one
wave per SIMD with row blocks twice as tall, half the cone rows) with the
balancing weights, on the driver's config (8192^2, one K = 20 pass per run).
Each setting: 50 ms of back-to-back passes (the chip settles at its power
cap), then 200 back-to-back passes between two events; settings interleaved,
3 rounds.  Scheduling only: bit-identical for every setting
(test_ring_geometry_is_bit_neutral); the script checks the bits too.
usage: tune_waves.py [tile] [waves,ce16,rev16 ...]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import smi_amd  # noqa: E402
from smi_amd import stencil  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
specs = [tuple(int(v) for v in a.split(",")) for a in sys.argv[2:]] or [
    (0, 10, 6), (1024, 10, 6), (1024, 6, 4), (1024, 14, 8), (1280, 10, 6), (1536, 10, 6), (3072, 10, 6)]
T = 20
torch.cuda.set_device(0)
smi_amd.load(build_if_missing=False)
comm = smi_amd.LocalGroup(1).comm(0)
g = torch.Generator(device="cuda")
g.manual_seed(7)
a0 = torch.rand((N, N), device="cuda", generator=g)
a = a0.clone()
b = torch.empty_like(a)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
base = stencil.get_deep()
ref = None
res = {s: [] for s in specs}
for rnd in range(3):
    for s in specs:
        stencil.set_deep(s[1], s[2], s[0])
        out = stencil.run(comm, a0.clone(), T, 1, 1, b)
        bits = out.view(torch.int32)
        if ref is None:
            ref = bits.clone()
        assert torch.equal(bits, ref), s
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.05:
            for _ in range(20):
                stencil.run(comm, a, T, 1, 1, b)
            torch.cuda.synchronize()
        ev[0].record()
        for _ in range(200):
            stencil.run(comm, a, T, 1, 1, b)
        ev[1].record()
        torch.cuda.synchronize()
        res[s].append(ev[0].elapsed_time(ev[1]) / 200)
for s in specs:
    v = sorted(res[s])
    print(json.dumps({"waves": s[0], "ce16": s[1], "rev16": s[2], "ms_per_pass": [round(x, 5) for x in res[s]],
                      "median": round(v[len(v) // 2], 5), "GCells": round(N * N * T / (v[len(v) // 2] * 1e-3) / 1e9, 1)}),
          flush=True)
stencil.set_deep(base["ce16"], base["rev16"], base["waves"])
comm.finalize()
