#!/usr/bin/env python3
"""Multi-rank schedule overhead on ONE GPU: R ranks of an in-process group
share device 0, so ideal time per step = R x (one rank alone).  Reports the
ratio for 1x1, 1x2, 2x2 decompositions (tile per rank = N x N)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import smi_amd  # noqa: E402
from smi_amd import profiling, stencil  # noqa: E402


def run(PX, PY, n, steps, overlap):
    stencil.set_tuning(overlap=overlap)
    grp = smi_amd.LocalGroup(PX * PY)

    def fn(comm):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            t = torch.rand((n, n), device="cuda")
            sc = torch.empty_like(t)
            stencil.run(comm, t, 24, PX, PY, sc)
            s.synchronize()
            t0 = time.perf_counter()
            stencil.run(comm, t, steps, PX, PY, sc)
            s.synchronize()
            return time.perf_counter() - t0

    profiling.reset()
    profiling.enable(True)
    t = max(grp.run(fn))
    profiling.enable(False)
    sw = profiling.read(profiling.SWEEPK if stencil.get_fusion()["steps_per_pass"] >= 4 else profiling.SWEEP)
    ed = profiling.read(profiling.EDGE)
    print(json.dumps({"decomp": f"{PX}x{PY}", "overlap": overlap,
                      "sweep_avg_ms": sw[0] / max(sw[1], 1), "sweep_n": sw[1],
                      "edge_or_ring_avg_ms": ed[0] / max(ed[1], 1), "edge_n": ed[1]}), flush=True)
    return t


def main():
    smi_amd.load()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    steps = 120
    if len(sys.argv) > 2:
        stencil.set_fusion(int(sys.argv[2]))
    base = run(1, 1, n, steps, 1)
    print(json.dumps({"decomp": "1x1", "ms_per_step": base / steps * 1e3}), flush=True)
    for (PX, PY) in ((1, 2), (2, 1), (2, 2)):
        for ov in (1, 0):
            t = run(PX, PY, n, steps, ov)
            print(json.dumps({"decomp": f"{PX}x{PY}", "overlap": ov, "ms_per_step": t / steps * 1e3,
                              "ratio_vs_ideal": t / (base * PX * PY)}), flush=True)


if __name__ == "__main__":
    main()
