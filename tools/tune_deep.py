#!/usr/bin/env python3
"""Tuning table for the K-step sweep on one GPU: kernel time per pass and per
Jacobi STEP (HIP events around every launch) for steps_per_pass K x rows per
wave (row-block height; -1 = automatic, one round of resident waves).

    python tools/tune_deep.py [N] [passes] [K,K,..] [ht,ht,..]

SMI_LIB_VARIANT selects an experiment build (smi_amd/build.py VARIANT_FLAGS).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import smi_amd  # noqa: E402
from smi_amd import _lib, profiling, stencil  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ks = [int(k) for k in (sys.argv[3].split(",") if len(sys.argv) > 3 else ["12", "8"])]
    hts = [int(h) for h in (sys.argv[4].split(",") if len(sys.argv) > 4 else ["-1"])]
    smi_amd.load()
    comm = smi_amd.LocalGroup(1).comm(0)
    a = torch.rand((n, n), device="cuda")
    b = torch.empty_like(a)
    settings = [(k, ht) for k in ks for ht in hts]
    # warm the clock: ~100 ms of passes
    stencil.set_fusion(12, -1)
    for _ in range(10):
        stencil.run(comm, a, 120, 1, 1, b)
    torch.cuda.synchronize()
    res = {}
    for rnd in range(3):
        for (k, ht) in settings:
            stencil.set_fusion(k, ht)
            stencil.run(comm, a, 2 * k, 1, 1, b)
            torch.cuda.synchronize()
            profiling.reset()
            profiling.enable(True)
            stencil.run(comm, a, passes * k, 1, 1, b)
            torch.cuda.synchronize()
            profiling.enable(False)
            ms, cnt, _ = profiling.read_tag(profiling.SWEEPK if k >= 3 else profiling.SWEEP, k)
            res.setdefault((k, ht), []).append(ms / cnt)
    stencil.set_fusion(12, -1)
    for (k, ht), v in res.items():
        med = sorted(v)[1]
        print(json.dumps({"variant": _lib.variant() or "release", "K": k, "ht": ht, "ms_per_pass": round(med, 5),
                          "ms_per_step": round(med / k, 5), "GCells": round(n * n * k / med / 1e6, 1),
                          "hbm_GBs_if_one_step_of_traffic": round(8 * n * n / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
