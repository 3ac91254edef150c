#!/usr/bin/env python3
"""Microbenchmarks of the non-stencil kernels on one GPU (GB/s vs HBM peak).

    python tools/bench_aux.py [--rows 4096] [--cols 32768] [--fold-count 67108864]

* gemv_rows_kernel -- BASELINE config 5 per-GPU share of gesummv (32768^2 fp32
  row-sharded over 8 GPUs: 4096 rows of A and of B, 1 GiB): algorithmic bytes
  = 4*(2*n*m + m + n) per launch.
* fold_kernel -- the owner-side canonical fold of smi_reduce over n=8
  contributions of `count` fp32: algorithmic bytes = 4*count*(n+1).
Kernel times are live HIP-event timings on the launch stream
(include/smi/profiling.h); each line is one JSON object.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import smi_amd  # noqa: E402
from smi_amd import collectives, gesummv, profiling  # noqa: E402

PEAK = 8000.0


def timed(fn, kernel, reps):
    fn()
    torch.cuda.synchronize()
    profiling.reset()
    profiling.enable(True)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    profiling.enable(False)
    ms, n = profiling.read(kernel)
    return ms / max(n, 1)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4096)
    ap.add_argument("--cols", type=int, default=32768)
    ap.add_argument("--fold-count", type=int, default=1 << 26)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    smi_amd.load()
    dev = torch.device("cuda", 0)

    n, m = a.rows, a.cols
    g = torch.Generator(device=dev).manual_seed(7)
    A = torch.rand(n, m, device=dev, generator=g) * 2 - 1
    B = torch.rand(n, m, device=dev, generator=g) * 2 - 1
    x = torch.rand(m, device=dev, generator=g) * 2 - 1
    y = torch.empty(n, device=dev)
    ms = timed(lambda: gesummv.gemv_rows(A, B, x, 1.5, 0.5, y), profiling.GEMV, a.reps)
    byts = 4 * (2 * n * m + m + n)
    print(json.dumps({"kernel": "gemv_rows_kernel<HAS_B>", "rows": n, "cols": m, "avg_ms": round(ms, 4),
                      "bytes": byts, "GB/s": round(byts / ms / 1e6, 1),
                      "frac": round(byts / ms / 1e6 / PEAK, 4)}), flush=True)
    del A, B

    cnt, nr = a.fold_count, 8
    c = torch.rand(nr, cnt, device=dev, generator=g)
    out = torch.empty(cnt, device=dev)
    ms = timed(lambda: collectives.reduce_fold(c, "add", out), profiling.REDUCE_FOLD, a.reps)
    byts = 4 * cnt * (nr + 1)
    print(json.dumps({"kernel": "fold_kernel<float,4,ADD>", "contributions": nr, "count": cnt,
                      "avg_ms": round(ms, 4), "bytes": byts, "GB/s": round(byts / ms / 1e6, 1),
                      "frac": round(byts / ms / 1e6 / PEAK, 4)}), flush=True)


if __name__ == "__main__":
    main()
