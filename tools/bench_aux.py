#!/usr/bin/env python3
"""Microbenchmarks of the non-stencil kernels on one GPU (GB/s vs HBM peak).

    python tools/bench_aux.py [--rows 4096] [--cols 32768] [--fold-count 67108864]

* gemv_rows_kernel -- BASELINE config 5 per-GPU share of gesummv (32768^2 fp32
  row-sharded over 8 GPUs: 4096 rows of A and of B, 1 GiB): algorithmic bytes
  = 4*(2*n*m + m + n) per launch.
* fold_kernel -- the owner-side canonical fold of smi_reduce over n=8
  contributions of `count` fp32: algorithmic bytes = 4*count*(n+1).
* kmeans_smi (reference build shape: 8 clusters x 64 dims, W = 16) on one
  rank's `kmeans-points` points: assign_kernel (algorithmic bytes = the point
  streamed once + its assignment, 4*dims + 4 per point), the per-cluster sum
  chains (fold_kernel: ns per chain element = time / longest cluster), and
  whole iterations of smi_kmeans.
Kernel times are live HIP-event timings on the launch stream
(include/smi/profiling.h); each line is one JSON object.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import smi_amd  # noqa: E402
from smi_amd import collectives, gesummv, kmeans, profiling  # noqa: E402

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
    ap.add_argument("--kmeans-points", type=int, default=1 << 22)
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
    del c, out

    npts, dims, K, W = a.kmeans_points, kmeans.REFERENCE_DIMS, kmeans.REFERENCE_CLUSTERS, kmeans.REFERENCE_WIDTH
    P, C0 = kmeans.synthetic_points(npts, K, dims, device=dev)
    idx = torch.empty(npts, dtype=torch.int32, device=dev)
    ms = timed(lambda: kmeans.assign(P, C0, W, idx), profiling.KMEANS_ASSIGN, a.reps)
    byts = npts * (4 * dims + 4)
    print(json.dumps({"kernel": "kmeans assign_kernel<REG>", "points": npts, "dims": dims, "clusters": K,
                      "width": W, "avg_ms": round(ms, 4), "bytes": byts, "GB/s": round(byts / ms / 1e6, 1),
                      "frac": round(byts / ms / 1e6 / PEAK, 4)}), flush=True)
    sums = torch.empty((K, dims), device=dev)
    cnts = torch.empty(K, dtype=torch.int32, device=dev)
    ms = timed(lambda: kmeans.accumulate(P, idx, K, sums, cnts), profiling.KMEANS_FOLD, a.reps)
    chain = int(cnts.max())
    print(json.dumps({"kernel": "kmeans fold_kernel (serial fp32 chains)", "points": npts, "longest_chain": chain,
                      "avg_ms": round(ms, 4), "ns_per_chain_element": round(ms * 1e6 / max(chain, 1), 3),
                      "rows_per_s": round(npts / ms * 1e3, 1)}), flush=True)
    comm = smi_amd.LocalGroup(1).comm(0)
    C = C0.clone()
    kmeans.kmeans(comm, P, C, 1, W)
    torch.cuda.synchronize()
    iters = 10
    t0 = time.perf_counter()
    kmeans.kmeans(comm, P, C, iters, W)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    print(json.dumps({"program": "smi_kmeans (1 rank)", "points": npts, "ms_per_iteration": round(dt * 1e3, 4),
                      "points_per_s": round(npts / dt, 1)}), flush=True)
    comm.finalize()


if __name__ == "__main__":
    main()
