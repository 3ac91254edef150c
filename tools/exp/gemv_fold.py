#!/usr/bin/env python3
"""Experiment: gemv_rows row-split vs one-wave-per-row over shard heights, and
the reduce fold's sensitivity to the contribution rows' stride.

    SMI_GEMV_VARIANT=0|1 python tools/exp/gemv_fold.py
One JSON object per line; kernel times are HIP events on the launch stream.
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import smi_amd  # noqa: E402
from smi_amd import collectives, gesummv, profiling  # noqa: E402

PEAK = 8000.0


def timed(fn, kernel, reps=20):
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


def main():
    smi_amd.load()
    dev = torch.device("cuda", 0)
    var = os.environ.get("SMI_GEMV_VARIANT", "0")
    g = torch.Generator(device=dev).manual_seed(7)
    m = 32768
    x = torch.rand(m, device=dev, generator=g) * 2 - 1
    for n in (1024, 2048, 4096, 8192, 16384, 32768):
        A = torch.rand(n, m, device=dev, generator=g) * 2 - 1
        B = torch.rand(n, m, device=dev, generator=g) * 2 - 1
        y = torch.empty(n, device=dev)
        ms = timed(lambda: gesummv.gemv_rows(A, B, x, 1.5, 0.5, y), profiling.GEMV)
        byts = 4 * (2 * n * m + m + n)
        print(json.dumps({"exp": "gemv", "variant": var, "rows": n, "cols": m, "avg_ms": round(ms, 4),
                          "GB/s": round(byts / ms / 1e6, 1), "frac": round(byts / ms / 1e6 / PEAK, 4),
                          "y_sha": hashlib.sha1(y.cpu().numpy().tobytes()).hexdigest()[:12]}), flush=True)
        del A, B
    if var != "0":
        return
    cnt, nr = 1 << 26, 8
    for pad in (0, 1024, 4096 + 256, 65536 + 4096):
        c = torch.rand(nr, cnt + pad, device=dev, generator=g)[:, :cnt]
        out = torch.empty(cnt, device=dev)
        ms = timed(lambda: collectives.reduce_fold(c, "add", out), profiling.REDUCE_FOLD)
        byts = 4 * cnt * (nr + 1)
        print(json.dumps({"exp": "fold", "pad_elems": pad, "count": cnt, "avg_ms": round(ms, 4),
                          "GB/s": round(byts / ms / 1e6, 1), "frac": round(byts / ms / 1e6 / PEAK, 4)}),
              flush=True)
        del c, out


if __name__ == "__main__":
    main()
