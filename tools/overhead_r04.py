#!/usr/bin/env python3
"""Where the non-kernel time of bench.py's short timed region goes (VERDICT r3
item 4): for the driver's config (8192^2, T = 20, one K = 20 pass) time, over
many repetitions,
  sync_idle   -- torch.cuda.synchronize() on an idle device
  enqueue     -- the host call stencil.run(...) alone (no sync)
  region      -- barrier-free version of bench.py's timed region: sync, t0,
                 stencil.run, sync, t1
  kernel      -- HIP events around the same call on the stream
and, to split the enqueue: the Python wrapper with the library call stubbed
out (wrapper_us), the bare ctypes call with pre-built arguments (ctypes_*),
and a one-element torch kernel's region (floor_region_us: launch + dispatch +
sync of the smallest kernel).  Prints medians in microseconds (one JSON line).
"""
import ctypes
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import smi_amd  # noqa: E402
from smi_amd import _lib, stencil  # noqa: E402

N, T, REPS = 8192, int(sys.argv[1]) if len(sys.argv) > 1 else 20, 200
torch.cuda.set_device(0)
comm = smi_amd.LocalGroup(1).comm(0)
a = torch.rand((N, N), device="cuda")
b = torch.empty_like(a)
s = torch.cuda.Stream()


def med(xs):
    return round(statistics.median(xs) * 1e6, 2)


out = {"T": T}
with torch.cuda.stream(s):
    for _ in range(20):
        stencil.run(comm, a, T, 1, 1, b)
    torch.cuda.synchronize()
    sync_idle, enq, region, kern = [], [], [], []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(REPS):
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        sync_idle.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        stencil.run(comm, a, T, 1, 1, b)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append(t1 - t0)
        region.append(t2 - t0)
        e0.record(s)
        stencil.run(comm, a, T, 1, 1, b)
        e1.record(s)
        torch.cuda.synchronize()
        kern.append(e0.elapsed_time(e1) * 1e-3)
    out.update({"sync_idle_us": med(sync_idle), "enqueue_us": med(enq), "region_us": med(region),
                "kernel_events_us": med(kern), "region_minus_kernel_us": round(med(region) - med(kern), 2)})

    # the wrapper alone (library call stubbed out)
    real_call = _lib.call
    _lib.call = lambda name, *args: None
    try:
        w = []
        for _ in range(REPS):
            t0 = time.perf_counter()
            stencil.run(comm, a, T, 1, 1, b)
            w.append(time.perf_counter() - t0)
    finally:
        _lib.call = real_call
    out["wrapper_us"] = med(w)

    # the bare ctypes call, arguments built once
    fn = _lib.load().smi_stencil_run
    idx = ctypes.c_int()
    args = (comm.handle, a.data_ptr(), b.data_ptr(), N, N, 1, 1, T, s.cuda_stream, ctypes.byref(idx))
    ce, cr = [], []
    for _ in range(REPS):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc = fn(*args)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        assert rc == 0
        ce.append(t1 - t0)
        cr.append(t2 - t0)
    out.update({"ctypes_enqueue_us": med(ce), "ctypes_region_us": med(cr)})

    # floor: the smallest torch kernel, launch + dispatch + sync
    x = torch.zeros(1, device="cuda")
    fl = []
    for _ in range(REPS):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x.add_(1.0)
        torch.cuda.synchronize()
        fl.append(time.perf_counter() - t0)
    out["floor_region_us"] = med(fl)
print(json.dumps(out))
comm.finalize()
