"""Live per-kernel timing through the C ABI (include/smi/profiling.h)."""
from __future__ import annotations

import ctypes

from . import _lib

SWEEP = _lib.PROF_STENCIL_SWEEP
EDGE = _lib.PROF_STENCIL_EDGE
REDUCE_FOLD = _lib.PROF_REDUCE_FOLD
GEMV = _lib.PROF_GEMV
SWEEPK = _lib.PROF_STENCIL_SWEEPK
KMEANS_ASSIGN = _lib.PROF_KMEANS_ASSIGN
KMEANS_FOLD = _lib.PROF_KMEANS_FOLD


def enable(on: bool = True) -> None:
    _lib.call("smi_prof_enable", 1 if on else 0)


def reset() -> None:
    _lib.call("smi_prof_reset")


def read(kernel: int) -> tuple[float, int]:
    """(summed kernel milliseconds, number of timed launches)."""
    ms = ctypes.c_double()
    n = ctypes.c_long()
    _lib.call("smi_prof_read", kernel, ctypes.byref(ms), ctypes.byref(n))
    return ms.value, n.value


def read_tag(kernel: int, tag: int = -1) -> tuple[float, int, float]:
    """(summed milliseconds, launches, summed algorithmic units -- cell-steps
    for the stencil kernels) of the launches of `kernel` recorded with `tag`
    (the K of a K-step sweep; -1: every tag)."""
    ms = ctypes.c_double()
    n = ctypes.c_long()
    u = ctypes.c_double()
    _lib.call("smi_prof_read_tag", kernel, tag, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(u))
    return ms.value, n.value, u.value


def entries() -> list[tuple[int, int]]:
    """Distinct (kernel, tag) pairs recorded since the last reset."""
    n = ctypes.c_int()
    _lib.call("smi_prof_list", None, None, 0, ctypes.byref(n))
    k = (ctypes.c_int * max(n.value, 1))()
    t = (ctypes.c_int * max(n.value, 1))()
    _lib.call("smi_prof_list", k, t, n.value, ctypes.byref(n))
    return [(k[i], t[i]) for i in range(n.value)]


NAMES = {SWEEP: "sweep", EDGE: "edge", REDUCE_FOLD: "reduce_fold", GEMV: "gemv", SWEEPK: "sweepk",
         KMEANS_ASSIGN: "kmeans_assign", KMEANS_FOLD: "kmeans_fold"}
