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
