"""smi_amd -- MI355X-native hot path of SMI (Streaming Message Interface).

The product is ``libsmi_amd.so`` (C ABI in ``include/smi/*.h``): hand-written
gfx950 HIP kernels for the stencil_smi Jacobi sweep, the SMI_Reduce fold,
the gesummv row GEMV and the kmeans_smi program, plus a native runtime that moves halos and collective
chunks with RCCL over xGMI.  This package is the Python host mirror of the
reference host programs (examples/host/*.cpp, microbenchmarks/host/*.cpp):
device buffers are torch tensors, every compute call goes through the C ABI.
"""
from ._lib import (  # noqa: F401
    SMI_ADD, SMI_CHAR, SMI_DOUBLE, SMI_FLOAT, SMI_INT, SMI_MAX, SMI_MIN, SMI_SHORT,
    SIDE_COPY, SIDE_HALO, SIDE_SKIP, SMIError, load,
)
from .comm import Comm, LocalGroup  # noqa: F401
from . import stencil, collectives, gesummv, kmeans, profiling, channels  # noqa: F401

__all__ = ["Comm", "LocalGroup", "stencil", "collectives", "gesummv", "kmeans", "profiling", "channels", "SMIError", "load"]
