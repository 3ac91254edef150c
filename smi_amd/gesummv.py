"""Host mirror of gesummv_smi (examples/host/gesummv_smi.cpp).

Reference test data: A[i][j] = B[i][j] = i, x = 1 (gesummv_smi.cpp:22-36);
acceptance: relative error < 1e-4 against sgemv(beta, B) followed by
sgemv(alpha, A, +y) (:40-46, 299-313).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .comm import Comm


def reference_matrix(n: int, m: int) -> np.ndarray:
    """generate_float_matrix: A[i][j] = i (gesummv_smi.cpp:22-29)."""
    return np.repeat(np.arange(n, dtype=np.float32)[:, None], m, axis=1)


def reference_vector(m: int) -> np.ndarray:
    """generate_float_vector: x = 1 (gesummv_smi.cpp:31-36)."""
    return np.ones(m, dtype=np.float32)


def gemv_rows(A: torch.Tensor, B: torch.Tensor | None, x: torch.Tensor, alpha: float, beta: float,
              y: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """Local rows: y = fold(A, alpha) + fold(B, beta) (smi_gemv_rows)."""
    n, m = A.shape
    if y is None:
        y = torch.empty(n, dtype=torch.float32, device=A.device)
    _lib.call("smi_gemv_rows", A.data_ptr(), None if B is None else B.data_ptr(), x.data_ptr(),
              y.data_ptr(), n, m, A.stride(0), float(alpha), float(beta), _lib.stream_handle(stream))
    return y


def gesummv(comm: Comm, A_rows: torch.Tensor, B_rows: torch.Tensor, x: torch.Tensor, n_global: int,
            alpha: float, beta: float, y: torch.Tensor | None = None, root: int = 0,
            stream=None) -> torch.Tensor | None:
    """Row-sharded gesummv; the full y lands on `root`."""
    m = x.numel()
    if comm.rank == root and y is None:
        y = torch.empty(n_global, dtype=torch.float32, device=x.device)
    _lib.call("smi_gesummv", comm.handle, A_rows.data_ptr(), B_rows.data_ptr(), x.data_ptr(),
              None if y is None else y.data_ptr(), n_global, m, float(alpha), float(beta), root,
              _lib.stream_handle(stream))
    return y


def row_range(n_global: int, size: int, rank: int) -> tuple[int, int]:
    """Rows owned by `rank` (same split as smi_gesummv)."""
    return n_global * rank // size, n_global * (rank + 1) // size
