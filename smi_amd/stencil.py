"""Host mirror of the stencil_smi program (examples/host/stencil_smi.cpp).

Same decomposition and naming as the reference host: the X x Y grid is split
into PX x PY tiles, rank = i_px*PY + i_py owns rows [i_px*X_LOCAL, ..) and
columns [i_py*Y_LOCAL, ..) (SplitMemory / CombineMemory,
stencil_smi.cpp:48-62,80-93; rank map :133-134); the default test grid is 0
in the interior and 1 on the four edges (:175-187).  Every sweep runs in the
HIP kernels of libsmi_amd.so; device buffers are torch tensors.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .comm import Comm

BOUNDARY_VALUE = 1.0  # examples/include/stencil.h.in:8


def init_grid(X: int, Y: int) -> np.ndarray:
    """0 interior, BOUNDARY_VALUE on the four edges (stencil_smi.cpp:175-187)."""
    g = np.zeros((X, Y), dtype=np.float32)
    g[0, :] = BOUNDARY_VALUE
    g[X - 1, :] = BOUNDARY_VALUE
    g[:, 0] = BOUNDARY_VALUE
    g[:, Y - 1] = BOUNDARY_VALUE
    return g


def split_memory(grid: np.ndarray, PX: int, PY: int) -> list[np.ndarray]:
    """SplitMemory (stencil_smi.cpp:48-62): tile of rank px*PY+py."""
    X, Y = grid.shape
    if X % PX or Y % PY:
        raise ValueError("grid not divisible by the process grid")
    XL, YL = X // PX, Y // PY
    return [np.ascontiguousarray(grid[px * XL:(px + 1) * XL, py * YL:(py + 1) * YL])
            for px in range(PX) for py in range(PY)]


def combine_memory(tiles: list[np.ndarray], PX: int, PY: int) -> np.ndarray:
    """CombineMemory (stencil_smi.cpp:80-93)."""
    XL, YL = tiles[0].shape
    out = np.empty((PX * XL, PY * YL), dtype=np.float32)
    for px in range(PX):
        for py in range(PY):
            out[px * XL:(px + 1) * XL, py * YL:(py + 1) * YL] = tiles[px * PY + py]
    return out


def rank_coords(rank: int, PY: int) -> tuple[int, int]:
    """i_px = rank / PY, i_py = rank % PY (stencil_smi.cpp:133-134)."""
    return rank // PY, rank % PY


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def step(inp: torch.Tensor, out: torch.Tensor, modes=(0, 0, 0, 0), halos=(None, None, None, None),
         send_left: torch.Tensor | None = None, send_right: torch.Tensor | None = None,
         stream=None) -> None:
    """One Jacobi step of one tile (smi_stencil_step).  modes per side
    (top, bottom, left, right): SIDE_COPY / SIDE_HALO / SIDE_SKIP."""
    X, Y = inp.shape
    m = (ctypes.c_int * 4)(*modes)
    h = (ctypes.c_void_p * 4)(*[_ptr(t) for t in halos])
    _lib.call("smi_stencil_step", inp.data_ptr(), out.data_ptr(), X, Y, m, h,
              _ptr(send_left), _ptr(send_right), _lib.stream_handle(stream))


def run(comm: Comm, tile: torch.Tensor, timesteps: int, PX: int, PY: int,
        scratch: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """The whole stencil_smi run on this rank's tile (smi_stencil_run):
    returns the tensor (tile or scratch) holding the result, like the
    reference's copy-back of half timesteps%2 (stencil_smi.cpp:344)."""
    if scratch is None:
        scratch = torch.empty_like(tile)
    X, Y = tile.shape
    idx = ctypes.c_int()
    _lib.call("smi_stencil_run", comm.handle, tile.data_ptr(), scratch.data_ptr(), X, Y, PX, PY,
              timesteps, _lib.stream_handle(stream, tile.get_device()), ctypes.byref(idx))
    return tile if idx.value == 0 else scratch


class _Phase(ctypes.Structure):
    _fields_ = [("steps_per_pass", ctypes.c_int), ("passes", ctypes.c_int)]


def plan(x_local: int, y_local: int, PX: int, PY: int, rank: int, timesteps: int) -> dict:
    """The schedule smi_stencil_run follows on `rank` (host only, no GPU):
    phases [(steps_per_pass, passes), ...], the neighbour ranks (top, bottom,
    left, right, tl, tr, bl, br; -1 on the global edge) and the index of the
    buffer that ends up holding the result."""
    ph = (_Phase * 4)()
    n = ctypes.c_int()
    nb = (ctypes.c_int * 8)()
    ri = ctypes.c_int()
    _lib.call("smi_stencil_plan", x_local, y_local, PX, PY, rank, timesteps, ph, 4, ctypes.byref(n), nb,
              ctypes.byref(ri))
    return {"phases": [(ph[i].steps_per_pass, ph[i].passes) for i in range(n.value)],
            "neighbours": list(nb), "result_index": ri.value}


def set_tuning(rows_per_wave: int = 0, rows_in_flight: int = 0, nontemporal: int = -1,
               overlap: int = -1) -> None:
    _lib.call("smi_stencil_set_tuning", rows_per_wave, rows_in_flight, nontemporal, overlap)


def get_tuning() -> dict:
    v = [ctypes.c_int() for _ in range(4)]
    _lib.call("smi_stencil_get_tuning", *[ctypes.byref(x) for x in v])
    return dict(rows_per_wave=v[0].value, rows_in_flight=v[1].value, nontemporal=v[2].value,
                overlap=v[3].value)


def set_bands(reserve_waves: int = -1, interior_rounds: int = -1) -> None:
    """Multi-rank K-step scheduling (bit-neutral): wave slots the interior
    sweep leaves free for the band kernel and the exchange (0 = none) and
    rounds of resident waves the interior sweep is cut into.  -1 keeps a
    setting."""
    _lib.call("smi_stencil_set_bands", reserve_waves, interior_rounds)


def get_bands() -> dict:
    v = [ctypes.c_int() for _ in range(2)]
    _lib.call("smi_stencil_get_bands", *[ctypes.byref(x) for x in v])
    return dict(reserve_waves=v[0].value, interior_rounds=v[1].value)


def set_fusion(steps_per_pass: int = 0, rows_per_wave: int = 0, rows_in_flight: int = 0) -> None:
    """Up to steps_per_pass (1..20) Jacobi steps fused per pass over HBM
    (same bits for every setting); the remainder of a run is one shallower
    pass (smi_stencil_plan)."""
    _lib.call("smi_stencil_set_fusion", steps_per_pass, rows_per_wave, rows_in_flight)


def get_fusion() -> dict:
    v = [ctypes.c_int() for _ in range(3)]
    _lib.call("smi_stencil_get_fusion", *[ctypes.byref(x) for x in v])
    return dict(steps_per_pass=v[0].value, rows_per_wave=v[1].value, rows_in_flight=v[2].value)


def set_band_kernel(lean: int = -1) -> None:
    """Multi-rank K >= 13 band kernel (bit-neutral): 1 = lean, beside the
    interior sweep (default); 0 = one wave per segment.  -1 keeps it."""
    _lib.call("smi_stencil_set_band_kernel", lean)


def get_band_kernel() -> int:
    v = ctypes.c_int()
    _lib.call("smi_stencil_get_band_kernel", ctypes.byref(v))
    return v.value


def set_join(host_join: int = -1) -> None:
    """Multi-rank K-step pass join (bit-neutral): 1 = host-observed (default;
    the host runs about one pass ahead of the GPU), 0 = a device-side stream
    wait per pass (the host enqueues the whole run; ~3 % more GPU time per
    pass, host stalls absorbed).  -1 keeps it (smi_stencil_set_join)."""
    _lib.call("smi_stencil_set_join", host_join)


def get_join() -> int:
    v = ctypes.c_int()
    _lib.call("smi_stencil_get_join", ctypes.byref(v))
    return v.value


def deep_geometry(rows: int, cols: int, k: int, side_mask: int = 0) -> dict:
    """The rotating-ring sweep's work split for one K-step pass (host only;
    with no device set the launch's waves first: set_deep(waves=...))."""
    v = [ctypes.c_int() for _ in range(5)]
    _lib.call("smi_stencil_deep_geometry", rows, cols, k, side_mask, *[ctypes.byref(x) for x in v])
    return dict(waves=v[0].value, strips=v[1].value, row_blocks=v[2].value, row_blocks_edge=v[3].value,
                min_block_rows=v[4].value)


def set_deep(ce16: int = -1, rev16: int = -1, waves: int = -1) -> None:
    """Rotating-ring sweep (K = 13..20) geometry, scheduling only: extra work
    of edge-column strips / upward bottom blocks in 16ths, waves per launch
    (0 = one round of resident waves).  -1 keeps a setting."""
    _lib.call("smi_stencil_set_deep", ce16, rev16, waves)


def get_deep() -> dict:
    v = [ctypes.c_int() for _ in range(3)]
    _lib.call("smi_stencil_get_deep", *[ctypes.byref(x) for x in v])
    return dict(ce16=v[0].value, rev16=v[1].value, waves=v[2].value)
