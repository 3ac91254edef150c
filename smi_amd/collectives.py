"""Host mirror of SMI_Reduce / SMI_Bcast on whole device buffers.

Reference call shape: every rank opens a channel with the same count, type,
op, port and root, then streams its elements (microbenchmarks/kernels/
reduce.cl:9-26, broadcast.cl:9-23).  Here one call moves the whole buffer:
reduce(comm, send, recv, op, root, port) / bcast(comm, buf, root, port).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .comm import Comm

TORCH_TO_SMI = {
    torch.int32: _lib.SMI_INT,
    torch.float32: _lib.SMI_FLOAT,
    torch.float64: _lib.SMI_DOUBLE,
    torch.int8: _lib.SMI_CHAR,
    torch.int16: _lib.SMI_SHORT,
}
OPS = {"add": _lib.SMI_ADD, "max": _lib.SMI_MAX, "min": _lib.SMI_MIN}


def _smi_type(t: torch.Tensor) -> int:
    try:
        return TORCH_TO_SMI[t.dtype]
    except KeyError:
        raise _lib.SMIError(f"unsupported dtype {t.dtype}") from None


def _op(op) -> int:
    return OPS[op] if isinstance(op, str) else int(op)


def reduce(comm: Comm, send: torch.Tensor, recv: torch.Tensor | None, op="add", root: int = 0,
           port: int = 0, stream=None) -> None:
    """Element-wise reduce of every rank's `send` into the root's `recv`
    (codegen/templates/reduce.cl fold, canonical rank order)."""
    rptr = recv.data_ptr() if recv is not None else None
    _lib.call("smi_reduce", comm.handle, send.data_ptr(), rptr, send.numel(), _smi_type(send), _op(op),
              root, port, _lib.stream_handle(stream))


def bcast(comm: Comm, buf: torch.Tensor, root: int = 0, port: int = 0, stream=None) -> None:
    """Root's `buf` copied into every rank's `buf` (bcast.cl)."""
    _lib.call("smi_bcast", comm.handle, buf.data_ptr(), buf.numel(), _smi_type(buf), root, port,
              _lib.stream_handle(stream))


def set_pipeline_bytes(piece_bytes: int) -> None:
    """Piece size (bytes per owner chunk) of the pipelined reduce/bcast;
    0 = one piece.  Process-wide, same value on every rank."""
    _lib.call("smi_set_pipeline_bytes", piece_bytes)


def get_pipeline_bytes() -> int:
    v = ctypes.c_size_t()
    _lib.call("smi_get_pipeline_bytes", ctypes.byref(v))
    return v.value


def reduce_fold(contribs: torch.Tensor, op="add", out: torch.Tensor | None = None,
                stream=None) -> torch.Tensor:
    """Local fold of a (nranks, count) tensor in row order (smi_reduce_fold)."""
    n, count = contribs.shape
    if out is None:
        out = torch.empty(count, dtype=contribs.dtype, device=contribs.device)
    _lib.call("smi_reduce_fold", contribs.data_ptr(), out.data_ptr(), n, count, contribs.stride(0),
              _smi_type(contribs), _op(op), _lib.stream_handle(stream))
    return out


def scatter(comm: Comm, send: torch.Tensor | None, recv: torch.Tensor, root: int = 0, port: int = 0,
            stream=None) -> None:
    """Root's `send` (size*count elements) split over the ranks' `recv`."""
    _lib.call("smi_scatter", comm.handle, None if send is None else send.data_ptr(), recv.data_ptr(),
              recv.numel(), _smi_type(recv), root, port, _lib.stream_handle(stream))


def gather(comm: Comm, send: torch.Tensor, recv: torch.Tensor | None, root: int = 0, port: int = 0,
           stream=None) -> None:
    """Every rank's `send` (count elements) concatenated in rank order in the
    root's `recv`."""
    _lib.call("smi_gather", comm.handle, send.data_ptr(), None if recv is None else recv.data_ptr(),
              send.numel(), _smi_type(send), root, port, _lib.stream_handle(stream))


def send(comm: Comm, buf: torch.Tensor, dest: int, port: int = 0, stream=None) -> None:
    """Bulk send channel: every element of device tensor `buf` to `dest`
    (smi_send; a SMI_Open_send_channel + SMI_Push loop in the reference)."""
    _lib.call("smi_send", comm.handle, buf.data_ptr(), buf.numel(), _smi_type(buf), dest, port,
              _lib.stream_handle(stream))


def recv(comm: Comm, buf: torch.Tensor, source: int, port: int = 0, stream=None) -> None:
    """Bulk receive channel into device tensor `buf` from `source` (smi_recv)."""
    _lib.call("smi_recv", comm.handle, buf.data_ptr(), buf.numel(), _smi_type(buf), source, port,
              _lib.stream_handle(stream))
