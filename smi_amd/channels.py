"""Host mirror of the element-granular channel API (include/smi/push.h,
pop.h, bcast.h, reduce.h, scatter.h, gather.h).

Same names and call shape as the reference primitives
(include/smi/push.h:19-48, pop.h:20-39, bcast.h:43-63, reduce.h:55-76,
scatter.h:49-72, gather.h:47-68): open a transient channel, then push / pop /
bcast / reduce / scatter / gather ONE element per call.  A failed call raises
SMIError (the C descriptors carry the status; the reference's are void).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .comm import Comm

_FIELDS = [("handle", ctypes.c_int), ("status", ctypes.c_int), ("my_rank", ctypes.c_int),
           ("num_ranks", ctypes.c_int), ("peer", ctypes.c_int), ("port", ctypes.c_int),
           ("data_type", ctypes.c_int), ("message_size", ctypes.c_uint),
           ("processed_elements", ctypes.c_uint)]


class SMI_Channel(ctypes.Structure):
    _fields_ = _FIELDS


class SMI_BChannel(ctypes.Structure):
    _fields_ = _FIELDS


class SMI_RChannel(ctypes.Structure):
    _fields_ = _FIELDS + [("reduce_op", ctypes.c_int)]


class SMI_ScatterChannel(ctypes.Structure):
    _fields_ = _FIELDS + [("recv_count", ctypes.c_uint)]


class SMI_GatherChannel(ctypes.Structure):
    _fields_ = _FIELDS + [("recv_count", ctypes.c_uint)]


NP = {_lib.SMI_INT: np.int32, _lib.SMI_FLOAT: np.float32, _lib.SMI_DOUBLE: np.float64,
      _lib.SMI_CHAR: np.int8, _lib.SMI_SHORT: np.int16}

_C = _lib.SMI_Comm
_I = ctypes.c_int
_P = ctypes.c_void_p
SIGNATURES = {
    "SMI_Open_send_channel": (SMI_Channel, [_I, _I, _I, _I, _C]),
    "SMI_Open_send_channel_ad": (SMI_Channel, [_I, _I, _I, _I, _C, _I]),
    "SMI_Open_receive_channel": (SMI_Channel, [_I, _I, _I, _I, _C]),
    "SMI_Open_receive_channel_ad": (SMI_Channel, [_I, _I, _I, _I, _C, _I]),
    "SMI_Push": (None, [ctypes.POINTER(SMI_Channel), _P]),
    "SMI_Push_flush": (None, [ctypes.POINTER(SMI_Channel), _P, _I]),
    "SMI_Pop": (None, [ctypes.POINTER(SMI_Channel), _P]),
    "SMI_Open_bcast_channel": (SMI_BChannel, [_I, _I, _I, _I, _C]),
    "SMI_Open_bcast_channel_ad": (SMI_BChannel, [_I, _I, _I, _I, _C, _I]),
    "SMI_Bcast": (None, [ctypes.POINTER(SMI_BChannel), _P]),
    "SMI_Open_reduce_channel": (SMI_RChannel, [_I, _I, _I, _I, _I, _C]),
    "SMI_Open_reduce_channel_ad": (SMI_RChannel, [_I, _I, _I, _I, _I, _C, _I]),
    "SMI_Reduce": (None, [ctypes.POINTER(SMI_RChannel), _P, _P]),
    "SMI_Open_scatter_channel": (SMI_ScatterChannel, [_I, _I, _I, _I, _I, _C]),
    "SMI_Open_scatter_channel_ad": (SMI_ScatterChannel, [_I, _I, _I, _I, _I, _C, _I]),
    "SMI_Scatter": (None, [ctypes.POINTER(SMI_ScatterChannel), _P, _P]),
    "SMI_Open_gather_channel": (SMI_GatherChannel, [_I, _I, _I, _I, _I, _C]),
    "SMI_Open_gather_channel_ad": (SMI_GatherChannel, [_I, _I, _I, _I, _I, _C, _I]),
    "SMI_Gather": (None, [ctypes.POINTER(SMI_GatherChannel), _P, _P]),
}
_lib.SIGNATURES.update(SIGNATURES)


def _fn(name):
    lib = _lib.load()
    f = getattr(lib, name)
    res, args = SIGNATURES[name]
    f.restype = res
    f.argtypes = args
    return f


def _check(chan, what):
    if chan.status != 0:
        _lib.check(chan.status, what)


class _Elem:
    """One host element of an SMI data type, passed by pointer."""

    def __init__(self, dtype: int, value=0):
        self.np = NP[dtype]
        self.buf = np.array([value], dtype=self.np)

    @property
    def ptr(self):
        return self.buf.ctypes.data

    @property
    def value(self):
        return self.buf[0]


class Channel:
    """Point-to-point transient channel (send or receive side)."""

    def __init__(self, c, dtype):
        self.c = c
        self.dtype = dtype
        self._tmp = _Elem(dtype)
        _check(c, "open channel")

    def push(self, value, immediate: bool = False):
        self._tmp.buf[0] = value
        _fn("SMI_Push_flush")(ctypes.byref(self.c), self._tmp.ptr, 1 if immediate else 0)
        _check(self.c, "SMI_Push")

    def pop(self):
        _fn("SMI_Pop")(ctypes.byref(self.c), self._tmp.ptr)
        _check(self.c, "SMI_Pop")
        return self._tmp.value


def open_send_channel(count: int, dtype: int, destination: int, port: int, comm: Comm,
                      asynch_degree: int | None = None) -> Channel:
    """SMI_Open_send_channel, or SMI_Open_send_channel_ad when asynch_degree
    is given (at most that many elements packed per message)."""
    if asynch_degree is None:
        return Channel(_fn("SMI_Open_send_channel")(count, dtype, destination, port, comm.handle), dtype)
    return Channel(_fn("SMI_Open_send_channel_ad")(count, dtype, destination, port, comm.handle, asynch_degree),
                   dtype)


def open_receive_channel(count: int, dtype: int, source: int, port: int, comm: Comm,
                         asynch_degree: int | None = None) -> Channel:
    if asynch_degree is None:
        return Channel(_fn("SMI_Open_receive_channel")(count, dtype, source, port, comm.handle), dtype)
    return Channel(_fn("SMI_Open_receive_channel_ad")(count, dtype, source, port, comm.handle, asynch_degree),
                   dtype)


class BChannel:
    def __init__(self, count, dtype, port, root, comm: Comm, asynch_degree: int | None = None):
        if asynch_degree is None:
            self.c = _fn("SMI_Open_bcast_channel")(count, dtype, port, root, comm.handle)
        else:
            self.c = _fn("SMI_Open_bcast_channel_ad")(count, dtype, port, root, comm.handle, asynch_degree)
        self._tmp = _Elem(dtype)
        _check(self.c, "SMI_Open_bcast_channel")

    def bcast(self, value=0):
        self._tmp.buf[0] = value
        _fn("SMI_Bcast")(ctypes.byref(self.c), self._tmp.ptr)
        _check(self.c, "SMI_Bcast")
        return self._tmp.value


class RChannel:
    def __init__(self, count, dtype, op, port, root, comm: Comm, asynch_degree: int | None = None):
        if asynch_degree is None:
            self.c = _fn("SMI_Open_reduce_channel")(count, dtype, op, port, root, comm.handle)
        else:
            self.c = _fn("SMI_Open_reduce_channel_ad")(count, dtype, op, port, root, comm.handle, asynch_degree)
        self._s = _Elem(dtype)
        self._r = _Elem(dtype)
        _check(self.c, "SMI_Open_reduce_channel")

    def reduce(self, value):
        self._s.buf[0] = value
        _fn("SMI_Reduce")(ctypes.byref(self.c), self._s.ptr, self._r.ptr)
        _check(self.c, "SMI_Reduce")
        return self._r.value


class ScatterChannel:
    def __init__(self, send_count, recv_count, dtype, port, root, comm: Comm):
        self.c = _fn("SMI_Open_scatter_channel")(send_count, recv_count, dtype, port, root, comm.handle)
        self._s = _Elem(dtype)
        self._r = _Elem(dtype)
        _check(self.c, "SMI_Open_scatter_channel")

    def scatter(self, value=0):
        self._s.buf[0] = value
        _fn("SMI_Scatter")(ctypes.byref(self.c), self._s.ptr, self._r.ptr)
        _check(self.c, "SMI_Scatter")
        return self._r.value


class GatherChannel:
    def __init__(self, send_count, recv_count, dtype, port, root, comm: Comm):
        self.c = _fn("SMI_Open_gather_channel")(send_count, recv_count, dtype, port, root, comm.handle)
        self._s = _Elem(dtype)
        self._r = _Elem(dtype)
        _check(self.c, "SMI_Open_gather_channel")

    def gather(self, value=0):
        self._s.buf[0] = value
        _fn("SMI_Gather")(ctypes.byref(self.c), self._s.ptr, self._r.ptr)
        _check(self.c, "SMI_Gather")
        return self._r.value
