"""Communicator bring-up (host mirror of SmiInit_<program>,
codegen/templates/host_hlslib.cl:8-90, and of the MPI rank/size setup in
examples/host/stencil_smi.cpp:128-135).

* :meth:`Comm.from_env` -- one process per GPU (torchrun): rank 0 creates the
  RCCL unique id through the C ABI, the torch.distributed store carries the
  128 bytes to every rank, and each rank builds its RCCL communicator.
* :class:`LocalGroup` -- ranks as host threads of one process (all on one
  GPU), transfers are device-to-device copies: used by the multi-rank parity
  tests on the single-GPU test box.
"""
from __future__ import annotations

import ctypes
import os
import threading

from . import _lib


class Comm:
    def __init__(self, c: _lib.SMI_Comm, device: int):
        self._c = c
        self.device = device
        self._alive = True

    @property
    def rank(self) -> int:
        return self._c.rank

    @property
    def size(self) -> int:
        return self._c.size

    @property
    def handle(self) -> _lib.SMI_Comm:
        if not self._alive:
            raise _lib.SMIError("communicator finalized")
        return self._c

    def dup(self) -> "Comm":
        """smi_comm_dup: a communicator over the same ranks whose bulk
        operations are matched independently of this one's (one per port for
        concurrent bulk collectives from different threads).  Collective."""
        c = _lib.SMI_Comm()
        _lib.call("smi_comm_dup", self.handle, ctypes.byref(c))
        return Comm(c, self.device)

    def finalize(self) -> None:
        if self._alive:
            _lib.call("smi_finalize", self._c)
            self._alive = False

    # -- bring-up ---------------------------------------------------------
    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(_lib.SMI_UNIQUE_ID_BYTES)
        _lib.call("smi_get_unique_id", buf, _lib.SMI_UNIQUE_ID_BYTES)
        return buf.raw

    @classmethod
    def create(cls, rank: int, size: int, device: int, unique_id: bytes) -> "Comm":
        c = _lib.SMI_Comm()
        buf = ctypes.create_string_buffer(unique_id, _lib.SMI_UNIQUE_ID_BYTES)
        _lib.call("smi_init", rank, size, device, buf, _lib.SMI_UNIQUE_ID_BYTES, ctypes.byref(c))
        return cls(c, device)

    @classmethod
    def from_env(cls, store=None, device: int | None = None) -> "Comm":
        """RANK / WORLD_SIZE / LOCAL_RANK from the torchrun environment; the
        unique id goes through `store` (default: torch.distributed's default
        store, which requires init_process_group to have run)."""
        rank = int(os.environ.get("RANK", "0"))
        size = int(os.environ.get("WORLD_SIZE", "1"))
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        uid = exchange_unique_id(rank, size, store)
        return cls.create(rank, size, device, uid)


def exchange_unique_id(rank: int, size: int, store=None, key: str = "smi_amd/uid") -> bytes:
    """Rank 0 generates the RCCL unique id; every rank returns the same bytes."""
    if size == 1:
        return Comm.unique_id()
    if store is None:
        import torch.distributed as dist
        store = dist.distributed_c10d._get_default_store()
    if rank == 0:
        uid = Comm.unique_id()
        store.set(key, uid)
        return uid
    return bytes(store.get(key))


class LocalGroup:
    """`size` ranks run as host threads of this process, sharing `device`."""

    def __init__(self, size: int, device: int = 0):
        gid = ctypes.c_int()
        _lib.call("smi_local_group_create", size, ctypes.byref(gid))
        self.group_id = gid.value
        self.size = size
        self.device = device

    def comm(self, rank: int) -> Comm:
        c = _lib.SMI_Comm()
        _lib.call("smi_init_local", self.group_id, rank, self.device, ctypes.byref(c))
        return Comm(c, self.device)

    def run(self, fn, *args):
        """Run fn(comm, *args) on `size` threads (one per rank); returns the
        per-rank results and re-raises the first exception."""
        results = [None] * self.size
        errors = [None] * self.size

        def body(r):
            import torch
            torch.cuda.set_device(self.device)
            comm = None
            try:
                comm = self.comm(r)
                results[r] = fn(comm, *args)
            except BaseException as e:  # noqa: BLE001
                errors[r] = e
            finally:
                if comm is not None:
                    try:
                        comm.finalize()
                    except Exception as e:  # noqa: BLE001
                        errors[r] = errors[r] or e

        threads = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(self.size)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=600)
            if t.is_alive():
                raise TimeoutError("local group rank did not finish (deadlock?)")
        for e in errors:
            if e is not None:
                raise e
        return results
