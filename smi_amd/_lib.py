"""ctypes binding of libsmi_amd.so (the C ABI of include/smi/*.h).

torch is imported first on purpose: its wheel ships its own HIP runtime
(libamdhip64.so.7) and RCCL (librccl.so.1); loading them before our library
makes the dynamic linker resolve our library's dependencies to those same
copies, so device pointers, streams and events are shared with torch.

There is no fallback: if the library is missing or fails to load, every
entry point raises.  The product path never touches the CPU oracle.
"""
from __future__ import annotations

import ctypes
import os
import sys

import torch  # noqa: F401  (see module docstring)

from . import build as _build

_lib = None

SMI_SUCCESS = 0
SMI_UNIQUE_ID_BYTES = 128

# include/smi/data_types.h (same values as the reference's data_types.h:10-16)
SMI_INT, SMI_FLOAT, SMI_DOUBLE, SMI_CHAR, SMI_SHORT = 1, 2, 3, 4, 5
# include/smi/reduce.h (reference reduce.h:18-22)
SMI_ADD, SMI_MAX, SMI_MIN = 0, 1, 2
# include/smi/stencil.h
SIDE_COPY, SIDE_HALO, SIDE_SKIP = 0, 1, 2
# include/smi/profiling.h
(PROF_STENCIL_SWEEP, PROF_STENCIL_EDGE, PROF_REDUCE_FOLD, PROF_GEMV, PROF_STENCIL_SWEEPK, PROF_KMEANS_ASSIGN,
 PROF_KMEANS_FOLD) = 0, 1, 2, 3, 4, 5, 6


class SMIError(RuntimeError):
    pass


class SMI_Comm(ctypes.Structure):
    _fields_ = [("rank", ctypes.c_int), ("size", ctypes.c_int), ("handle", ctypes.c_int)]


P = ctypes.c_void_p
I = ctypes.c_int
SZ = ctypes.c_size_t
F = ctypes.c_float

# name -> (restype, argtypes); every symbol declared in include/smi/*.h
SIGNATURES = {
    "smi_last_error": (ctypes.c_char_p, []),
    "smi_get_unique_id": (I, [P, I]),
    "smi_init": (I, [I, I, I, P, I, ctypes.POINTER(SMI_Comm)]),
    "smi_local_group_create": (I, [I, ctypes.POINTER(I)]),
    "smi_init_local": (I, [I, I, I, ctypes.POINTER(SMI_Comm)]),
    "smi_finalize": (I, [SMI_Comm]),
    "smi_comm_dup": (I, [SMI_Comm, ctypes.POINTER(SMI_Comm)]),
    "smi_device_count": (I, [ctypes.POINTER(I)]),
    "smi_stream_synchronize": (I, [P]),
    "smi_stencil_step": (I, [P, P, I, I, ctypes.POINTER(I), ctypes.POINTER(P), P, P, P]),
    "smi_stencil_run": (I, [SMI_Comm, P, P, I, I, I, I, I, P, ctypes.POINTER(I)]),
    "smi_stencil_set_tuning": (I, [I, I, I, I]),
    "smi_stencil_get_tuning": (I, [ctypes.POINTER(I)] * 4),
    "smi_stencil_set_fusion": (I, [I, I, I]),
    "smi_stencil_get_fusion": (I, [ctypes.POINTER(I)] * 3),
    "smi_stencil_set_bands": (I, [I, I]),
    "smi_stencil_get_bands": (I, [ctypes.POINTER(I)] * 2),
    "smi_stencil_set_band_kernel": (I, [I]),
    "smi_stencil_get_band_kernel": (I, [ctypes.POINTER(I)]),
    "smi_stencil_set_join": (I, [I]),
    "smi_stencil_get_join": (I, [ctypes.POINTER(I)]),
    "smi_stencil_set_deep": (I, [I, I, I]),
    "smi_stencil_deep_geometry": (I, [I, I, I, I] + [ctypes.POINTER(I)] * 5),
    "smi_stencil_get_deep": (I, [ctypes.POINTER(I)] * 3),
    "smi_reduce": (I, [SMI_Comm, P, P, SZ, I, I, I, I, P]),
    "smi_reduce_fold": (I, [P, P, I, SZ, SZ, I, I, P]),
    "smi_bcast": (I, [SMI_Comm, P, SZ, I, I, I, P]),
    "smi_set_pipeline_bytes": (I, [SZ]),
    "smi_get_pipeline_bytes": (I, [ctypes.POINTER(SZ)]),
    "smi_type_size": (SZ, [I]),
    "smi_scatter": (I, [SMI_Comm, P, P, SZ, I, I, I, P]),
    "smi_gather": (I, [SMI_Comm, P, P, SZ, I, I, I, P]),
    "smi_send": (I, [SMI_Comm, P, SZ, I, I, I, P]),
    "smi_recv": (I, [SMI_Comm, P, SZ, I, I, I, P]),
    "smi_gemv_rows": (I, [P, P, P, P, I, I, I, F, F, P]),
    "smi_gesummv": (I, [SMI_Comm, P, P, P, P, I, I, F, F, I, P]),
    "smi_kmeans_assign": (I, [P, I, I, P, I, I, P, P]),
    "smi_kmeans_accumulate": (I, [P, I, I, P, I, P, P, P]),
    "smi_kmeans": (I, [SMI_Comm, P, I, I, I, I, P, I, P]),
    "smi_prof_enable": (I, [I]),
    "smi_prof_reset": (I, []),
    "smi_prof_read": (I, [I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_long)]),
    "smi_prof_read_tag": (I, [I, I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_long),
                              ctypes.POINTER(ctypes.c_double)]),
    "smi_prof_list": (I, [ctypes.POINTER(I), ctypes.POINTER(I), I, ctypes.POINTER(I)]),
    "smi_stencil_plan": (I, [I, I, I, I, I, I, P, I, ctypes.POINTER(I), ctypes.POINTER(I), ctypes.POINTER(I)]),
}


def variant() -> str:
    """SMI_LIB_VARIANT=debug selects the bounds-checked diagnostic build."""
    return os.environ.get("SMI_LIB_VARIANT", "")


def lib_path() -> str:
    return _build.lib_path(variant())


def recorded_srchash(path: str | None = None) -> str | None:
    """The source hash recorded beside the library when it was linked
    (smi_amd.build writes <lib>.srchash), or None."""
    try:
        with open((path or lib_path()) + ".srchash") as f:
            return f.read().strip() or None
    except OSError:
        return None


def verify_fresh(path: str | None = None) -> str:
    """Raise SMIError unless the library at `path` was built from exactly the
    sources, headers and flags of this tree (content hash, not mtimes);
    returns the hash."""
    path = path or lib_path()
    want = _build._src_hash(variant())
    got = recorded_srchash(path)
    if got != want:
        raise SMIError(f"{path} was not built from these sources (recorded source hash "
                       f"{(got or 'missing')[:16]}, tree {want[:16]}): rebuild with python smi_amd/build.py "
                       f"on the build host")
    return want


def load(build_if_missing: bool = True) -> ctypes.CDLL:
    """Load libsmi_amd.so, refusing a library that was not built from this
    tree's sources.  A missing or stale library is (re)built only where it is
    built -- a host without a GPU -- and only if build_if_missing; on a GPU
    host (the library travels there prebuilt) a stale library raises."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not os.path.exists(path) or recorded_srchash(path) != _build._src_hash(variant()):
        if build_if_missing and torch.cuda.device_count() == 0:  # counts devices without initialising HIP
            _build.build(variant=variant())
        elif not os.path.exists(path):
            raise SMIError(f"{path} missing: run python smi_amd/build.py on the build host")
    verify_fresh(path)
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in list(SIGNATURES.items()):
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str = "") -> None:
    if rc != SMI_SUCCESS:
        msg = load().smi_last_error()
        msg = msg.decode(errors="replace") if msg else ""
        raise SMIError(f"{what} failed with code {rc}: {msg}")


_fns: dict = {}


def call(name: str, *args) -> None:
    # (the bound functions are cached: a short timed region pays every
    # microsecond of host enqueue before its kernel starts)
    fn = _fns.get(name)
    if fn is None:
        fn = _fns[name] = getattr(load(), name)
    rc = fn(*args)
    if rc != SMI_SUCCESS:
        check(rc, name)


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_handle(stream=None, device: int | None = None) -> int:
    """hipStream_t of a torch stream (default: torch's current stream on
    `device`, or on the current device)."""
    if stream is None:
        if _raw_stream is not None:  # no Stream object built (~1.5 us less)
            return _raw_stream(torch.cuda.current_device() if device is None or device < 0 else device)
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)
