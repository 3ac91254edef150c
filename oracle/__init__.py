"""CPU oracle for the SMI hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package, and only as the checker or as
the timed CPU baseline.  The product (``smi_amd``) never imports it and fails
loudly when its HIP library is missing.

The arithmetic lives in ``smi_oracle.c`` (plain C, built by ``Makefile`` with
``-ffp-contract=off``); this module is a thin numpy/ctypes wrapper plus a few
pure-Python restatements used to pin the C code on small cases:

* :func:`stencil_exact` -- exact rational Jacobi (``fractions.Fraction``) used
  to pin the C stencil bit-for-bit on the steps where every value is a short
  dyadic rational (any summation order gives the same bits there).
* :func:`reduce_fold_py` -- a loop restatement of the root-side reduce fold of
  ``codegen/templates/reduce.cl:42-148`` used to cross-check the C fold.
* :func:`kmeans_reference_data` -- the kmeans_smi host's input generator
  (``kmeans_data.cpp``, same libstdc++ engine and distributions).

Parity status per path is recorded in DESIGN.md ("Oracle").
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from fractions import Fraction

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libsmi_oracle.so")
_lib = None

# include/smi/data_types.h:10-16
SMI_INT, SMI_FLOAT, SMI_DOUBLE, SMI_CHAR, SMI_SHORT = 1, 2, 3, 4, 5
# include/smi/reduce.h:18-22
SMI_ADD, SMI_MAX, SMI_MIN = 0, 1, 2

NP_DTYPE = {
    SMI_INT: np.int32,
    SMI_FLOAT: np.float32,
    SMI_DOUBLE: np.float64,
    SMI_CHAR: np.int8,
    SMI_SHORT: np.int16,
}

# codegen/ops.py:110-116 -- SHIFT_REG per data type
SHIFT_REG = {SMI_DOUBLE: 4, SMI_FLOAT: 4, SMI_INT: 1, SMI_SHORT: 1, SMI_CHAR: 1}


_SOURCES = ("smi_oracle.c", "kmeans_data.cpp", "Makefile")


def build(force: bool = False) -> str:
    """Compile smi_oracle.c + kmeans_data.cpp with the committed Makefile."""
    if force or not os.path.exists(_LIB_PATH) or any(
        os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, f)) for f in _SOURCES
    ):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        I = ctypes.c_int
        _lib.oracle_stencil.argtypes = [P, P, I, I, I, I, I]
        _lib.oracle_stencil_decomposed.argtypes = [P, P, I, I, I, I, I, I]
        _lib.oracle_stencil_steps.argtypes = [P, P, I, I, I, I]
        _lib.oracle_reduce.argtypes = [P, P, I, ctypes.c_long, I, I, P, I]
        _lib.oracle_bcast.argtypes = [P, I, I, ctypes.c_long, I]
        _lib.oracle_gesummv.argtypes = [P, P, P, P, I, I, ctypes.c_float, ctypes.c_float, I]
        L = ctypes.c_long
        _lib.oracle_kmeans_assign.argtypes = [P, L, I, P, I, I, P]
        _lib.oracle_kmeans_accumulate.argtypes = [P, L, I, P, I, P, P]
        _lib.oracle_kmeans.argtypes = [P, L, I, I, I, I, P, I]
        _lib.oracle_kmeans_reference_data.argtypes = [I, I, I, P, P, P]
        _lib.oracle_minstd_rand0_10000.argtypes = []
        _lib.oracle_minstd_rand0_10000.restype = ctypes.c_ulong
        for f in ("oracle_stencil", "oracle_stencil_decomposed", "oracle_stencil_steps", "oracle_reduce", "oracle_bcast",
                  "oracle_gesummv", "oracle_max_threads", "oracle_kmeans_assign",
                  "oracle_kmeans_accumulate", "oracle_kmeans", "oracle_kmeans_reference_data"):
            getattr(_lib, f).restype = ctypes.c_int
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


# ---------------------------------------------------------------- stencil --
def init_edges(X: int, Y: int) -> np.ndarray:
    """Reference test pattern: 0 interior, 1 on all four edges
    (examples/host/stencil_smi.cpp:175-187)."""
    g = np.zeros((X, Y), dtype=np.float32)
    g[0, :] = 1
    g[X - 1, :] = 1
    g[:, 0] = 1
    g[:, Y - 1] = 1
    return g


def init_uniform(X: int, Y: int, seed: int = 42) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return rng.random((X, Y), dtype=np.float32)


STENCIL_ORDERS = {"device": 0, "host": 1, "tree": 2}


def stencil(grid: np.ndarray, T: int, order: str = "device", threads: int = 0) -> np.ndarray:
    """T Jacobi steps.  order='device' is the stencil_smi.cl:153-156 order
    (S+W+E+N); order='host' is the reference host Reference() order
    (N+S+W+E, stencil_smi.cpp:33-46); order='tree' is the balanced tree
    (S+W)+(E+N) an -fp-relaxed build may reassociate the device order into
    (CMakeLists.txt:70,188) -- test-only, to quantify that divergence."""
    g = np.ascontiguousarray(grid, dtype=np.float32)
    out = np.empty_like(g)
    X, Y = g.shape
    rc = lib().oracle_stencil(_ptr(g), _ptr(out), X, Y, T, STENCIL_ORDERS[order], threads)
    if rc:
        raise ValueError(f"oracle_stencil rc={rc}")
    return out


def stencil_steps(a: np.ndarray, b: np.ndarray, T: int, threads: int = 0) -> np.ndarray:
    """T device-order steps ping-ponging between two preallocated C-contiguous
    float32 buffers (a holds the input; both are overwritten).  Returns the
    buffer holding the result.  No allocation inside: bench.py times this."""
    assert a.flags.c_contiguous and b.flags.c_contiguous and a.shape == b.shape
    assert a.dtype == np.float32 and b.dtype == np.float32
    X, Y = a.shape
    rc = lib().oracle_stencil_steps(_ptr(a), _ptr(b), X, Y, T, threads)
    if rc < 0:
        raise ValueError(f"oracle_stencil_steps rc={rc}")
    return b if rc else a


def stencil_decomposed(grid: np.ndarray, T: int, PX: int, PY: int, threads: int = 1) -> np.ndarray:
    """Rank-decomposed emulation of the stencil_smi program (Read/Stencil/
    Write per rank with halo queues, stencil_smi.cl:20-386); threads > 1 runs
    the ranks as threads (threads-as-ranks, same bits)."""
    g = np.ascontiguousarray(grid, dtype=np.float32)
    out = np.empty_like(g)
    X, Y = g.shape
    rc = lib().oracle_stencil_decomposed(_ptr(g), _ptr(out), X, Y, PX, PY, T, threads)
    if rc:
        raise ValueError(f"oracle_stencil_decomposed rc={rc}")
    return out


def stencil_exact(grid, T: int):
    """Exact rational Jacobi (no rounding at all) -- pins the fp32 oracle
    while every intermediate is exactly representable."""
    X = len(grid)
    Y = len(grid[0])
    cur = [[Fraction(float(v)) for v in row] for row in grid]
    q = Fraction(1, 4)
    for _ in range(T):
        nxt = [row[:] for row in cur]
        for i in range(1, X - 1):
            for j in range(1, Y - 1):
                nxt[i][j] = q * (cur[i + 1][j] + cur[i][j - 1] + cur[i][j + 1] + cur[i - 1][j])
        cur = nxt
    return cur


def reference_check(result: np.ndarray, reference: np.ndarray) -> bool:
    """The reference host's acceptance test: |ref - res| < 1e-4 * mean(ref)
    for every cell (examples/host/stencil_smi.cpp:391-405; the mean is
    accumulated in double and stored as Data_t=float)."""
    average = np.float32(np.sum(reference, dtype=np.float64) / reference.size)
    diff = np.abs(reference.astype(np.float32) - result.astype(np.float32))
    return bool(np.all(diff < 1e-4 * float(average)))


# ----------------------------------------------------------------- reduce --
def reduce(contribs: np.ndarray, dtype: int, op: int, arrival=None, threads: int = 1) -> np.ndarray:
    """Root-side reduce fold (codegen/templates/reduce.cl:42-148).
    contribs: (nranks, count) array, row r = rank r's send buffer; threads > 1
    folds `threads` owner chunks side by side (same bits)."""
    npdt = NP_DTYPE[dtype]
    c = np.ascontiguousarray(contribs, dtype=npdt)
    n, count = c.shape
    out = np.empty(count, dtype=npdt)
    arr = None
    arr_ptr = None
    if arrival is not None:
        arr = np.ascontiguousarray(arrival, dtype=np.int32)
        arr_ptr = _ptr(arr)
    rc = lib().oracle_reduce(_ptr(c), _ptr(out), n, count, dtype, op, arr_ptr, threads)
    if rc:
        raise ValueError(f"oracle_reduce rc={rc}")
    return out


def bcast(bufs: np.ndarray, root: int, threads: int = 1) -> np.ndarray:
    """Threads-as-ranks broadcast (codegen/templates/bcast.cl:3-111): row r of
    `bufs` (nranks, n) is rank r's buffer; every row becomes a copy of row
    `root`, packet by packet.  In place; returns bufs."""
    assert bufs.flags.c_contiguous
    n = bufs.shape[0]
    rc = lib().oracle_bcast(_ptr(bufs), n, root, bufs.nbytes // n, threads)
    if rc:
        raise ValueError(f"oracle_bcast rc={rc}")
    return bufs


def _init_value(dtype: int, op: int):
    """codegen/ops.py:124-141 SHIFT_REG_INIT."""
    npdt = NP_DTYPE[dtype]
    if op == SMI_ADD:
        return npdt(0)
    if dtype in (SMI_FLOAT, SMI_DOUBLE):
        fi = np.finfo(npdt)
        return npdt(fi.tiny) if op == SMI_MAX else npdt(fi.max)  # FLT_MIN / FLT_MAX
    ii = np.iinfo(npdt)
    return npdt(ii.min) if op == SMI_MAX else npdt(ii.max)


def reduce_fold_py(values, dtype: int, op: int):
    """Pure-Python loop restatement of one element's fold, in the given
    arrival order (reduce.cl:65-69, 100-105, 120-125)."""
    npdt = NP_DTYPE[dtype]
    S = SHIFT_REG[dtype]
    init = _init_value(dtype, op)

    def apply(a, b):
        if op == SMI_ADD:
            return _wrap_add(a, b, npdt)
        if op == SMI_MAX:
            return a if a > b else b
        return a if a < b else b

    q = [init] * (S + 1)
    for d in values:
        q[S] = apply(npdt(d), q[0])
        for j in range(S):
            q[j] = q[j + 1]
    res = init
    for j in range(S):
        res = apply(res, q[j])
    return npdt(res)


def _wrap_add(a, b, npdt):
    if np.issubdtype(npdt, np.floating):
        return npdt(npdt(a) + npdt(b))
    bits = 8 * np.dtype(npdt).itemsize
    s = (int(a) + int(b)) & ((1 << bits) - 1)
    if s >= 1 << (bits - 1):
        s -= 1 << bits
    return npdt(s)


# ---------------------------------------------------------------- gesummv --
def gesummv(A: np.ndarray, B: np.ndarray, x: np.ndarray, alpha: float, beta: float,
            threads: int = 0) -> np.ndarray:
    """y = alpha*A*x + beta*B*x with the row-streamed fold of
    examples/kernels/gesummv_rank0.cl:53-203."""
    A = np.ascontiguousarray(A, dtype=np.float32)
    B = np.ascontiguousarray(B, dtype=np.float32)
    x = np.ascontiguousarray(x, dtype=np.float32)
    N, M = A.shape
    y = np.empty(N, dtype=np.float32)
    rc = lib().oracle_gesummv(_ptr(A), _ptr(B), _ptr(x), _ptr(y), N, M,
                              ctypes.c_float(alpha), ctypes.c_float(beta), threads)
    if rc:
        raise ValueError(f"oracle_gesummv rc={rc}")
    return y


def gesummv_reference_check(result: np.ndarray, A, B, x, alpha, beta) -> bool:
    """The reference host's acceptance test (gesummv_smi.cpp:40-46,299-313):
    rel. err < 1e-4 against sgemv(beta,B) then sgemv(alpha,A,+y); here the
    BLAS is replaced by a float64 evaluation of the same expression."""
    ref = (beta * (B.astype(np.float64) @ x.astype(np.float64))
           + alpha * (A.astype(np.float64) @ x.astype(np.float64))).astype(np.float32)
    res = result.astype(np.float32)
    ok = np.isfinite(res) & np.isfinite(ref)
    both_zero = (res == 0) & (ref == 0)
    with np.errstate(divide="ignore", invalid="ignore"):
        rel = np.abs(res - ref) / np.abs(ref)
    return bool(np.all(ok & (both_zero | (rel < 1e-4))))


def max_threads() -> int:
    return int(lib().oracle_max_threads())


# ----------------------------------------------------------------- kmeans --
def kmeans_assign(points: np.ndarray, centroids: np.ndarray, width: int = 16) -> np.ndarray:
    """ComputeDistance (examples/kernels/kmeans_smi.cl:54-85), W = width."""
    p = np.ascontiguousarray(points, dtype=np.float32)
    c = np.ascontiguousarray(centroids, dtype=np.float32)
    idx = np.empty(p.shape[0], dtype=np.int32)
    rc = lib().oracle_kmeans_assign(_ptr(p), p.shape[0], p.shape[1], _ptr(c), c.shape[0], width, _ptr(idx))
    if rc:
        raise ValueError(f"oracle_kmeans_assign rc={rc}")
    return idx


def kmeans_accumulate(points: np.ndarray, assignment: np.ndarray, clusters: int):
    """ComputeMeans accumulation (kmeans_smi.cl:98-127): (sums, counts)."""
    p = np.ascontiguousarray(points, dtype=np.float32)
    a = np.ascontiguousarray(assignment, dtype=np.int32)
    sums = np.empty((clusters, p.shape[1]), dtype=np.float32)
    counts = np.empty(clusters, dtype=np.int32)
    rc = lib().oracle_kmeans_accumulate(_ptr(p), p.shape[0], p.shape[1], _ptr(a), clusters, _ptr(sums),
                                        _ptr(counts))
    if rc:
        raise ValueError(f"oracle_kmeans_accumulate rc={rc}")
    return sums, counts


def kmeans(points: np.ndarray, centroids: np.ndarray, iterations: int, ranks: int = 1,
           width: int = 16) -> np.ndarray:
    """The kmeans_smi program over `ranks` ranks; returns the final centroids."""
    p = np.ascontiguousarray(points, dtype=np.float32)
    c = np.array(centroids, dtype=np.float32, order="C", copy=True)
    rc = lib().oracle_kmeans(_ptr(p), p.shape[0], ranks, p.shape[1], c.shape[0], width, _ptr(c), iterations)
    if rc:
        raise ValueError(f"oracle_kmeans rc={rc}")
    return c


def kmeans_reference_data(num_points: int, clusters: int = 8, dims: int = 64):
    """(means, points, initial centroids) exactly as the reference host
    generates them on rank 0 (examples/host/kmeans_smi.cpp:96-147)."""
    means = np.empty((clusters, dims), dtype=np.float32)
    pts = np.empty((num_points, dims), dtype=np.float32)
    cen = np.empty((clusters, dims), dtype=np.float32)
    rc = lib().oracle_kmeans_reference_data(num_points, clusters, dims, _ptr(means), _ptr(pts), _ptr(cen))
    if rc:
        raise ValueError("the reference host would copy a centroid from past the end of its input "
                         "(uniform_int_distribution(0, num_points) is inclusive, kmeans_smi.cpp:141)")
    return means, pts, cen


def minstd_rand0_10000() -> int:
    return int(lib().oracle_minstd_rand0_10000())
