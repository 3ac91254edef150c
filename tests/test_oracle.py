"""Pin the CPU oracle (CPU only, no GPU).

* reduce: the reference's own known-answer tests (test/reduce/reduce.cl:7-172,
  microbenchmarks/kernels/reduce.cl:13-24) over its parameter grid, the
  SURVEY's closed forms for the canonical fold, and a pure-Python loop
  restatement of reduce.cl:65-125.
* stencil: exact rational arithmetic while every value is a short dyadic
  rational (any summation order gives the same bits), the reference host
  acceptance check at 32 steps (stencil_smi.cpp:391-405), and equality of the
  full-grid and the rank-decomposed emulator restatements.
* gesummv: the reference host check on the reference test pattern.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle as o

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


# ---------------------------------------------------------------- reduce --
@pytest.mark.parametrize("n", [2, 4, 8])
def test_reduce_reference_kats(n):
    for ml in (1, 128, 300):
        i = np.arange(ml)
        # float add: everyone sends i -> n*i   (test/reduce/reduce.cl:7-23)
        c = np.stack([i.astype(np.float32)] * n)
        assert np.array_equal(o.reduce(c, o.SMI_FLOAT, o.SMI_ADD), (n * i).astype(np.float32))
        # int max / int add of rank+1 -> n, n(n+1)/2     (:25-61)
        c = np.stack([np.full(ml, r + 1, np.int32) for r in range(n)])
        assert (o.reduce(c, o.SMI_INT, o.SMI_MAX) == n).all()
        assert (o.reduce(c, o.SMI_INT, o.SMI_ADD) == n * (n + 1) // 2).all()
        # float min of i + 0.1*rank -> i                 (:63-79)
        c = np.stack([(i + 0.1 * r).astype(np.float32) for r in range(n)])
        assert np.array_equal(o.reduce(c, o.SMI_FLOAT, o.SMI_MIN), i.astype(np.float32))
        # double add -> n*i                               (:119-135)
        c = np.stack([i.astype(np.float64)] * n)
        assert np.array_equal(o.reduce(c, o.SMI_DOUBLE, o.SMI_ADD), (n * i).astype(np.float64))
        # char max -> n, short min -> 1                   (:137-172)
        c = np.stack([np.full(ml, r + 1, np.int8) for r in range(n)])
        assert (o.reduce(c, o.SMI_CHAR, o.SMI_MAX) == n).all()
        c = np.stack([np.full(ml, r + 1, np.int16) for r in range(n)])
        assert (o.reduce(c, o.SMI_SHORT, o.SMI_MIN) == 1).all()
        # microbenchmark: fp32 rank+1 -> n(n+1)/2 (microbenchmarks/kernels/reduce.cl:13-24)
        c = np.stack([np.full(ml, r + 1, np.float32) for r in range(n)])
        assert (o.reduce(c, o.SMI_FLOAT, o.SMI_ADD) == n * (n + 1) / 2).all()


def test_reduce_closed_forms():
    """with arrival = rank order the S=4 fold is
    n=2: d0+d1; n=4: ((d0+d1)+d2)+d3; n=8: (((d0+d4)+(d1+d5))+(d2+d6))+(d3+d7)."""
    rng = np.random.default_rng(0)
    for n in (2, 4, 8):
        d = (rng.random((n, 4096)) * 2 - 1).astype(np.float32) * np.float32(1e3)
        got = o.reduce(d, o.SMI_FLOAT, o.SMI_ADD)
        if n == 2:
            want = d[0] + d[1]
        elif n == 4:
            want = ((d[0] + d[1]) + d[2]) + d[3]
        else:
            want = (((d[0] + d[4]) + (d[1] + d[5])) + (d[2] + d[6])) + (d[3] + d[7])
        want = want + np.float32(0)  # the +0.0 accumulator turns -0 into +0
        assert np.array_equal(got.view(np.uint32), want.astype(np.float32).view(np.uint32))


@pytest.mark.parametrize("t", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("op", [0, 1, 2])
def test_reduce_c_matches_python_loop(t, op):
    rng = np.random.default_rng(t * 3 + op)
    npdt = o.NP_DTYPE[t]
    for n in (1, 2, 3, 5, 8):
        if t in (2, 3):
            c = ((rng.random((n, 40)) * 2 - 1) * 100).astype(npdt)
        else:
            info = np.iinfo(npdt)
            c = rng.integers(info.min, info.max, size=(n, 40), endpoint=True, dtype=npdt)
        order = rng.permutation(n)
        got = o.reduce(c, t, op, arrival=order)
        want = np.array([o.reduce_fold_py(c[order, j], t, op) for j in range(c.shape[1])], dtype=npdt)
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


def test_reduce_float_max_init_quirk():
    """codegen/ops.py:133 initialises float MAX with FLT_MIN (smallest
    positive normal), so an all-negative max returns FLT_MIN."""
    c = np.full((4, 3), -5.0, np.float32)
    assert np.all(o.reduce(c, o.SMI_FLOAT, o.SMI_MAX) == np.finfo(np.float32).tiny)


def test_reduce_int_wraps():
    c = np.array([[2 ** 31 - 1], [5]], dtype=np.int32)
    assert o.reduce(c, o.SMI_INT, o.SMI_ADD)[0] == np.int32(-2 ** 31 + 4)


# --------------------------------------------------------------- stencil --
def test_stencil_exact_dyadic_steps():
    g = o.init_edges(24, 20)
    for T in (1, 4, 10):
        ex = o.stencil_exact(g.tolist(), T)
        want = np.array([[float(v) for v in row] for row in ex], dtype=np.float32)
        assert np.array_equal(o.stencil(g, T), want)
        assert np.array_equal(o.stencil(g, T, order="host"), want)


def test_stencil_reference_check_config1():
    g = o.init_edges(256, 256)
    dev = o.stencil(g, 32)
    host = o.stencil(g, 32, order="host")
    assert o.reference_check(dev, host)


@pytest.mark.parametrize("pxpy", [(1, 1), (2, 2), (2, 4), (4, 2), (1, 8)])
def test_stencil_decomposed_equals_full(pxpy):
    PX, PY = pxpy
    g = o.init_uniform(64, 128, seed=11)
    full = o.stencil(g, 17)
    dec = o.stencil_decomposed(g, 17, PX, PY)
    assert np.array_equal(full.view(np.uint32), dec.view(np.uint32))
    # threads-as-ranks (the CPU baseline's emulator legs): same bits
    thr = o.stencil_decomposed(g, 17, PX, PY, threads=PX * PY)
    assert np.array_equal(full.view(np.uint32), thr.view(np.uint32))


@pytest.mark.parametrize("dtype,op", [(2, 0), (1, 0), (3, 1), (5, 2)])
def test_reduce_threads_as_ranks_same_bits(dtype, op):
    rng = np.random.default_rng(dtype * 3 + op)
    c = (rng.random((8, 10007)) * 200 - 100).astype(o.NP_DTYPE[dtype])
    assert np.array_equal(o.reduce(c, dtype, op), o.reduce(c, dtype, op, threads=8))


def test_bcast_threads_as_ranks_copies_root():
    b = np.random.default_rng(9).random((8, 1001), dtype=np.float32)   # 4004 B: a partial last packet
    want = b[5].copy()
    o.bcast(b, 5, threads=8)
    assert all(np.array_equal(b[r].view(np.uint32), want.view(np.uint32)) for r in range(8))


def test_stencil_order_matters():
    """The device order S+W+E+N differs from the host order N+S+W+E on random
    data -- which is why the GPU is held to the device order bit for bit."""
    g = o.init_uniform(64, 64, seed=5)
    a = o.stencil(g, 8)
    b = o.stencil(g, 8, order="host")
    assert not np.array_equal(a, b)
    assert o.reference_check(a, b)


def _ulp_gap(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """|a - b| in units in the last place (ordered-integer view of fp32)."""
    def ordered(x):
        i = x.view(np.int32).astype(np.int64)
        return np.where(i < 0, -(i & 0x7FFFFFFF), i)
    return np.abs(ordered(a) - ordered(b))


@pytest.mark.parametrize("case", ["config1_256x256_T32_edges", "config2_8192x8192_T20_uniform"])
def test_fp_relaxed_tree_order_divergence(case, capsys):
    """The reference builds every target, the emulator included, with
    -fp-relaxed (/root/reference/CMakeLists.txt:66-73, :188), which licenses
    reassociating stencil_smi.cl:153-156's ((S+W)+E)+N into a tree such as
    (S+W)+(E+N).  Which tree (if any) the emulator forms is unknowable here,
    so the GPU is held to the source order; this quantifies what the tree
    order would change: the fraction of cells that differ and the largest
    gap in ulp, at BASELINE config 1 (reference init) and at the driver's
    config 2 (8192^2, 20 steps, the bench's seeded input).  Both orders pass
    the reference host's own acceptance check against Reference()
    (stencil_smi.cpp:391-405)."""
    if case.startswith("config1"):
        g, T = o.init_edges(256, 256), 32
    else:
        g, T = o.init_uniform(8192, 8192, seed=42), 20
    src = o.stencil(g, T)
    tree = o.stencil(g, T, order="tree")
    host = o.stencil(g, T, order="host")
    gap = _ulp_gap(src, tree)
    frac = float(np.count_nonzero(gap)) / gap.size
    with capsys.disabled():
        print(f"\n[fp-relaxed] {case}: {frac:.4%} of cells differ between ((S+W)+E)+N and (S+W)+(E+N), "
              f"max {int(gap.max())} ulp, mean {float(gap.mean()):.3f} ulp")
    assert o.reference_check(src, host) and o.reference_check(tree, host)
    if case.startswith("config1"):
        # the first 10 steps are dyadic (any order is exact); by step 32 the
        # orders may part, but only by a few ulp
        assert int(gap.max()) <= 16
    else:
        assert frac > 0.0 and int(gap.max()) <= 64


def test_golden_fixtures_reproduce():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        gold = json.load(f)
    for case in gold["stencil"]:
        X, Y, T = case["X"], case["Y"], case["T"]
        g = o.init_edges(X, Y) if case["init"] == "edges" else o.init_uniform(X, Y, seed=case["seed"])
        if case.get("PX", 1) * case.get("PY", 1) > 1:
            out = o.stencil_decomposed(g, T, case["PX"], case["PY"])
        else:
            out = o.stencil(g, T)
        assert hashlib.sha256(out.tobytes()).hexdigest() == case["sha256"], case
    arr = np.load(os.path.join(GOLDEN, "stencil_uniform_64x96_T16.npy"))
    assert np.array_equal(o.stencil(o.init_uniform(64, 96, seed=42), 16), arr)
    for case in gold["kmeans"]:
        _, pts, cen = o.kmeans_reference_data(case["num_points"], case["clusters"], case["dims"])
        c = o.kmeans(pts, cen, case["iterations"], ranks=case["ranks"], width=case["width"])
        assert hashlib.sha256(c.tobytes()).hexdigest() == case["sha256"], case


# --------------------------------------------------------------- gesummv --
def test_gesummv_reference_pattern():
    n, m = 128, 256
    A = np.repeat(np.arange(n, dtype=np.float32)[:, None], m, axis=1)
    x = np.ones(m, np.float32)
    y = o.gesummv(A, A, x, 1.5, 0.5)
    assert o.gesummv_reference_check(y, A, A, x, 1.5, 0.5)
    assert np.array_equal(y, (2.0 * np.arange(n) * m).astype(np.float32))


def test_gesummv_fold_restatement():
    """Direct Python restatement of gesummv_rank0.cl:111-171 on one row."""
    rng = np.random.default_rng(1)
    m = 64 * 5
    a = rng.random(m, dtype=np.float32)
    b = rng.random(m, dtype=np.float32)
    x = rng.random(m, dtype=np.float32)

    def fold(row, alpha):
        f = np.float32
        y = f(0)
        chunks = m // 64
        for t in range((chunks + 1) // 2):
            acc_o = f(0)
            for jj in range(2):
                k = 2 * t + jj
                acc_i = f(0)
                if k < chunks:
                    for j in range(64):
                        acc_i = f(acc_i + f(row[64 * k + j] * x[64 * k + j]))
                acc_o = f(acc_o + f(f(alpha) * acc_i))
            y = f(y + acc_o)
        return y

    want = np.float32(fold(a, 1.5) + fold(b, 0.5))
    got = o.gesummv(a[None, :], b[None, :], x, 1.5, 0.5)[0]
    assert got.view(np.uint32) == want.view(np.uint32)


# ---------------------------------------------------------------- kmeans --
def test_kmeans_generator_engine_kat():
    """The reference host seeds std::default_random_engine (libstdc++:
    minstd_rand0); the C++ standard's check value pins the engine."""
    assert o.minstd_rand0_10000() == 1043618065


def test_kmeans_reference_data():
    """kmeans_smi.cpp:99-147: means in [-5, 5), point i ~ N(mean_{i%K}, 1),
    initial centroids copied from input points."""
    means, pts, cen = o.kmeans_reference_data(2048, 8, 64)
    assert means.min() >= -5 and means.max() < 5
    d = pts.reshape(256, 8, 64) - means[None]
    assert abs(float(d.mean())) < 0.02 and abs(float(d.std()) - 1) < 0.02
    rows = {r.tobytes() for r in pts}
    assert all(c.tobytes() in rows for c in cen)


def _assign_numpy(pts, cen, width):
    """Vectorised restatement of kmeans_smi.cl:54-85: the last lane of each
    W-wide vector, fp32 mul then add, strict < from +inf."""
    f = np.float32
    xs, cs = pts[:, width - 1::width], cen[:, width - 1::width]
    dist = np.zeros((len(pts), len(cen)), f)
    for j in range(xs.shape[1]):
        diff = (xs[:, None, j] - cs[None, :, j]).astype(f)
        dist = (dist + (diff * diff).astype(f)).astype(f)
    best = np.zeros(len(pts), np.int32)
    mind = np.full(len(pts), np.inf, f)
    for k in range(len(cen)):
        upd = dist[:, k] < mind
        best[upd] = k
        mind[upd] = dist[upd, k]
    return best


@pytest.mark.parametrize("width", [1, 4, 16])
def test_kmeans_assign_restatement(width):
    rng = np.random.default_rng(width)
    pts = rng.standard_normal((500, 64), dtype=np.float32)
    cen = rng.standard_normal((8, 64), dtype=np.float32)
    cen[3] = cen[1]                      # tie: the lower index wins
    pts[7] = np.nan                      # all-NaN distances: cluster 0
    got = o.kmeans_assign(pts, cen, width)
    assert np.array_equal(got, _assign_numpy(pts, cen, width))
    assert got[7] == 0 and not np.any(got == 3)


def test_kmeans_accumulate_restatement():
    """Sequential Python restatement of the per-cluster chains; the form that
    skips other clusters' points (the GPU's) gives the same bits as the
    literal `+= (index == k) ? x : 0` of kmeans_smi.cl:122."""
    rng = np.random.default_rng(4)
    n, dims, K = 300, 5, 4
    pts = (rng.standard_normal((n, dims)) * 100).astype(np.float32)
    pts[::17] *= -1
    pts[5, 2] = -0.0
    asg = rng.integers(-1, K + 1, n).astype(np.int32)   # -1 and K belong to no cluster
    f = np.float32
    want = np.zeros((K, dims), f)
    for p in range(n):
        if 0 <= asg[p] < K:
            want[asg[p]] = (want[asg[p]] + pts[p]).astype(f)
    sums, counts = o.kmeans_accumulate(pts, asg, K)
    assert np.array_equal(sums.view(np.uint32), want.view(np.uint32))
    assert np.array_equal(counts, np.array([(asg == k).sum() for k in range(K)]))


@pytest.mark.parametrize("ranks", [1, 4, 8])
def test_kmeans_program_composition(ranks):
    """oracle_kmeans = per-rank assign + accumulate, the reduce fold over the
    ranks, and IEEE division -- composed here from the pieces."""
    _, pts, cen = o.kmeans_reference_data(1024, 8, 64)
    c = cen.copy()
    per = len(pts) // ranks
    for _ in range(3):
        s, n = [], []
        for r in range(ranks):
            mine = pts[r * per:(r + 1) * per]
            a, b = o.kmeans_accumulate(mine, o.kmeans_assign(mine, c, 16), 8)
            s.append(a.ravel())
            n.append(b)
        rs = o.reduce(np.stack(s), o.SMI_FLOAT, o.SMI_ADD).reshape(8, 64)
        rc = o.reduce(np.stack(n), o.SMI_INT, o.SMI_ADD)
        with np.errstate(invalid="ignore", divide="ignore"):
            c = (rs / rc.astype(np.float32)[:, None]).astype(np.float32)
    want = o.kmeans(pts, cen, 3, ranks=ranks, width=16)
    assert np.array_equal(np.isnan(c), np.isnan(want))
    assert np.array_equal(c[~np.isnan(c)], want[~np.isnan(want)])
