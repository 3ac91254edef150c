"""BASELINE configs 3-5 at their full size on one GPU (in-process rank groups).

* Config 3 (examples/CMakeLists.txt:2-7, stencil_smi 16384^2 as 2x2 and 2x4):
  4 ranks x 8192^2 and 8 ranks x 8192x4096 tiles, T = 43 steps under the
  default K = 20 (three balanced passes of 15 + 14 + 14 steps: the
  rotating-ring interior, depth-K bands and halo exchanges), bit-exact vs
  the oracle.
* Config 4 (microbenchmarks reduce/bcast, 64 MiB and 256 MiB, 8 ranks): the
  rank+1 known answer of test/reduce/reduce.cl:7-61 on every element, and
  random contributions checked against the oracle's canonical rank-order fold
  on a strided sample of columns; bcast bitwise on every rank.
* Config 5 (gesummv 32768^2 row-sharded 8 ways, examples/host/
  gesummv_smi.cpp:22-36,299-313): the reference pattern A = B = i, x = 1 under
  the reference's own check on every row and bit-exact vs the oracle on a row
  sample; seeded random A, B, x bit-exact vs the oracle on a row sample.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


# ------------------------------------------------------------------ config 3
@pytest.mark.parametrize("pxpy", [(2, 2), (2, 4)])
def test_config3_stencil_16384(gpu, oracle_mod, pxpy):
    from smi_amd import LocalGroup, stencil
    PX, PY = pxpy
    # the default plan (K = 20): T = 43 as three balanced passes of the
    # rotating-ring interior with depth-15 / depth-14 halo exchanges
    assert stencil.get_fusion()["steps_per_pass"] == 20
    N, T = 16384, 2 * 20 + 3
    g = oracle_mod.init_uniform(N, N, seed=33 + PY)
    tiles = stencil.split_memory(g, PX, PY)
    assert stencil.plan(N // PX, N // PY, PX, PY, 0, T)["phases"] == [(15, 1), (14, 2)]

    def rank_fn(comm):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            t = torch.from_numpy(tiles[comm.rank]).cuda()
            res = stencil.run(comm, t, T, PX, PY)
            s.synchronize()
            return res.cpu().numpy()

    out = LocalGroup(PX * PY).run(rank_fn)
    del tiles
    got = stencil.combine_memory(out, PX, PY)
    del out
    want = oracle_mod.stencil(g, T)
    assert np.array_equal(bits(got), bits(want))


# ------------------------------------------------------------------ config 4
def _rand_contrib(rank, count, dtype):
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1000 + rank)
    if dtype == torch.float32:
        return torch.rand(count, generator=gen, device="cuda") * 2 - 1
    return torch.randint(-(1 << 31), (1 << 31) - 1, (count,), generator=gen, device="cuda", dtype=torch.int32)


@pytest.mark.parametrize("mib", [64, 256])
@pytest.mark.parametrize("dtype", [torch.int32, torch.float32])
def test_config4_reduce_at_size(gpu, oracle_mod, mib, dtype):
    from smi_amd import LocalGroup, collectives
    n, root = 8, 3
    count = mib * (1 << 20) // 4
    t = 1 if dtype == torch.int32 else 2
    cols = np.arange(0, count, 4099)
    cols = np.concatenate([cols, [count - 1]])

    def fn(comm):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            # rank+1 known answer: sum = n(n+1)/2 on every element
            snd = torch.full((count,), comm.rank + 1, dtype=dtype, device="cuda")
            rcv = torch.empty_like(snd) if comm.rank == root else None
            collectives.reduce(comm, snd, rcv, "add", root)
            s.synchronize()
            kat = None if rcv is None else bool(torch.all(rcv == n * (n + 1) // 2).item())
            # random contributions: canonical fold on a strided sample
            snd = _rand_contrib(comm.rank, count, dtype)
            collectives.reduce(comm, snd, rcv, "add", root)
            s.synchronize()
            sample = snd[torch.from_numpy(cols).cuda()].cpu().numpy()
            got = None if rcv is None else rcv[torch.from_numpy(cols).cuda()].cpu().numpy()
            return kat, sample, got

    res = LocalGroup(n).run(fn)
    assert res[root][0] is True
    contribs = np.stack([r[1] for r in res])
    want = oracle_mod.reduce(contribs, t, 0)
    assert np.array_equal(res[root][2].view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("mib", [64, 256])
def test_config4_bcast_at_size(gpu, mib):
    from smi_amd import LocalGroup, collectives
    n, root = 8, 5
    count = mib * (1 << 20) // 4

    def fn(comm):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            want = _rand_contrib(root, count, torch.float32)
            buf = want.clone() if comm.rank == root else torch.zeros(count, device="cuda")
            collectives.bcast(comm, buf, root)
            s.synchronize()
            return bool(torch.equal(buf.view(torch.int32), want.view(torch.int32)))

    assert all(LocalGroup(n).run(fn))


# ------------------------------------------------------------------ config 5
def _gesummv_8way(A_fn, B_fn, x, n, alpha, beta, rows):
    from smi_amd import LocalGroup, gesummv
    nranks, root = 8, 0

    def fn(comm):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            r0, r1 = gesummv.row_range(n, comm.size, comm.rank)
            A = A_fn(r0, r1)
            B = B_fn(r0, r1)
            y = gesummv.gesummv(comm, A, B, x.cuda(), n, alpha, beta, root=root)
            s.synchronize()
            # the sampled rows this rank holds (for the oracle on the host)
            mine = [r for r in rows if r0 <= r < r1]
            idx = torch.tensor([r - r0 for r in mine], dtype=torch.long, device="cuda")
            samp = (mine, A[idx].cpu().numpy(), B[idx].cpu().numpy()) if mine else (mine, None, None)
            return (None if y is None else y.cpu().numpy()), samp

    res = LocalGroup(nranks).run(fn)
    y = res[root][0]
    rA, rB = {}, {}
    for _, (mine, a, b) in res:
        for j, r in enumerate(mine):
            rA[r], rB[r] = a[j], b[j]
    return y, np.stack([rA[r] for r in rows]), np.stack([rB[r] for r in rows])


def test_config5_gesummv_reference_pattern(gpu, oracle_mod):
    n = m = 32768
    alpha, beta = 1.5, 0.5  # any alpha/beta; the reference host takes them from argv
    rows = sorted({0, 1, 2, 3, 255, 4095, 4096, 8191, 16384, 20000, 32766, 32767} | set(range(7, n, 2999)))

    def mat(r0, r1):  # A[i][j] = i (gesummv_smi.cpp:21-27)
        return torch.arange(r0, r1, dtype=torch.float32, device="cuda")[:, None].expand(r1 - r0, m).contiguous()

    x = torch.ones(m, dtype=torch.float32)  # gesummv_smi.cpp:30-34
    y, As, Bs = _gesummv_8way(mat, mat, x, n, alpha, beta, rows)
    # the reference host's own acceptance check on every row (rel. err < 1e-4
    # vs sgemv; the exact value is (alpha + beta) * i * m)
    exact = (alpha + beta) * np.arange(n, dtype=np.float64) * m
    ok = (y == exact) | (np.abs(y - exact) / np.maximum(np.abs(exact), 1e-300) < 1e-4)
    assert ok.all()
    assert np.array_equal(bits(y[rows]), bits(oracle_mod.gesummv(As, Bs, x.numpy(), alpha, beta)))


def test_config5_gesummv_random(gpu, oracle_mod):
    n = m = 32768
    alpha, beta = 1.25, -0.75
    rows = sorted({0, 4095, 4096, 32767} | set(range(11, n, 1777)))

    def rnd(seed):
        def f(r0, r1):
            gen = torch.Generator(device="cuda")
            gen.manual_seed(seed * 100003 + r0)
            return torch.rand((r1 - r0, m), generator=gen, device="cuda") * 2 - 1
        return f

    gx = torch.Generator()
    gx.manual_seed(9)
    x = torch.rand(m, generator=gx) * 2 - 1
    y, As, Bs = _gesummv_8way(rnd(1), rnd(2), x, n, alpha, beta, rows)
    assert np.array_equal(bits(y[rows]), bits(oracle_mod.gesummv(As, Bs, x.numpy(), alpha, beta)))
