"""kmeans_smi parity on the GPU (examples/kernels/kmeans_smi.cl,
examples/host/kmeans_smi.cpp), all through the C ABI.

Contract: bit-exact vs the oracle's restatement (oracle/smi_oracle.c) --
assignments and counts exactly; per-cluster sums bitwise (fp32 chains in
point order; the oracle restates the literal `+= (index == k) ? x : 0` of
kmeans_smi.cl:122); centroids bitwise after the canonical reduce fold and
IEEE division, NaN payloads aside (an empty cluster is 0/0 in both).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def same_bits(a, b):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return bool(np.array_equal(na, nb) and np.array_equal(a.view(np.uint32)[~na], b.view(np.uint32)[~nb]))


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("n,dims,clusters,width", [
    (1, 64, 8, 16), (1000, 64, 8, 16), (4099, 64, 8, 1), (777, 48, 5, 3), (300, 8, 256, 4),
    (2500, 256, 16, 16), (513, 100, 3, 100), (65536, 64, 8, 16)])
def test_assign_matches_oracle(gpu, oracle_mod, n, dims, clusters, width):
    from smi_amd import kmeans
    rng = np.random.default_rng(n * 7 + dims)
    pts = rng.standard_normal((n, dims), dtype=np.float32)
    cen = rng.standard_normal((clusters, dims), dtype=np.float32)
    want = oracle_mod.kmeans_assign(pts, cen, width)
    got = kmeans.assign(dev(pts), dev(cen), width).cpu().numpy()
    assert np.array_equal(got, want)


def test_assign_ties_nan_inf(gpu, oracle_mod):
    """Strict < from +inf (kmeans_smi.cl:75-83): duplicate centroids keep the
    lower index, NaN distances never win, all-NaN/inf points go to 0."""
    from smi_amd import kmeans
    rng = np.random.default_rng(3)
    pts = rng.standard_normal((600, 32), dtype=np.float32)
    pts[5] = np.nan
    pts[6] = np.inf
    c = rng.standard_normal((2, 32), dtype=np.float32)
    cen = np.stack([c[0], c[0], np.full(32, np.nan, np.float32), np.full(32, np.inf, np.float32), c[1]])
    for width in (1, 4, 16):
        want = oracle_mod.kmeans_assign(pts, cen, width)
        got = kmeans.assign(dev(pts), dev(cen), width).cpu().numpy()
        assert np.array_equal(got, want), width
        assert not np.any(got == 1) and got[5] == 0 and got[6] == 0


@pytest.mark.parametrize("n,dims,clusters", [(0, 64, 8), (1, 64, 8), (255, 64, 8), (257, 64, 3), (5000, 64, 8),
                                             (70000, 130, 11), (200000, 64, 8), (3000, 16, 256), (900, 64, 1)])
def test_accumulate_matches_oracle(gpu, oracle_mod, n, dims, clusters):
    from smi_amd import kmeans
    rng = np.random.default_rng(n + clusters)
    pts = rng.standard_normal((n, dims), dtype=np.float32) * 3
    asg = rng.integers(0, max(clusters - 1, 1), n).astype(np.int32)  # the last cluster stays empty
    if n > 10:
        asg[::97] = -1          # outside [0, clusters): no cluster (`index == k` never holds)
        asg[1::89] = clusters
    want_s, want_c = oracle_mod.kmeans_accumulate(pts, asg, clusters)
    s, c = kmeans.accumulate(dev(pts), dev(asg), clusters)
    assert np.array_equal(c.cpu().numpy(), want_c)
    assert np.array_equal(s.cpu().numpy().view(np.uint32), want_s.view(np.uint32))


def test_accumulate_long_chain(gpu, oracle_mod):
    """A cluster holding almost all of 2^20 points: one ~10^6-long fp32 chain
    per dimension across thousands of LDS tiles."""
    from smi_amd import kmeans
    n, dims = 1 << 20, 64
    rng = np.random.default_rng(9)
    pts = rng.random((n, dims), dtype=np.float32)
    asg = np.zeros(n, np.int32)
    asg[rng.integers(0, n, 1000)] = 1
    want_s, want_c = oracle_mod.kmeans_accumulate(pts, asg, 2)
    s, c = kmeans.accumulate(dev(pts), dev(asg), 2)
    assert np.array_equal(c.cpu().numpy(), want_c)
    assert np.array_equal(s.cpu().numpy().view(np.uint32), want_s.view(np.uint32))


def _run_program(pts, cen0, iters, ranks, width):
    from smi_amd import LocalGroup, kmeans

    def fn(comm):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            local = dev(kmeans.split_points(pts, comm.size, comm.rank))
            c = dev(cen0.copy())
            kmeans.kmeans(comm, local, c, iters, width=width)
            s.synchronize()
            return c.cpu().numpy()

    return LocalGroup(ranks).run(fn)


@pytest.mark.parametrize("ranks", [1, 2, 4, 8])
def test_program_matches_oracle(gpu, oracle_mod, ranks):
    """The kmeans_smi program on the reference host's own input (its
    generator, seed 5, 8 clusters x 64 dims, W = 16) split over `ranks`."""
    _, pts, cen0 = oracle_mod.kmeans_reference_data(4096, 8, 64)
    want = oracle_mod.kmeans(pts, cen0, 6, ranks=ranks, width=16)
    for got in _run_program(pts, cen0, 6, ranks, 16):
        assert same_bits(got, want)


def test_program_golden_fixture(gpu, oracle_mod):
    """The committed fixture (tests/golden/golden.json, 8 ranks, W = 16,
    10 iterations) reproduced by the HIP path."""
    import hashlib
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")) as f:
        case = json.load(f)["kmeans"][0]
    _, pts, cen0 = oracle_mod.kmeans_reference_data(case["num_points"], case["clusters"], case["dims"])
    got = _run_program(pts, cen0, case["iterations"], case["ranks"], case["width"])[0]
    assert hashlib.sha256(got.tobytes()).hexdigest() == case["sha256"]


def test_program_plain_distance_and_empty_cluster(gpu, oracle_mod):
    """width = 1 (the plain squared distance) on 3 ranks with a centroid no
    point ever picks: 0/0 = NaN, which then stays empty."""
    _, pts, cen0 = oracle_mod.kmeans_reference_data(1536, 8, 64)
    cen0 = cen0.copy()
    cen0[4] = 1e6
    want = oracle_mod.kmeans(pts, cen0, 5, ranks=3, width=1)
    assert np.isnan(want[4]).all()
    for got in _run_program(pts, cen0, 5, 3, 1):
        assert same_bits(got, want)


def test_bad_arguments_raise(gpu):
    from smi_amd import SMIError, kmeans
    pts = torch.zeros((10, 64), device="cuda")
    with pytest.raises(SMIError):
        kmeans.assign(pts, torch.zeros((8, 64), device="cuda"), width=5)      # 64 % 5 != 0
    with pytest.raises(SMIError):
        kmeans.assign(pts, torch.zeros((257, 64), device="cuda"), width=16)   # > 256 clusters
    with pytest.raises(SMIError):
        kmeans.assign(pts.double(), torch.zeros((8, 64), device="cuda"))
