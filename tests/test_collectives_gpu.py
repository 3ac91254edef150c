"""SMI_Reduce / SMI_Bcast parity on the GPU.

Reduce contract: bit-exact vs the oracle's canonical rank-order fold
(codegen/templates/reduce.cl:42-148) for every type and op; the reference's
own known-answer tests (test/reduce/reduce.cl:7-172,
microbenchmarks/kernels/reduce.cl:13-24) replayed over its parameter grid
(lengths {1,128,300} x roots {1,4,7} x 8 ranks).  Bcast: bitwise copy
(test/broadcast/broadcast.cl:9-111, lengths {1,128,1024,10000} x roots
{0,4,7}).  Multi-rank cases run as an in-process rank group on one GPU.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TYPES = {1: torch.int32, 2: torch.float32, 3: torch.float64, 4: torch.int8, 5: torch.int16}


def _contribs(oracle_mod, n, count, t, seed):
    rng = np.random.default_rng(seed)
    npdt = oracle_mod.NP_DTYPE[t]
    if t in (2, 3):
        return (rng.random((n, count)) * 2 - 1).astype(npdt) * npdt(1000.0)
    info = np.iinfo(npdt)
    return rng.integers(info.min, info.max, size=(n, count), endpoint=True, dtype=npdt)


@pytest.mark.parametrize("t", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("op", [0, 1, 2])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 8])
def test_fold_kernel_matches_oracle(gpu, oracle_mod, t, op, n):
    from smi_amd import collectives
    for count in (1, 7, 33, 300, 4099):
        c = _contribs(oracle_mod, n, count, t, seed=count * 7 + n)
        want = oracle_mod.reduce(c, t, op)
        got = collectives.reduce_fold(torch.from_numpy(c).cuda(), op).cpu().numpy()
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), (t, op, n, count)


def test_fold_signed_zero_and_nan(gpu, oracle_mod):
    from smi_amd import collectives
    c = np.array([[-0.0, np.nan, -0.0, 1.0], [-0.0, 1.0, np.nan, -1.0]], dtype=np.float32)
    for op in (0, 1, 2):
        want = oracle_mod.reduce(c, 2, op)
        got = collectives.reduce_fold(torch.from_numpy(c).cuda(), op).cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), op


def _group_reduce(n, sends, t, op, root):
    from smi_amd import LocalGroup, collectives

    def fn(comm):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            snd = torch.from_numpy(sends[comm.rank]).cuda()
            rcv = torch.zeros_like(snd) if comm.rank == root else None
            collectives.reduce(comm, snd, rcv, op, root)
            s.synchronize()
            return None if rcv is None else rcv.cpu().numpy()

    return LocalGroup(n).run(fn)[root]


@pytest.mark.parametrize("root", [1, 4, 7])
@pytest.mark.parametrize("ml", [1, 128, 300])
def test_reduce_reference_kats(gpu, oracle_mod, root, ml):
    """test/reduce/reduce.cl known answers with 8 ranks."""
    n = 8
    i = np.arange(ml)
    cases = [  # (type, op, per-rank send, expected)
        (2, 0, lambda r: i.astype(np.float32), (n * i).astype(np.float32)),            # float add
        (1, 1, lambda r: np.full(ml, r + 1, np.int32), np.full(ml, n, np.int32)),       # int max
        (1, 0, lambda r: np.full(ml, r + 1, np.int32), np.full(ml, n * (n + 1) // 2, np.int32)),
        (2, 2, lambda r: (i + 0.1 * r).astype(np.float32), i.astype(np.float32)),      # float min
        (3, 0, lambda r: i.astype(np.float64), (n * i).astype(np.float64)),             # double add
        (4, 1, lambda r: np.full(ml, r + 1, np.int8), np.full(ml, n, np.int8)),         # char max
        (5, 2, lambda r: np.full(ml, r + 1, np.int16), np.full(ml, 1, np.int16)),       # short min
        (2, 0, lambda r: np.full(ml, r + 1, np.float32), np.full(ml, 36, np.float32)),  # microbench
    ]
    for t, op, mk, expect in cases:
        sends = [mk(r) for r in range(n)]
        got = _group_reduce(n, sends, t, op, root)
        assert np.array_equal(got, expect), (t, op)
        assert np.array_equal(got.view(np.uint8), oracle_mod.reduce(np.stack(sends), t, op).view(np.uint8))


@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("t", [1, 2])
def test_reduce_random_matches_oracle(gpu, oracle_mod, n, t):
    for count in (5, 1000, 1 << 16):
        c = _contribs(oracle_mod, n, count, t, seed=n * count)
        for root in {0, n - 1}:
            got = _group_reduce(n, list(c), t, 0, root)
            assert np.array_equal(got.view(np.uint8), oracle_mod.reduce(c, t, 0).view(np.uint8))


def _group_bcast(n, data, root):
    from smi_amd import LocalGroup, collectives

    def fn(comm):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            buf = torch.from_numpy(data).cuda() if comm.rank == root else torch.zeros(
                data.shape, dtype=torch.from_numpy(data).dtype, device="cuda")
            collectives.bcast(comm, buf, root)
            s.synchronize()
            return buf.cpu().numpy()

    return LocalGroup(n).run(fn)


@pytest.mark.parametrize("root", [0, 4, 7])
@pytest.mark.parametrize("ml", [1, 128, 1024, 10000])
def test_bcast_reference_kats(gpu, root, ml):
    """test/broadcast/broadcast.cl: int i, float i+0.1f, double i+0.1f, char/short root."""
    i = np.arange(ml)
    for data in (i.astype(np.int32), (i + np.float32(0.1)).astype(np.float32),
                 (i + np.float64(np.float32(0.1))).astype(np.float64), np.full(ml, root, np.int8),
                 np.full(ml, root, np.int16)):
        for got in _group_bcast(8, data, root):
            assert np.array_equal(got.view(np.uint8), data.view(np.uint8))


@pytest.mark.parametrize("n", [2, 4, 8])
def test_bcast_large_scatter_allgather(gpu, n):
    rng = np.random.default_rng(n)
    data = rng.integers(0, 1 << 30, size=(1 << 20) + 3, dtype=np.int32)
    for root in (0, n - 1):
        for got in _group_bcast(n, data, root):
            assert np.array_equal(got, data)


@pytest.fixture
def piece_bytes():
    """Set the reduce/bcast pipeline piece size for one test, restore after."""
    from smi_amd import collectives
    old = collectives.get_pipeline_bytes()
    yield collectives.set_pipeline_bytes
    collectives.set_pipeline_bytes(old)


@pytest.mark.parametrize("pb", [0, 16, 1024, 4 << 20])
@pytest.mark.parametrize("n", [2, 3, 8])
def test_reduce_pipelined_pieces_bit_identical(gpu, oracle_mod, piece_bytes, pb, n):
    """The piece size changes the schedule only: every setting (one piece,
    16-byte pieces, many 1 KiB pieces, the 4 MiB default) gives the oracle's
    canonical fold bit for bit, ragged counts included."""
    piece_bytes(pb)
    for t in (1, 2, 3):
        for count in (5, 100003):
            c = _contribs(oracle_mod, n, count, t, seed=count + n + t)
            root = (count + t) % n
            got = _group_reduce(n, list(c), t, 0, root)
            assert np.array_equal(got.view(np.uint8), oracle_mod.reduce(c, t, 0).view(np.uint8)), (pb, t, count)


@pytest.mark.parametrize("n", [2, 5, 8])
def test_reduce_fan_in_boundary(gpu, oracle_mod, n):
    """Messages up to 256 KiB take the direct fan-in (every rank's buffer to
    the root, one fold there), longer ones the owner chunks: both sides of
    the threshold, for 4- and 8-byte types and every op, give the oracle's
    canonical rank-order fold bit for bit."""
    for t, esz in ((1, 4), (3, 8)):
        for count in ((256 << 10) // esz, (256 << 10) // esz + 1, 3, (256 << 10) // esz - 5):
            for op in (0, 1, 2):
                c = _contribs(oracle_mod, n, count, t, seed=count * 3 + n + op)
                root = (count + op) % n
                got = _group_reduce(n, list(c), t, op, root)
                want = oracle_mod.reduce(c, t, op)
                assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), (n, t, count, op)


@pytest.mark.parametrize("pb", [0, 16, 4096])
@pytest.mark.parametrize("n", [3, 8])
def test_bcast_pipelined_pieces(gpu, piece_bytes, pb, n):
    piece_bytes(pb)
    rng = np.random.default_rng(pb + n)
    data = rng.integers(0, 1 << 30, size=(1 << 18) + 7, dtype=np.int32)  # 1 MiB: scatter + all-gather
    for root in (0, n - 1):
        for got in _group_bcast(n, data, root):
            assert np.array_equal(got, data)


@pytest.mark.parametrize("n", [2, 4])
def test_comm_dup_concurrent_ports(gpu, oracle_mod, n):
    """smi_comm_dup: a communicator per port, each driven from its own host
    thread (the reference's collectives on distinct ports,
    microbenchmarks/kernels/multi_collectives.cl:50-76).  Every rank runs a
    reduce chain on the communicator and a bcast chain on its dup at the same
    time, the two threads of odd ranks starting in the opposite order; both
    results stay exact."""
    import threading
    from smi_amd import LocalGroup, collectives

    def fn(comm):
        d = comm.dup()
        out = {}
        count = 1 << 16

        def red():
            s = torch.cuda.Stream()
            snd = torch.full((count,), comm.rank + 1, dtype=torch.int32, device="cuda")
            rcv = torch.empty_like(snd)
            with torch.cuda.stream(s):
                for _ in range(5):
                    collectives.reduce(comm, snd, rcv, "add", root=0, stream=s)
                s.synchronize()
            out["reduce"] = rcv.cpu().numpy() if comm.rank == 0 else None

        def bc():
            s = torch.cuda.Stream()
            buf = (torch.arange(count, dtype=torch.float32, device="cuda") if comm.rank == n - 1
                   else torch.zeros(count, device="cuda"))
            with torch.cuda.stream(s):
                for _ in range(5):
                    collectives.bcast(d, buf, root=n - 1, stream=s)
                s.synchronize()
            out["bcast"] = buf.cpu().numpy()

        order = [red, bc] if comm.rank % 2 == 0 else [bc, red]
        ts = [threading.Thread(target=f) for f in order]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        torch.cuda.synchronize()
        d.finalize()
        return out

    res = LocalGroup(n).run(fn)
    assert (res[0]["reduce"] == n * (n + 1) // 2).all()
    for r in range(n):
        assert np.array_equal(res[r]["bcast"], np.arange(1 << 16, dtype=np.float32)), r
