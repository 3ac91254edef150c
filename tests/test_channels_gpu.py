"""Element-granular channels on the GPU transport (in-process 8-rank group).

Known-answer tests replayed from the reference's own suites:
  p2p       test/p2p/p2p_rank0.cl:8-124, p2p_rank1.cl:9-175, lengths
            {1,128,1024,10000} x receivers {1,4,7} (test/p2p/test_p2p.cpp:80-82)
  bcast     test/broadcast/broadcast.cl:9-111, lengths {1,128,1024,10000} x
            roots {0,4,7}
  reduce    test/reduce/reduce.cl:7-172, lengths {1,128,300} x roots {1,4,7}
  scatter   test/scatter/scatter.cl (root scatters i, rank r checks r*N+i)
  gather    test/gather/gather.cl (rank r sends r; root sees 0..n-1 in order)
  mixed     test/mixed/mixed.cl:11-35 (p2p pipeline, then a bcast)
  balanced  test/balanced_routing/balanced_routing.cl (two-port pipeline,
            two concurrent bcasts; lengths {2,8,10000}, roots {0,4,5},
            test_balanced_routing.cpp:75,105-107)
plus port demultiplexing and push-before-pop buffering, and the bulk
smi_scatter / smi_gather on device buffers.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

INT, FLOAT, DOUBLE, CHAR, SHORT = 1, 2, 3, 4, 5


def group(n, fn):
    from smi_amd import LocalGroup
    return LocalGroup(n).run(fn)


@pytest.mark.parametrize("N", [1, 128, 1024, 10000])
@pytest.mark.parametrize("dest", [1, 4, 7])
def test_p2p_reference_kats(gpu, N, dest):
    from smi_amd import channels as ch
    f1 = np.float32(1.1)
    cases = [  # (type, port, value(i)) -- p2p_rank0.cl / p2p_rank1.cl
        (CHAR, 1, lambda i: 3), (SHORT, 0, lambda i: 1001), (INT, 2, lambda i: i),
        (FLOAT, 3, lambda i: np.float32(i + f1)), (DOUBLE, 4, lambda i: np.float64(i) + np.float64(f1))]

    def fn(comm):
        ok = True
        for t, port, val in cases:
            if comm.rank == 0:
                c = ch.open_send_channel(N, t, dest, port, comm)
                for i in range(N):
                    c.push(val(i))
            elif comm.rank == dest:
                c = ch.open_receive_channel(N, t, 0, port, comm)
                for i in range(N):
                    ok &= bool(c.pop() == ch.NP[t](val(i)))
        return ok

    assert all(group(8, fn))


def test_ports_are_separate_fifos(gpu):
    """Interleaved pushes on two ports, popped port 1 first."""
    from smi_amd import channels as ch

    def fn(comm):
        if comm.rank == 0:
            a = ch.open_send_channel(300, INT, 1, 0, comm)
            b = ch.open_send_channel(300, INT, 1, 1, comm)
            for i in range(300):
                a.push(i)
                b.push(1000 + i, immediate=(i % 7 == 0))
            return True
        b = ch.open_receive_channel(300, INT, 0, 1, comm)
        got_b = [b.pop() for _ in range(300)]
        a = ch.open_receive_channel(300, INT, 0, 0, comm)
        got_a = [a.pop() for _ in range(300)]
        return got_a == list(range(300)) and got_b == list(range(1000, 1300))

    assert all(group(2, fn))


def test_push_before_pop_both_directions(gpu):
    """Both ranks push 5000 floats before popping (the credit-window case)."""
    from smi_amd import channels as ch

    def fn(comm):
        peer = 1 - comm.rank
        s = ch.open_send_channel(5000, FLOAT, peer, 2, comm)
        for i in range(5000):
            s.push(np.float32(comm.rank * 10000 + i))
        r = ch.open_receive_channel(5000, FLOAT, peer, 2, comm)
        return all(r.pop() == np.float32(peer * 10000 + i) for i in range(5000))

    assert all(group(2, fn))


@pytest.mark.parametrize("ad", [1, 3, 64, 1 << 20])
def test_asynch_degree_channels(gpu, ad):
    """The `_ad` opens (asynch degree = elements packed per message, the
    reference's FIFO depth): same data for every degree, sender and receiver
    degrees need not match; p2p, bcast and reduce."""
    from smi_amd import channels as ch

    def fn(comm):
        ok = True
        if comm.rank == 0:
            c = ch.open_send_channel(777, INT, 1, 0, comm, asynch_degree=ad)
            for i in range(777):
                c.push(3 * i)
        elif comm.rank == 1:
            c = ch.open_receive_channel(777, INT, 0, 0, comm, asynch_degree=5)
            ok &= all(c.pop() == 3 * i for i in range(777))
        b = ch.BChannel(300, FLOAT, 1, 2, comm, asynch_degree=ad)
        ok &= all(b.bcast(np.float32(i) if comm.rank == 2 else 0) == np.float32(i) for i in range(300))
        r = ch.RChannel(200, INT, 0, 2, 1, comm, asynch_degree=ad)
        for i in range(200):
            v = r.reduce(comm.rank + i)
            if comm.rank == 1:
                ok &= v == sum(k + i for k in range(comm.size))
        return ok

    assert all(group(3, fn))


ESZ = {CHAR: 1, SHORT: 2, INT: 4, FLOAT: 4, DOUBLE: 8}
PAYLOAD = 16384 - 16  # channels.cpp: 16 KiB messages, 16-byte header


@pytest.mark.parametrize("t", [CHAR, SHORT, INT, FLOAT, DOUBLE])
def test_packet_boundaries(gpu, t):
    """Counts at and around whole packets for every type (per packet:
    16,368 bytes of elements): the last element of a full packet, the first
    of the next, a lone element in a packet of its own; p2p and bcast."""
    from smi_amd import channels as ch
    per = PAYLOAD // ESZ[t]
    counts = [per - 1, per, per + 1, 2 * per + 1]
    mod = {CHAR: 127, SHORT: 32749}.get(t, 1 << 30)

    def val(i):
        return ch.NP[t](i % mod)

    def fn(comm):
        ok = True
        for n in counts:
            if comm.rank == 0:
                c = ch.open_send_channel(n, t, 1, 3, comm)
                for i in range(n):
                    c.push(val(i))
            else:
                c = ch.open_receive_channel(n, t, 0, 3, comm)
                ok &= all(c.pop() == val(i) for i in range(n))
            b = ch.BChannel(n, t, 4, 0, comm)
            got = [b.bcast(val(i) if comm.rank == 0 else 0) for i in range(n)]
            ok &= all(g == val(i) for i, g in enumerate(got))
        return ok

    assert all(group(2, fn))


def test_transient_channel_ends_after_count(gpu):
    from smi_amd import SMIError
    from smi_amd import channels as ch

    def fn(comm):
        if comm.rank == 0:
            c = ch.open_send_channel(3, INT, 1, 0, comm)
            for i in range(3):
                c.push(i)
            with pytest.raises(SMIError):
                c.push(99)
            return True
        c = ch.open_receive_channel(3, INT, 0, 0, comm)
        return [c.pop() for _ in range(3)] == [0, 1, 2]

    assert all(group(2, fn))


@pytest.mark.parametrize("N", [1, 128, 1024, 10000])
@pytest.mark.parametrize("root", [0, 4, 7])
def test_bcast_reference_kats(gpu, N, root):
    from smi_amd import channels as ch
    off = np.float32(0.1)
    cases = [(INT, 0, lambda i: i), (FLOAT, 1, lambda i: np.float32(i + off)),
             (DOUBLE, 2, lambda i: np.float64(i) + np.float64(off)), (CHAR, 3, lambda i: root),
             (SHORT, 4, lambda i: root)]

    def fn(comm):
        ok = True
        for t, port, val in cases:
            c = ch.BChannel(N, t, port, root, comm)
            for i in range(N):
                got = c.bcast(val(i) if comm.rank == root else 0)
                ok &= bool(got == ch.NP[t](val(i)))
        return ok

    assert all(group(8, fn))


@pytest.mark.parametrize("N", [1, 128, 300])
@pytest.mark.parametrize("root", [1, 4, 7])
def test_reduce_reference_kats(gpu, N, root):
    from smi_amd import channels as ch
    n = 8
    cases = [  # (type, op, port, send(rank,i), expected(i))  -- test/reduce/reduce.cl
        (FLOAT, 0, 0, lambda r, i: np.float32(i), lambda i: np.float32(n * i)),
        (INT, 1, 2, lambda r, i: r + 1, lambda i: n),
        (INT, 0, 1, lambda r, i: r + 1, lambda i: n * (n + 1) // 2),
        (FLOAT, 2, 3, lambda r, i: np.float32(i + 0.1 * r), lambda i: np.float32(i)),
        (DOUBLE, 0, 6, lambda r, i: np.float64(i), lambda i: np.float64(n * i)),
        (CHAR, 1, 7, lambda r, i: r + 1, lambda i: n),
        (SHORT, 2, 8, lambda r, i: r + 1, lambda i: 1)]

    def fn(comm):
        ok = True
        for t, op, port, snd, exp in cases:
            c = ch.RChannel(N, t, op, port, root, comm)
            for i in range(N):
                got = c.reduce(snd(comm.rank, i))
                if comm.rank == root:
                    ok &= bool(got == ch.NP[t](exp(i)))
        return ok

    assert all(group(n, fn))


@pytest.mark.parametrize("N", [1, 128, 1000])
@pytest.mark.parametrize("root", [0, 3])
def test_scatter_gather_reference_kats(gpu, N, root):
    from smi_amd import channels as ch
    n = 4

    def fn(comm):
        ok = True
        for t, port in ((INT, 0), (FLOAT, 1), (DOUBLE, 2)):
            c = ch.ScatterChannel(N, N, t, port, root, comm)
            bound = N * n if comm.rank == root else N
            for i in range(bound):
                got = c.scatter(i if comm.rank == root else 0)
                if comm.rank != root:
                    ok &= bool(got == ch.NP[t](comm.rank * N + i))
                elif i // N == root:
                    ok &= bool(got == ch.NP[t](i))  # the root's own segment
        for t, port in ((CHAR, 3), (SHORT, 4), (INT, 5)):
            c = ch.GatherChannel(N, N, t, port, root, comm)
            bound = N * n if comm.rank == root else N
            for i in range(bound):
                got = c.gather(comm.rank)
                if comm.rank == root:
                    ok &= bool(got == i // N)
        return ok

    assert all(group(n, fn))


@pytest.mark.parametrize("n", [1, 2, 8])
def test_bulk_scatter_gather(gpu, n):
    from smi_amd import collectives
    count = 1000
    root = n - 1
    data = np.arange(n * count, dtype=np.int32) * 3

    def fn(comm):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            send = torch.from_numpy(data).cuda() if comm.rank == root else None
            recv = torch.zeros(count, dtype=torch.int32, device="cuda")
            collectives.scatter(comm, send, recv, root)
            back = torch.zeros(n * count, dtype=torch.int32, device="cuda") if comm.rank == root else None
            collectives.gather(comm, recv, back, root)
            s.synchronize()
            ok = np.array_equal(recv.cpu().numpy(), data[comm.rank * count:(comm.rank + 1) * count])
            if comm.rank == root:
                ok &= np.array_equal(back.cpu().numpy(), data)
            return ok

    assert all(group(n, fn))


@pytest.mark.parametrize("start", [0, 41])
def test_mixed_reference_kat(gpu, start):
    """test/mixed/mixed.cl:11-35: rank r pops from r-1, adds one, pushes to
    r+1; the last rank then broadcasts on port 1 -- all end with start+n-1."""
    from smi_amd import channels as ch

    def fn(comm):
        r, n = comm.rank, comm.size
        data = start
        if r > 0:
            data = int(ch.open_receive_channel(1, INT, r - 1, 0, comm).pop()) + 1
        if r < n - 1:
            ch.open_send_channel(1, INT, r + 1, 0, comm).push(data)
        final = data if r == n - 1 else 0
        return int(ch.BChannel(1, INT, 1, n - 1, comm).bcast(final))

    assert group(8, fn) == [start + 7] * 8


@pytest.mark.parametrize("N", [2, 8, 10000])
def test_balanced_routing_pipeline_kat(gpu, N):
    """balanced_routing.cl:8-48: two channels per direction along the rank
    pipeline; the last rank sees i + n - 1 and i + n."""
    from smi_amd import channels as ch

    def fn(comm):
        r, n = comm.rank, comm.size
        if r > 0:
            r1 = ch.open_receive_channel(N, INT, r - 1, 0, comm)
            r2 = ch.open_receive_channel(N, INT, r - 1, 1, comm)
        if r < n - 1:
            s1 = ch.open_send_channel(N, INT, r + 1, 0, comm)
            s2 = ch.open_send_channel(N, INT, r + 1, 1, comm)
        ok, e1, e2 = True, n - 1, n
        for i in range(N):
            if r > 0:
                d1, d2 = int(r1.pop()) + 1, int(r2.pop()) + 1
            else:
                d1, d2 = i, i + 1
            if r < n - 1:
                s1.push(d1)
                s2.push(d2)
            else:
                ok &= d1 == e1 and d2 == e2
                e1 += 1
                e2 += 1
        return ok

    assert all(group(8, fn))


@pytest.mark.parametrize("N", [2, 8, 10000])
@pytest.mark.parametrize("root", [0, 4, 5])
def test_balanced_routing_broadcast_kat(gpu, N, root):
    """balanced_routing.cl:51-69: two broadcasts (ports 2, 3) interleaved
    element by element."""
    from smi_amd import channels as ch

    def fn(comm):
        b1 = ch.BChannel(N, INT, 2, root, comm)
        b2 = ch.BChannel(N, INT, 3, root, comm)
        ok = True
        for i in range(N):
            a = b1.bcast(i if comm.rank == root else -1)
            b = b2.bcast(i if comm.rank == root else -1)
            ok &= a == i and b == i
        return ok

    assert all(group(8, fn))


@pytest.mark.parametrize("N", [1, 1000, 1 << 20])
@pytest.mark.parametrize("dest", [1, 4, 7])
def test_bulk_p2p_bandwidth_kat(gpu, N, dest):
    """microbenchmarks/kernels/bandwidth_0.cl / bandwidth_1.cl: rank 0 streams
    N doubles 0.1f + i to `dest` on two ports; the receiver checks every one."""
    from smi_amd import collectives
    start = np.float64(np.float32(0.1))
    want = start + np.arange(N, dtype=np.float64)

    def fn(comm):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            ok = True
            for port in (0, 1):
                if comm.rank == 0:
                    collectives.send(comm, torch.from_numpy(want).cuda(), dest, port, stream=s)
                elif comm.rank == dest:
                    got = torch.zeros(N, dtype=torch.float64, device="cuda")
                    collectives.recv(comm, got, 0, port, stream=s)
                    s.synchronize()
                    ok &= np.array_equal(got.cpu().numpy(), want)
            s.synchronize()
            return ok

    assert all(group(8, fn))


def test_bulk_p2p_latency_pingpong_and_order(gpu):
    """microbenchmarks/kernels/latency_0.cl / latency_1.cl: one int bounces
    between ranks 0 and 1, rank 1 increments it; then three messages of
    different sizes between one pair arrive in issue order."""
    from smi_amd import collectives

    def fn(comm):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            v = torch.zeros(1, dtype=torch.int32, device="cuda")
            for _ in range(50):
                if comm.rank == 0:
                    collectives.send(comm, v, 1, stream=s)
                    collectives.recv(comm, v, 1, stream=s)
                else:
                    collectives.recv(comm, v, 0, stream=s)
                    v += 1
                    collectives.send(comm, v, 0, stream=s)
            sizes = (3, 1 << 16, 17)
            if comm.rank == 0:
                for k, n in enumerate(sizes):
                    collectives.send(comm, torch.full((n,), k + 1, dtype=torch.int16, device="cuda"), 1,
                                     stream=s)
                s.synchronize()
                return int(v.item()) == 50
            got = [torch.zeros(n, dtype=torch.int16, device="cuda") for n in sizes]
            for k, g in enumerate(got):
                collectives.recv(comm, g, 0, stream=s)
            s.synchronize()
            return int(v.item()) == 50 and all(bool((g == k + 1).all()) for k, g in enumerate(got))

    assert all(group(2, fn))


def test_bulk_p2p_errors(gpu):
    from smi_amd import LocalGroup, collectives
    from smi_amd._lib import SMIError
    comm = LocalGroup(1).comm(0)
    buf = torch.zeros(4, device="cuda")
    with pytest.raises(SMIError):
        collectives.send(comm, buf, 0)      # to self
    with pytest.raises(SMIError):
        collectives.recv(comm, buf, 3)      # peer out of range
    comm.finalize()


def test_finalize_with_detached_sends_in_flight(gpu):
    """Round 3's crash (gpurun_out/r03_full1/gpu_tests.log: ranks finalizing
    while peers were still inside element bcasts; the in-process transport
    destroyed a `done` event a peer still waited on -- fixed in 1074c45 with
    pool-owned event handles), made deterministic: rank 0 posts detached
    element sends and calls finalize at once (finalize drains, i.e. returns
    once the peer has received them); rank 1 waits until rank 0 is inside
    finalize, pops every element, waits until rank 0's finalize has
    returned and then keeps exchanging with rank 2 over the same group, whose
    event pool must outlive rank 0's transport."""
    import threading
    import time
    from smi_amd import LocalGroup, channels as ch
    g = LocalGroup(3)
    n = 1000
    entering, done = threading.Event(), threading.Event()
    res = {}
    errs = []

    def r0():
        torch.cuda.set_device(0)
        c = g.comm(0)
        s = ch.open_send_channel(n, INT, 1, 3, c)
        for i in range(n):
            s.push(7 * i + 1)
        entering.set()
        c.finalize()
        done.set()

    def r1():
        torch.cuda.set_device(0)
        c = g.comm(1)
        assert entering.wait(60)
        time.sleep(0.05)
        r = ch.open_receive_channel(n, INT, 0, 3, c)
        res["from0"] = [r.pop() for _ in range(n)]
        assert done.wait(60)
        s = ch.open_send_channel(n, INT, 2, 4, c)
        for i in range(n):
            s.push(5 * i)
        c.finalize()

    def r2():
        torch.cuda.set_device(0)
        c = g.comm(2)
        assert done.wait(60)
        r = ch.open_receive_channel(n, INT, 1, 4, c)
        res["from1"] = [r.pop() for _ in range(n)]
        c.finalize()

    def wrap(f):
        def run():
            try:
                f()
            except BaseException as e:  # noqa: BLE001
                errs.append(e)
        return run

    ts = [threading.Thread(target=wrap(f), daemon=True) for f in (r0, r1, r2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
        assert not t.is_alive(), "rank thread hung"
    assert not errs, errs
    assert res["from0"] == [7 * i + 1 for i in range(n)]
    assert res["from1"] == [5 * i for i in range(n)]


def test_local_group_refuses_second_device(gpu):
    """An in-process group runs on one device (its copy kernel reads the
    sender's buffer, its ordering events skip the system-scope fence):
    smi_init_local refuses a rank on another device."""
    import ctypes
    from smi_amd import LocalGroup, _lib
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs (the check sits behind the device-range check)")
    g = LocalGroup(2)
    c0 = g.comm(0)
    bad = _lib.SMI_Comm()
    rc = _lib.load().smi_init_local(g.group_id, 1, 1, ctypes.byref(bad))
    assert rc != 0
    c1 = g.comm(1)
    c0.finalize()
    c1.finalize()
