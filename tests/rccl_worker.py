#!/usr/bin/env python3
"""One rank of the multi-process RCCL parity run (started by
tests/test_rccl_multiproc_gpu.py as a fresh child process, never exec'd).

Production path end to end: gloo process group for the control plane, the
RCCL unique id through its store, smi_init (Comm.from_env), then bulk
collectives, the decomposed stencil, gesummv and the element-granular
channels -- each checked bit for bit against the CPU oracle.  On a 1-GPU box
every rank sets its own NCCL_HOSTID before any GPU call (the parent does it
in the child's environment), so RCCL treats the ranks as separate hosts and
moves the bytes over its socket transport; on an 8-GPU node rank r drives
GPU r and RCCL uses xGMI.  Reference: test/CMakeLists.txt:48-88 runs every
known-answer test as `mpirun -np 8`.

Prints one "CASE <name> OK|MISMATCH" line per check (rank 0 / the root) and
exits 0 only if every rank passed every case.
"""
import os
import sys
import time
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle  # noqa: E402
import smi_amd  # noqa: E402
from smi_amd import channels, collectives, gesummv, stencil  # noqa: E402
from smi_amd import _lib  # noqa: E402

OK = True


def report(rank, name, good):
    global OK
    OK &= bool(good)
    print(f"[{rank}] CASE {name} {'OK' if good else 'MISMATCH'}", flush=True)


def bulk_cases(comm, rank, world, s):
    # reduce: rank+1 known answer (test/reduce/reduce.cl:7-61) and random
    # contributions vs the canonical fold, default and 1 KiB pipeline pieces
    for pb in (4 << 20, 1024):
        collectives.set_pipeline_bytes(pb)
        for t, npdt in ((1, np.int32), (2, np.float32)):
            root = world - 1
            kat = torch.full((4099,), rank + 1, dtype=torch.from_numpy(np.zeros(1, npdt)).dtype, device="cuda")
            rk = torch.zeros_like(kat)
            collectives.reduce(comm, kat, rk, "add", root=root)
            s.synchronize()
            if rank == root:
                report(rank, f"reduce_kat t={t} pb={pb}", bool(torch.all(rk == world * (world + 1) // 2)))
            for count in (7, 100003, 1 << 20):
                rng = np.random.default_rng(count + t)
                allc = ((rng.random((world, count)) * 2 - 1) * 1000).astype(npdt)
                snd = torch.from_numpy(allc[rank].copy()).cuda()
                rcv = torch.zeros_like(snd)
                collectives.reduce(comm, snd, rcv, "add", root=root)
                s.synchronize()
                if rank == root:
                    want = oracle.reduce(allc, t, 0)
                    report(rank, f"reduce t={t} n={count} pb={pb}",
                           np.array_equal(rcv.cpu().numpy().view(np.uint8), want.view(np.uint8)))
        # bcast: fan-out (small) and pipelined scatter + all-gather (1 MiB+)
        for n in (1000, (1 << 18) + 5):
            data = np.arange(n, dtype=np.int32) * 7 + 3
            buf = torch.from_numpy(data).cuda() if rank == 0 else torch.zeros(n, dtype=torch.int32, device="cuda")
            collectives.bcast(comm, buf, root=0)
            s.synchronize()
            report(rank, f"bcast n={n} pb={pb}", np.array_equal(buf.cpu().numpy(), data))
    collectives.set_pipeline_bytes(4 << 20)
    # bulk p2p (bandwidth_*.cl KAT) and bulk scatter/gather
    n = (1 << 20) + 3
    want = np.float64(np.float32(0.1)) + np.arange(n, dtype=np.float64)
    if rank == 0:
        collectives.send(comm, torch.from_numpy(want).cuda(), world - 1)
    elif rank == world - 1:
        got = torch.zeros(n, dtype=torch.float64, device="cuda")
        collectives.recv(comm, got, 0)
        s.synchronize()
        report(rank, "p2p send/recv", np.array_equal(got.cpu().numpy(), want))
    s.synchronize()
    m = 1000
    full = np.arange(world * m, dtype=np.int32)
    snd = torch.from_numpy(full).cuda() if rank == 1 else None
    part = torch.zeros(m, dtype=torch.int32, device="cuda")
    collectives.scatter(comm, snd, part, root=1)
    back = torch.zeros(world * m, dtype=torch.int32, device="cuda") if rank == 0 else None
    collectives.gather(comm, part, back, root=0)
    s.synchronize()
    if rank == 0:
        report(rank, "scatter+gather", np.array_equal(back.cpu().numpy(), full))
    # gesummv, rows sharded, y gathered on root 0
    n, m = 1000, 1024
    rng = np.random.default_rng(7)
    A = rng.random((n, m), dtype=np.float32)
    B = rng.random((n, m), dtype=np.float32)
    x = rng.random(m, dtype=np.float32)
    r0, r1 = gesummv.row_range(n, world, rank)
    y = gesummv.gesummv(comm, torch.from_numpy(A[r0:r1].copy()).cuda(), torch.from_numpy(B[r0:r1].copy()).cuda(),
                        torch.from_numpy(x).cuda(), n, 1.5, 0.5, root=0)
    s.synchronize()
    if rank == 0:
        report(rank, "gesummv", np.array_equal(y.cpu().numpy().view(np.uint32),
                                               oracle.gesummv(A, B, x, 1.5, 0.5).view(np.uint32)))


def stencil_cases(comm, rank, world, s):
    PX, PY = (2, world // 2) if world >= 4 else (1, world)
    g = oracle.init_uniform(256 * PX, 256 * PY, seed=5)
    tiles = stencil.split_memory(g, PX, PY)
    for T in (13, 27):
        want = oracle.stencil(g, T) if rank == 0 else None
        for overlap in (1, 0):
            for fuse in (1, 2, 12, 20):
                stencil.set_tuning(overlap=overlap)
                stencil.set_fusion(steps_per_pass=fuse)
                t = torch.from_numpy(tiles[rank]).cuda()
                res = stencil.run(comm, t, T, PX, PY)
                s.synchronize()
                out = [None] * world
                dist.all_gather_object(out, res.cpu().numpy())
                if rank == 0:
                    got = stencil.combine_memory(out, PX, PY)
                    report(rank, f"stencil {PX}x{PY} T={T} overlap={overlap} K={fuse}",
                           np.array_equal(got.view(np.uint32), want.view(np.uint32)))
    # three K = 20 passes over RCCL, the pass boundary joined on the host
    # (default) and by a device-side stream wait (smi_stencil_set_join(0))
    T = 60
    want = oracle.stencil(g, T) if rank == 0 else None
    stencil.set_tuning(overlap=1)
    stencil.set_fusion(steps_per_pass=20)
    for join in (1, 0):
        stencil.set_join(join)
        t = torch.from_numpy(tiles[rank]).cuda()
        res = stencil.run(comm, t, T, PX, PY)
        s.synchronize()
        out = [None] * world
        dist.all_gather_object(out, res.cpu().numpy())
        if rank == 0:
            got = stencil.combine_memory(out, PX, PY)
            report(rank, f"stencil {PX}x{PY} T={T} overlap=1 K=20 (three passes) join={join}",
                   np.array_equal(got.view(np.uint32), want.view(np.uint32)))
    stencil.set_join(1)
    stencil.set_tuning(overlap=1)
    stencil.set_fusion(steps_per_pass=20)


def channel_cases(comm, rank, world, s):
    F = _lib.SMI_FLOAT
    per_msg = (16384 - 16) // 4
    partner = rank ^ 1
    if partner < world:
        # symmetric push-before-pop: both partners push 3 packets' worth, then pop
        cnt = 3 * per_msg + 5
        tx = channels.open_send_channel(cnt, F, partner, 0, comm)
        for i in range(cnt):
            tx.push(float(rank * 100000 + i))
        rx = channels.open_receive_channel(cnt, F, partner, 0, comm)
        got = [rx.pop() for _ in range(cnt)]
        want = [float(np.float32(partner * 100000 + i)) for i in range(cnt)]
        report(rank, "chan symmetric push-before-pop", got == want)
        # push, then a bulk collective, then pop: the packets must not be
        # consumed by the collective's receives
        tx = channels.open_send_channel(10, F, partner, 3, comm)
        for i in range(10):
            tx.push(float(i + 0.5))
    snd = torch.full((300,), rank + 1, dtype=torch.int32, device="cuda")
    rcv = torch.zeros_like(snd)
    collectives.reduce(comm, snd, rcv, "add", root=0)
    collectives.bcast(comm, rcv, root=0)
    s.synchronize()
    report(rank, "chan-interleaved bulk reduce+bcast", bool(torch.all(rcv == world * (world + 1) // 2)))
    if partner < world:
        rx = channels.open_receive_channel(10, F, partner, 3, comm)
        got = [rx.pop() for _ in range(10)]
        report(rank, "chan push-collective-pop", got == [i + 0.5 for i in range(10)])
    # more than 8 packets in flight one way: rank 0 pushes 12 packets to the
    # last rank, which pops them only after a pause
    cnt = 12 * per_msg
    if rank == 0:
        tx = channels.open_send_channel(cnt, F, world - 1, 5, comm)
        for i in range(cnt):
            tx.push(float(i))
    elif rank == world - 1:
        time.sleep(1.0)
        rx = channels.open_receive_channel(cnt, F, 0, 5, comm)
        got = np.array([rx.pop() for _ in range(cnt)], dtype=np.float32)
        report(rank, "chan 12 packets unpopped", np.array_equal(got, np.arange(cnt, dtype=np.float32)))
    # element bcast / reduce / scatter / gather (test/broadcast, test/reduce,
    # test/scatter, test/gather known answers)
    root = world - 1
    bc = channels.BChannel(1000, _lib.SMI_INT, 7, root, comm)
    vals = [bc.bcast(i if rank == root else 0) for i in range(1000)]
    report(rank, "chan bcast", vals == list(range(1000)))
    rc = channels.RChannel(128, _lib.SMI_INT, _lib.SMI_ADD, 8, root, comm)
    red = [rc.reduce(rank + 1) for _ in range(128)]
    if rank == root:
        report(rank, "chan reduce", red == [world * (world + 1) // 2] * 128)
    sc = channels.ScatterChannel(50, 50, _lib.SMI_INT, 9, 0, comm)
    got = [sc.scatter(i if rank == 0 else 0) for i in range(50 * (world if rank == 0 else 1))]
    if rank != 0:
        report(rank, "chan scatter", got == list(range(rank * 50, rank * 50 + 50)))
    ga = channels.GatherChannel(40, 40, _lib.SMI_INT, 10, 0, comm)
    got = [ga.gather(rank * 1000 + i) for i in range(40 * (world if rank == 0 else 1))]
    if rank == 0:
        report(rank, "chan gather", got == [r * 1000 + i for r in range(world) for i in range(40)])


def dup_cases(comm, rank, world, s):
    """smi_comm_dup (an RCCL communicator split off this one): a reduce on the
    communicator and a bcast on its dup, issued in OPPOSITE orders on even and
    odd ranks, on two streams -- RCCL matches the two communicators apart."""
    d = comm.dup()
    s2 = torch.cuda.Stream()
    count = 1 << 18
    snd = torch.full((count,), rank + 1, dtype=torch.int32, device="cuda")
    rcv = torch.zeros_like(snd)
    buf = (torch.arange(count, dtype=torch.float32, device="cuda") if rank == 0
           else torch.zeros(count, device="cuda"))
    torch.cuda.synchronize()

    def red():
        collectives.reduce(comm, snd, rcv, "add", root=world - 1, stream=s)

    def bc():
        collectives.bcast(d, buf, root=0, stream=s2)

    for f in ((red, bc) if rank % 2 == 0 else (bc, red)):
        f()
    s.synchronize()
    s2.synchronize()
    if rank == world - 1:
        report(rank, "dup reduce", bool(torch.all(rcv == world * (world + 1) // 2)))
    report(rank, "dup bcast", bool(torch.equal(buf, torch.arange(count, dtype=torch.float32, device="cuda"))))
    dist.barrier()
    d.finalize()


def finalize_cases(comm, rank, world, s):
    """The event-lifetime rule behind round 3's crash (a finalizing rank
    destroyed an event its peer still waited on; fixed in 1074c45), made
    deterministic: rank 0 posts detached element sends on a dup and calls
    finalize at once (finalize drains: it returns when the peer has received
    them); rank 1 waits until rank 0 is inside finalize, pops every element,
    waits until rank 0's finalize has returned, then uses its own streams
    again and finalizes."""
    from torch.distributed import distributed_c10d as c10d
    store = c10d._get_default_store()
    d = comm.dup()
    n = 1000
    if rank == 0:
        c = channels.open_send_channel(n, 1, 1, 3, d)
        for i in range(n):
            c.push(7 * i + 1)
        store.set("fin/r0_entering", "1")
        d.finalize()
        store.set("fin/r0_done", "1")
    elif rank == 1:
        store.wait(["fin/r0_entering"])
        time.sleep(0.05)
        c = channels.open_receive_channel(n, 1, 0, 3, d)
        got = [c.pop() for _ in range(n)]
        store.wait(["fin/r0_done"])
        x = torch.arange(1 << 16, device="cuda", dtype=torch.float32) * 3
        torch.cuda.synchronize()
        report(rank, "finalize with detached sends in flight",
               got == [7 * i + 1 for i in range(n)] and float(x[-1]) == 3 * ((1 << 16) - 1))
        d.finalize()
    else:
        d.finalize()


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = smi_amd.Comm.from_env(device=dev)
    s = torch.cuda.Stream()
    try:
        with torch.cuda.stream(s):
            for part in (bulk_cases, stencil_cases, channel_cases, dup_cases, finalize_cases):
                part(comm, rank, world, s)
                s.synchronize()
                dist.barrier()
    except Exception:  # noqa: BLE001
        traceback.print_exc()
        global OK
        OK = False
    comm.finalize()
    flag = torch.tensor([1 if OK else 0])
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    dist.destroy_process_group()
    if rank == 0:
        print("RCCL MULTIPROC", "PASS" if flag.item() else "FAIL", flush=True)
    sys.exit(0 if flag.item() else 1)


if __name__ == "__main__":
    main()
