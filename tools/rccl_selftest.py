#!/usr/bin/env python3
"""Multi-process RCCL self-test (launch with torch.distributed.run).

Exercises the production transport: smi_init over RCCL with the unique id
passed through the torch.distributed store, then SMI_Reduce, SMI_Bcast,
gesummv and a decomposed stencil, each checked against the CPU oracle on
rank 0.  On a 1-GPU box all ranks share device 0 (if RCCL permits it)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle  # noqa: E402
import smi_amd  # noqa: E402
from smi_amd import collectives, gesummv, stencil  # noqa: E402


def main():
    rank = int(os.environ["RANK"])
    if os.environ.get("SMI_FAKE_HOSTS") == "1":
        # One GPU, several ranks: RCCL refuses two ranks on one device of one
        # host ("Duplicate GPU detected"), so give every rank its own host id;
        # RCCL then moves the bytes over its socket transport on loopback.
        os.environ["NCCL_HOSTID"] = f"smi-selftest-host-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    world = int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = smi_amd.Comm.from_env(device=dev)
    ok = True
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        # reduce (fp32 add + int32 add) and bcast
        for t, npdt in ((2, np.float32), (1, np.int32)):
            for count in (7, 4099, 1 << 20):
                rng = np.random.default_rng(1234)
                allc = (rng.random((world, count)) * 100).astype(npdt)
                snd = torch.from_numpy(allc[rank].copy()).cuda()
                rcv = torch.zeros_like(snd)
                collectives.reduce(comm, snd, rcv, "add", root=world - 1)
                s.synchronize()
                if rank == world - 1:
                    want = oracle.reduce(allc, t, 0)
                    good = np.array_equal(rcv.cpu().numpy().view(np.uint8), want.view(np.uint8))
                    print(f"[{rank}] reduce t={t} n={count}: {'OK' if good else 'MISMATCH'}", flush=True)
                    ok &= good
        data = np.arange((1 << 20) + 5, dtype=np.int32)
        buf = torch.from_numpy(data).cuda() if rank == 0 else torch.zeros(len(data), dtype=torch.int32,
                                                                          device="cuda")
        collectives.bcast(comm, buf, root=0)
        s.synchronize()
        good = np.array_equal(buf.cpu().numpy(), data)
        print(f"[{rank}] bcast: {'OK' if good else 'MISMATCH'}", flush=True)
        ok &= good
        # bulk p2p (smi_send / smi_recv): rank 0 -> last rank, bandwidth_*.cl KAT
        n = (1 << 20) + 3
        want = np.float64(np.float32(0.1)) + np.arange(n, dtype=np.float64)
        if rank == 0:
            collectives.send(comm, torch.from_numpy(want).cuda(), world - 1)
        elif rank == world - 1:
            got = torch.zeros(n, dtype=torch.float64, device="cuda")
            collectives.recv(comm, got, 0)
            s.synchronize()
            good = np.array_equal(got.cpu().numpy(), want)
            print(f"[{rank}] p2p send/recv: {'OK' if good else 'MISMATCH'}", flush=True)
            ok &= good
        s.synchronize()
        # decomposed stencil (1 x world, or 2 x world/2)
        PX, PY = (2, world // 2) if world % 2 == 0 and world >= 4 else (1, world)
        g = oracle.init_uniform(256 * PX, 256 * PY, seed=5)
        tiles = stencil.split_memory(g, PX, PY)
        t = torch.from_numpy(tiles[rank]).cuda()
        want = oracle.stencil(g, 13) if rank == 0 else None
        for overlap in (1, 0):
            for fuse in (1, 2, 4, 12):
                stencil.set_tuning(overlap=overlap)
                stencil.set_fusion(steps_per_pass=fuse)
                res = stencil.run(comm, t.clone(), 13, PX, PY)
                s.synchronize()
                tiles_out = [None] * world
                dist.all_gather_object(tiles_out, res.cpu().numpy())
                if rank == 0:
                    got = stencil.combine_memory(tiles_out, PX, PY)
                    good = np.array_equal(got.view(np.uint32), want.view(np.uint32))
                    print(f"[0] stencil {PX}x{PY} overlap={overlap} fuse={fuse}: "
                          f"{'OK' if good else 'MISMATCH'}", flush=True)
                    ok &= good
        # gesummv
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
            good = np.array_equal(y.cpu().numpy().view(np.uint32),
                                  oracle.gesummv(A, B, x, 1.5, 0.5).view(np.uint32))
            print(f"[0] gesummv: {'OK' if good else 'MISMATCH'}", flush=True)
            ok &= good
    comm.finalize()
    flag = torch.tensor([1 if ok else 0])
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    dist.destroy_process_group()
    if rank == 0:
        print("RCCL SELFTEST", "PASS" if flag.item() else "FAIL", flush=True)
    sys.exit(0 if flag.item() else 1)


if __name__ == "__main__":
    main()
