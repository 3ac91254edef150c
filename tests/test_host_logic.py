"""Host-side logic on CPU: decomposition helpers (SplitMemory/CombineMemory,
rank map), gesummv row split, bench decomposition, and the world_size=2
gloo bring-up of the RCCL unique id + a decomposed stencil whose halos move
through gloo point-to-point (the Convert{Send,Receive}* protocol of
stencil_smi.cl:236-386 with the same neighbour/port mapping as the C++
runtime), checked against the single-grid oracle."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle as o


def test_split_combine_roundtrip():
    from smi_amd import stencil
    g = o.init_uniform(12, 20, seed=1)
    for PX, PY in [(1, 1), (2, 2), (3, 4), (4, 5), (12, 1)]:
        tiles = stencil.split_memory(g, PX, PY)
        assert len(tiles) == PX * PY
        assert np.array_equal(stencil.combine_memory(tiles, PX, PY), g)
        # tile (px,py) belongs to rank px*PY+py (stencil_smi.cpp:48-62,133-134)
        for r, t in enumerate(tiles):
            px, py = stencil.rank_coords(r, PY)
            XL, YL = 12 // PX, 20 // PY
            assert np.array_equal(t, g[px * XL:(px + 1) * XL, py * YL:(py + 1) * YL])


def test_split_rejects_ragged():
    from smi_amd import stencil
    with pytest.raises(ValueError):
        stencil.split_memory(np.zeros((10, 10), np.float32), 3, 1)


def test_init_grid_matches_reference_pattern():
    from smi_amd import stencil
    assert np.array_equal(stencil.init_grid(9, 13), o.init_edges(9, 13))


def test_gesummv_row_ranges_partition():
    from smi_amd import gesummv
    for n in (0, 1, 7, 32768):
        for size in (1, 2, 3, 8):
            rr = [gesummv.row_range(n, size, r) for r in range(size)]
            assert rr[0][0] == 0 and rr[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rr, rr[1:]))


def test_bench_decomposition():
    import bench
    assert bench.decomposition(1) == (1, 1)
    assert bench.decomposition(2) == (1, 2)
    assert bench.decomposition(4) == (2, 2)
    assert bench.decomposition(8) == (2, 4)
    for n in (3, 6, 12):
        px, py = bench.decomposition(n)
        assert px * py == n


def test_bench_halo_report_counts_neighbours():
    import bench
    # 2x4: an inner-column rank has 1 vertical, 2 horizontal, 2 diagonal neighbours
    h = bench.halo_report(2, 4, 8192, 8192, 12, 0.02)
    assert h["neighbours"] == {"vertical": 1, "horizontal": 2, "diagonal": 2}
    assert h["bytes_per_step_busiest_rank"] == 4 * (8192 + 2 * 8192) + 4 * 2 * 12
    # one 32 KiB column per step per link at 20 us per step
    assert abs(h["link_GBs_needed"] - 32768 / 20e-6 / 1e9) < 0.01
    h1 = bench.halo_report(1, 2, 8192, 8192, 12, 0.02)
    assert h1["neighbours"] == {"vertical": 0, "horizontal": 1, "diagonal": 0}


# ------------------------------------------------------ gloo, world_size 2 --
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _neighbours(rank, PX, PY):
    ipx, ipy = rank // PY, rank % PY
    return dict(top=(ipx - 1) * PY + ipy if ipx > 0 else -1,
                bottom=(ipx + 1) * PY + ipy if ipx < PX - 1 else -1,
                left=rank - 1 if ipy > 0 else -1,
                right=rank + 1 if ipy < PY - 1 else -1)


def _worker(rank, world, port, PX, PY, T, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from smi_amd.comm import exchange_unique_id
        uid = exchange_unique_id(rank, world, dist.distributed_c10d._get_default_store(), key="t/uid")
        ids = [None] * world
        dist.all_gather_object(ids, uid)
        g = o.init_uniform(16 * PX, 12 * PY, seed=9)
        XL, YL = 16, 12
        ipx, ipy = rank // PY, rank % PY
        tile = g[ipx * XL:(ipx + 1) * XL, ipy * YL:(ipy + 1) * YL].copy()
        nb = _neighbours(rank, PX, PY)
        for _ in range(T):
            ext = np.zeros((XL + 2, YL + 2), np.float32)
            ext[1:-1, 1:-1] = tile
            reqs = []
            bufs = {}
            for side, peer, data in (("top", nb["top"], tile[0]), ("bottom", nb["bottom"], tile[-1]),
                                     ("left", nb["left"], tile[:, 0]), ("right", nb["right"], tile[:, -1])):
                if peer < 0:
                    continue
                reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(data)), peer))
                bufs[side] = torch.empty(len(data))
                reqs.append(dist.irecv(bufs[side], peer))
            for r in reqs:
                r.wait()
            if "top" in bufs:
                ext[0, 1:-1] = bufs["top"].numpy()
            if "bottom" in bufs:
                ext[-1, 1:-1] = bufs["bottom"].numpy()
            if "left" in bufs:
                ext[1:-1, 0] = bufs["left"].numpy()
            if "right" in bufs:
                ext[1:-1, -1] = bufs["right"].numpy()
            new = o.stencil(ext, 1)[1:-1, 1:-1].copy()
            # global edges are copied (stencil_smi.cl:143-151)
            if nb["top"] < 0:
                new[0] = tile[0]
            if nb["bottom"] < 0:
                new[-1] = tile[-1]
            if nb["left"] < 0:
                new[:, 0] = tile[:, 0]
            if nb["right"] < 0:
                new[:, -1] = tile[:, -1]
            tile = new
        tiles = [None] * world
        dist.all_gather_object(tiles, tile)
        if rank == 0:
            from smi_amd import stencil
            got = stencil.combine_memory(tiles, PX, PY)
            q.put((ids[0] == ids[1] and len(ids[0]) == 128,
                   bool(np.array_equal(got.view(np.uint32), o.stencil(g, T).view(np.uint32)))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("pxpy", [(1, 2), (2, 1)])
def test_gloo_world2_halo_protocol(pxpy):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, pxpy[0], pxpy[1], 6, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    same_uid, exact = q.get(timeout=5)
    assert same_uid, "RCCL unique id not shared through the store"
    assert exact, "decomposed halo protocol differs from the single-grid oracle"
