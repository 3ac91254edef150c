"""Host-side logic on CPU: decomposition helpers (SplitMemory/CombineMemory,
rank map), the run planner of libsmi_amd (smi_stencil_plan: phases, the
neighbour map, the result buffer), gesummv row split, bench decomposition,
and the world_size=2 gloo bring-up of the RCCL unique id + a decomposed
stencil that follows libsmi_amd's own plan and neighbour map and moves its
depth-K halos (K rows / columns per side, K x K corner blocks) through gloo
point-to-point -- the schedule of smi_stencil_run replacing the
Convert{Send,Receive}* kernels of stencil_smi.cl:236-386 -- checked against
the single-grid oracle."""
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


# ------------------------------------------------------------ run planner --
def test_plan_splits_steps_into_balanced_deep_passes():
    """smi_stencil_plan (host only), default K = 20 on an 8192^2 single tile:
    a remainder r = T % 20 >= 3 is spread over ceil(T / 20) passes balanced
    to within one step; r = 1 or 2 stays T // 20 passes of 20 and a pair or
    a single step.  K > 12 needs a sweep rectangle of at least 4K rows (a
    multi-rank interior loses K rows per side with a neighbour), else K is
    clipped to 12."""
    from smi_amd import stencil
    assert stencil.get_fusion()["steps_per_pass"] == 20
    for T in range(0, 90):
        ph = stencil.plan(8192, 8192, 1, 1, 0, T)["phases"]
        assert sum(k * n for k, n in ph) == T
        q, r = divmod(T, 20)
        if r >= 3:
            base, extra = divmod(T, q + 1)
            want = ([(base + 1, extra)] if extra else []) + [(base, q + 1 - extra)]
        else:
            want = ([(20, q)] if q else []) + ([(r, 1)] if r else [])
        assert ph == want, (T, ph)
        assert max(k for k, _ in ph or [(0, 0)]) - min(k for k, _ in ph or [(0, 0)]) <= (1 if r >= 3 else 20)
        assert stencil.plan(8192, 8192, 1, 1, 0, T)["result_index"] == sum(n for _, n in ph) % 2
    assert stencil.plan(8192, 8192, 1, 1, 0, 20)["phases"] == [(20, 1)]  # the driver's --steps 20: one pass
    assert stencil.plan(8192, 8192, 1, 1, 0, 2400)["phases"] == [(20, 120)]  # bench defaults
    assert stencil.plan(8192, 8192, 2, 4, 3, 20)["phases"] == [(20, 1)]  # multi-rank interior: deep too
    assert stencil.plan(8192, 8192, 2, 4, 3, 2400)["phases"] == [(20, 120)]
    assert stencil.plan(79, 512, 1, 1, 0, 20)["phases"] == [(10, 2)]    # shorter than 4 x 20 rows
    assert stencil.plan(80, 512, 1, 1, 0, 20)["phases"] == [(20, 1)]
    assert stencil.plan(119, 512, 2, 2, 0, 20)["phases"] == [(10, 2)]   # interior (rows - 2K) under 4K
    assert stencil.plan(120, 512, 2, 2, 0, 20)["phases"] == [(20, 1)]


def test_plan_neighbours_follow_reference_rank_map():
    """rank = i_px * PY + i_py (stencil_smi.cpp:133-134); diagonals where both
    sides exist."""
    from smi_amd import stencil
    for PX, PY in [(1, 2), (2, 1), (2, 2), (2, 4), (3, 3)]:
        for r in range(PX * PY):
            ipx, ipy = divmod(r, PY)
            nb = stencil.plan(64, 64, PX, PY, r, 5)["neighbours"]
            at = lambda dx, dy: ((ipx + dx) * PY + ipy + dy  # noqa: E731
                                 if 0 <= ipx + dx < PX and 0 <= ipy + dy < PY else -1)
            assert nb == [at(-1, 0), at(1, 0), at(0, -1), at(0, 1), at(-1, -1), at(-1, 1), at(1, -1), at(1, 1)]


def test_plan_clips_k_to_the_tile():
    from smi_amd import stencil
    assert stencil.plan(10, 16, 2, 2, 0, 23)["phases"] == [(5, 3), (4, 2)]   # K clipped to 5, balanced
    assert stencil.plan(10, 16, 1, 1, 0, 23)["phases"] == [(12, 1), (11, 1)]  # single tile: no halo limit
    assert stencil.plan(4, 4, 1, 1, 0, 5)["phases"] == [(1, 5)]                # below 4 x 8: single steps
    assert stencil.plan(4, 8, 2, 2, 0, 5)["phases"] == [(2, 2), (1, 1)]


def test_plan_rejects_bad_arguments():
    from smi_amd import SMIError, stencil
    with pytest.raises(SMIError):
        stencil.plan(8, 6, 1, 1, 0, 3)      # y_local % 4
    with pytest.raises(SMIError):
        stencil.plan(8, 8, 2, 2, 4, 3)      # rank outside the grid
    with pytest.raises(SMIError):
        stencil.plan(8, 8, 1, 1, 0, -1)


def test_fusion_setting_drives_the_plan():
    from smi_amd import stencil
    old = stencil.get_fusion()
    try:
        stencil.set_fusion(8)
        assert stencil.plan(256, 256, 1, 1, 0, 20)["phases"] == [(7, 2), (6, 1)]
        stencil.set_fusion(2)
        assert stencil.plan(256, 256, 1, 1, 0, 7)["phases"] == [(2, 3), (1, 1)]
        stencil.set_fusion(1)
        assert stencil.plan(256, 256, 1, 1, 0, 7)["phases"] == [(1, 7)]
    finally:
        stencil.set_fusion(old["steps_per_pass"])


def test_band_settings_roundtrip_and_validate():
    """smi_stencil_set_bands: wave slots reserved for the band kernel + the
    exchange and the interior's rounds; -1 keeps a setting, out-of-range
    values are refused (host-only, no device needed)."""
    from smi_amd import stencil
    from smi_amd._lib import SMIError
    old = stencil.get_bands()
    assert old == dict(reserve_waves=0, interior_rounds=1)  # defaults
    try:
        stencil.set_bands(128, 2)
        assert stencil.get_bands() == dict(reserve_waves=128, interior_rounds=2)
        stencil.set_bands(-1, 3)
        assert stencil.get_bands() == dict(reserve_waves=128, interior_rounds=3)
        stencil.set_bands(0, -1)
        assert stencil.get_bands() == dict(reserve_waves=0, interior_rounds=3)
        with pytest.raises(SMIError):
            stencil.set_bands(65537, 1)
        with pytest.raises(SMIError):
            stencil.set_bands(0, 65)
        assert stencil.get_bands() == dict(reserve_waves=0, interior_rounds=3)
    finally:
        stencil.set_bands(old["reserve_waves"], old["interior_rounds"])


def test_band_kernel_setting_roundtrip_and_validate():
    """smi_stencil_set_band_kernel: 1 = the lean band kernel beside the
    interior (default), 0 = one wave per segment; -1 keeps it, anything else
    is refused."""
    from smi_amd import stencil
    from smi_amd._lib import SMIError
    old = stencil.get_band_kernel()
    assert old == 1  # default
    try:
        stencil.set_band_kernel(0)
        assert stencil.get_band_kernel() == 0
        stencil.set_band_kernel(-1)
        assert stencil.get_band_kernel() == 0
        with pytest.raises(SMIError):
            stencil.set_band_kernel(2)
        assert stencil.get_band_kernel() == 0
    finally:
        stencil.set_band_kernel(old)


def test_join_setting_roundtrip_and_validate():
    """smi_stencil_set_join: 1 = host-observed pass join (default), 0 = a
    device-side wait per pass; -1 keeps it, anything else is refused."""
    from smi_amd import stencil
    from smi_amd._lib import SMIError
    old = stencil.get_join()
    assert old == 1  # default
    try:
        stencil.set_join(0)
        assert stencil.get_join() == 0
        stencil.set_join(-1)
        assert stencil.get_join() == 0
        with pytest.raises(SMIError):
            stencil.set_join(2)
        assert stencil.get_join() == 0
    finally:
        stencil.set_join(old)


@pytest.mark.parametrize("waves", [1024, 2048, 3072])
def test_deep_geometry_every_block_holds_k_rows(waves):
    """sweepd_geometry (smi_stencil_deep_geometry, host only) over every K =
    13..20, every side mask and sweep rectangles from the 4K-row minimum up:
    it never fails on a rectangle sweepd_fits admits and every row block is
    at least K rows (the triangular prologue needs K rows per block) -- the
    balancing weights are dropped on short tiles.  Launch sizes of 1, 2 and
    3 resident waves per SIMD."""
    from smi_amd import stencil
    old = stencil.get_deep()
    stencil.set_deep(waves=waves)
    try:
        for k in range(13, 21):
            kc = 4 * ((k + 3) // 4)
            for mask in range(16):
                top, bot, left, right = (mask >> 0) & 1, (mask >> 1) & 1, (mask >> 2) & 1, (mask >> 3) & 1
                for rect in (4 * k, 4 * k + 1, 5 * k + 3, 8 * k, 300, 1000, 8192):
                    rows = rect + k * (top + bot)
                    for cols in (8, 64, 136, 264, 1028, 8192):
                        if cols - kc * (left + right) < 8:
                            continue
                        g = stencil.deep_geometry(rows, cols, k, mask)
                        assert g["min_block_rows"] >= k, (k, mask, rows, cols, g)
                        assert g["waves"] >= g["strips"] >= 1, (k, mask, rows, cols, g)
        with pytest.raises(Exception):
            stencil.deep_geometry(4 * 13 - 1, 264, 13, 0)  # shorter than 4K rows
        with pytest.raises(Exception):
            stencil.deep_geometry(8192, 8192, 12, 0)  # not a rotating-ring K
    finally:
        stencil.set_deep(old["ce16"], old["rev16"], old["waves"])


# ------------------------------------------------------ gloo, world_size 2 --
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _exchange_depth(dist, torch, tile, nb, k):
    """One depth-k exchange with the libsmi_amd neighbour map: k rows to the
    vertical neighbours, k columns to the horizontal ones, a k x k block to
    each diagonal one; returns the extended tile (padded only on sides that
    have a neighbour: global edges stay the grid's own edges)."""
    X, Y = tile.shape
    top, bottom, left, right, tl, tr, bl, br = nb
    parts = [(top, tile[:k]), (bottom, tile[X - k:]), (left, tile[:, :k]), (right, tile[:, Y - k:]),
             (tl, tile[:k, :k]), (tr, tile[:k, Y - k:]), (bl, tile[X - k:, :k]), (br, tile[X - k:, Y - k:])]
    reqs, recv = [], []
    for peer, data in parts:
        if peer < 0:
            recv.append(None)
            continue
        buf = torch.empty(data.shape)
        reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(data)), peer))
        reqs.append(dist.irecv(buf, peer))
        recv.append(buf)
    for r in reqs:
        r.wait()
    h = [None if b is None else b.numpy() for b in recv]
    pt, pb, pl, pr = (k if top >= 0 else 0), (k if bottom >= 0 else 0), (k if left >= 0 else 0), \
        (k if right >= 0 else 0)
    ext = np.zeros((X + pt + pb, Y + pl + pr), np.float32)
    ext[pt:pt + X, pl:pl + Y] = tile
    if h[0] is not None:
        ext[:pt, pl:pl + Y] = h[0]
    if h[1] is not None:
        ext[pt + X:, pl:pl + Y] = h[1]
    if h[2] is not None:
        ext[pt:pt + X, :pl] = h[2]
    if h[3] is not None:
        ext[pt:pt + X, pl + Y:] = h[3]
    if h[4] is not None:
        ext[:pt, :pl] = h[4]
    if h[5] is not None:
        ext[:pt, pl + Y:] = h[5]
    if h[6] is not None:
        ext[pt + X:, :pl] = h[6]
    if h[7] is not None:
        ext[pt + X:, pl + Y:] = h[7]
    return ext, pt, pl


def _worker(rank, world, port, PX, PY, T, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from smi_amd import stencil
        from smi_amd.comm import exchange_unique_id
        uid = exchange_unique_id(rank, world, dist.distributed_c10d._get_default_store(), key="t/uid")
        ids = [None] * world
        dist.all_gather_object(ids, uid)
        # the production bring-up itself: Comm.from_env exchanges a fresh id
        # through the same store and calls smi_init, which must fail loudly
        # here (no GPU: the product path has no CPU fallback)
        import smi_amd
        try:
            smi_amd.Comm.from_env(device=0)
            no_gpu_fails = False
        except smi_amd.SMIError:
            no_gpu_fails = True
        XL, YL = 24, 28
        g = o.init_uniform(XL * PX, YL * PY, seed=9)
        ipx, ipy = rank // PY, rank % PY
        tile = g[ipx * XL:(ipx + 1) * XL, ipy * YL:(ipy + 1) * YL].copy()
        plan = stencil.plan(XL, YL, PX, PY, rank, T)   # libsmi_amd's own schedule
        for k, passes in plan["phases"]:
            for _ in range(passes):
                ext, pt, pl = _exchange_depth(dist, torch, tile, plan["neighbours"], k)
                tile = o.stencil(ext, k)[pt:pt + XL, pl:pl + YL].copy()
        tiles = [None] * world
        dist.all_gather_object(tiles, tile)
        plans = [None] * world
        dist.all_gather_object(plans, plan["phases"])
        if rank == 0:
            got = stencil.combine_memory(tiles, PX, PY)
            q.put((all(i == ids[0] for i in ids) and len(ids[0]) == 128 and no_gpu_fails,
                   all(p == plans[0] for p in plans),
                   bool(np.array_equal(got.view(np.uint32), o.stencil(g, T).view(np.uint32)))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("pxpy,T", [((1, 2), 29), ((2, 1), 29), ((1, 2), 6), ((2, 2), 27)])
def test_gloo_world2_halo_protocol(pxpy, T):
    """world_size 2 (1x2, 2x1) and 4 (2x2: diagonal K x K corner blocks)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = pxpy[0] * pxpy[1]
    procs = [ctx.Process(target=_worker, args=(r, world, port, pxpy[0], pxpy[1], T, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    same_uid, same_plan, exact = q.get(timeout=5)
    assert same_uid, "RCCL unique id not shared through the store (or smi_init did not fail without a GPU)"
    assert same_plan, "ranks planned different phases"
    assert exact, "decomposed depth-K halo protocol differs from the single-grid oracle"
