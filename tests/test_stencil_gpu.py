"""Stencil parity on the GPU: HIP sweep (through the C ABI) vs the CPU oracle.

Contract: bit-exact fp32 against the device order 0.25*(((S+W)+E)+N) with
global-edge cells copied (examples/kernels/stencil_smi.cl:117-165), for every
tile shape, side mode, decomposition and tuning setting.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def run_steps(grid, T, **tune):
    from smi_amd import stencil
    if tune:
        old = stencil.get_tuning()
        stencil.set_tuning(**tune)
    try:
        a = torch.from_numpy(grid).cuda()
        b = torch.empty_like(a)
        for _ in range(T):
            stencil.step(a, b)
            a, b = b, a
        torch.cuda.synchronize()
        return a.cpu().numpy()
    finally:
        if tune:
            stencil.set_tuning(old["rows_per_wave"], old["rows_in_flight"], old["nontemporal"],
                               old["overlap"])


SHAPES = [(1, 4), (2, 4), (3, 8), (5, 12), (7, 260), (64, 64), (129, 260), (256, 256), (300, 1028),
          (1000, 516)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("init", ["edges", "uniform"])
def test_step_matches_oracle(gpu, oracle_mod, shape, init):
    X, Y = shape
    g = oracle_mod.init_edges(X, Y) if init == "edges" else oracle_mod.init_uniform(X, Y, seed=X * 31 + Y)
    for T in (1, 3):
        got = run_steps(g, T)
        want = oracle_mod.stencil(g, T)
        assert np.array_equal(bits(got), bits(want)), f"{shape} T={T}"


def test_config1_grid_256_t32(gpu, oracle_mod):
    """BASELINE config 1 problem (256x256, 32 steps) on one tile: bit-exact vs
    the oracle and accepted by the reference host check (stencil_smi.cpp:391-405)."""
    from smi_amd import stencil
    g = stencil.init_grid(256, 256)
    got = run_steps(g, 32)
    assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, 32)))
    assert oracle_mod.reference_check(got, oracle_mod.stencil(g, 32, order="host"))


@pytest.mark.parametrize("tune", [
    dict(rows_per_wave=1, rows_in_flight=1), dict(rows_per_wave=7, rows_in_flight=2),
    dict(rows_per_wave=64, rows_in_flight=8), dict(rows_per_wave=33, rows_in_flight=4, nontemporal=1),
    dict(rows_per_wave=256, rows_in_flight=8, nontemporal=1)])
def test_tuning_is_bit_neutral(gpu, oracle_mod, tune):
    g = oracle_mod.init_uniform(517, 1540, seed=7)
    assert np.array_equal(bits(run_steps(g, 2, **tune)), bits(oracle_mod.stencil(g, 2)))


def _ext_reference(oracle_mod, tile, halos, modes):
    """A HALO-mode step equals a full-grid step on the tile extended by its
    halo ring (corners never read); COPY sides are global edges."""
    X, Y = tile.shape
    ext = np.zeros((X + 2, Y + 2), dtype=np.float32)
    ext[1:-1, 1:-1] = tile
    ext[0, 1:-1] = halos[0]
    ext[-1, 1:-1] = halos[1]
    ext[1:-1, 0] = halos[2]
    ext[1:-1, -1] = halos[3]
    ref = oracle_mod.stencil(ext, 1)[1:-1, 1:-1].copy()
    # COPY sides keep their input cells
    if modes[0] == 0:
        ref[0, :] = tile[0, :]
    if modes[1] == 0:
        ref[-1, :] = tile[-1, :]
    if modes[2] == 0:
        ref[:, 0] = tile[:, 0]
    if modes[3] == 0:
        ref[:, -1] = tile[:, -1]
    return ref


@pytest.mark.parametrize("modes", [(1, 1, 1, 1), (0, 1, 0, 1), (1, 0, 1, 0), (0, 0, 1, 1), (1, 1, 0, 0)])
@pytest.mark.parametrize("shape", [(1, 4), (6, 8), (70, 516), (257, 1024)])
def test_halo_modes(gpu, oracle_mod, modes, shape):
    from smi_amd import stencil
    X, Y = shape
    rng = np.random.default_rng(X + Y)
    tile = rng.random((X, Y), dtype=np.float32)
    halos = [rng.random(Y, dtype=np.float32), rng.random(Y, dtype=np.float32),
             rng.random(X, dtype=np.float32), rng.random(X, dtype=np.float32)]
    want = _ext_reference(oracle_mod, tile, halos, modes)
    a = torch.from_numpy(tile).cuda()
    out = torch.full_like(a, -7.0)
    hd = [torch.from_numpy(h).cuda() if m == 1 else None for h, m in zip(halos, modes)]
    sl = torch.zeros(X, device="cuda")
    sr = torch.zeros(X, device="cuda")
    stencil.step(a, out, modes, hd, sl, sr)
    got = out.cpu().numpy()
    assert np.array_equal(bits(got), bits(want))
    assert np.array_equal(bits(sl.cpu().numpy()), bits(want[:, 0]))
    assert np.array_equal(bits(sr.cpu().numpy()), bits(want[:, -1]))


def test_skip_mode_leaves_cells(gpu, oracle_mod):
    from smi_amd import stencil
    X, Y = 40, 520
    tile = oracle_mod.init_uniform(X, Y, seed=3)
    halos = [torch.rand(Y, device="cuda"), torch.rand(Y, device="cuda"), torch.rand(X, device="cuda"),
             torch.rand(X, device="cuda")]
    a = torch.from_numpy(tile).cuda()
    out = torch.full_like(a, -7.0)
    stencil.step(a, out, (2, 2, 2, 2), halos)
    got = out.cpu().numpy()
    assert (got[0, :] == -7).all() and (got[-1, :] == -7).all()
    assert (got[:, 0] == -7).all() and (got[:, -1] == -7).all()
    ref = _ext_reference(oracle_mod, tile, [h.cpu().numpy() for h in halos], (1, 1, 1, 1))
    assert np.array_equal(bits(got[1:-1, 1:-1]), bits(ref[1:-1, 1:-1]))


def test_bad_arguments_raise(gpu):
    from smi_amd import SMIError, stencil
    a = torch.zeros((8, 6), device="cuda")  # y_local % 4 != 0
    with pytest.raises(SMIError):
        stencil.step(a, torch.empty_like(a))
    b = torch.zeros((8, 8), device="cuda")
    with pytest.raises(SMIError):
        stencil.step(b, b)  # in == out
    with pytest.raises(SMIError):
        stencil.step(b, torch.empty_like(b), (1, 0, 0, 0))  # HALO side without halo


def _decomposed_run(grid, T, PX, PY, overlap, priority=0, busy=False):
    from smi_amd import LocalGroup, stencil
    stencil.set_tuning(overlap=overlap)
    tiles = stencil.split_memory(grid, PX, PY)

    def rank_fn(comm):
        s = torch.cuda.Stream(priority=priority)
        with torch.cuda.stream(s):
            t = torch.from_numpy(tiles[comm.rank]).cuda()
            if busy:
                # the tile is produced by work still queued on the caller's
                # stream when the run is enqueued (t = t * 1 + 0 repeatedly)
                for _ in range(20):
                    t = torch.addcmul(torch.zeros_like(t), t, torch.ones_like(t))
            res = stencil.run(comm, t, T, PX, PY)
            s.synchronize()
            return res.cpu().numpy()

    out = LocalGroup(PX * PY).run(rank_fn)
    stencil.set_tuning(overlap=1)
    return stencil.combine_memory(out, PX, PY)


@pytest.mark.parametrize("overlap", [0, 1])
@pytest.mark.parametrize("pxpy", [(1, 1), (2, 1), (1, 2), (2, 2), (2, 4), (4, 2)])
def test_decomposed_matches_single(gpu, oracle_mod, pxpy, overlap):
    PX, PY = pxpy
    g = oracle_mod.init_uniform(64 * PX, 128 * PY, seed=PX * 10 + PY)
    got = _decomposed_run(g, 9, PX, PY, overlap)
    assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, 9)))


def test_config1_emulator_program(gpu, oracle_mod):
    """BASELINE config 1 exactly: 4 ranks (PX=PY=2), 256x256 fp32, 32 steps,
    reference init; bit-exact vs the rank-decomposed oracle and accepted by
    the reference host check."""
    from smi_amd import stencil
    g = stencil.init_grid(256, 256)
    got = _decomposed_run(g, 32, 2, 2, 1)
    assert np.array_equal(bits(got), bits(oracle_mod.stencil_decomposed(g, 32, 2, 2)))
    assert oracle_mod.reference_check(got, oracle_mod.stencil(g, 32, order="host"))


def test_zero_timesteps_and_tiny_tiles(gpu, oracle_mod):
    g = oracle_mod.init_uniform(8, 16, seed=1)
    got = _decomposed_run(g, 0, 2, 2, 1)
    assert np.array_equal(bits(got), bits(g))
    g = oracle_mod.init_uniform(2, 8, seed=2)   # 1-row x 4-col tiles
    got = _decomposed_run(g, 5, 2, 2, 1)
    assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, 5)))


def test_full_size_8192_sweep(gpu, oracle_mod):
    """BASELINE config 2 size (8192^2): two steps vs the threaded oracle."""
    g = oracle_mod.init_uniform(8192, 8192, seed=42)
    got = run_steps(g, 2)
    assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, 2)))


# ------------------------------------------------ two steps per pass (fused) --
def _run_fused(grid, T, PX=1, PY=1, overlap=1, ht2=0, u2=0, k=2, priority=0, busy=False):
    from smi_amd import stencil
    old = stencil.get_fusion()
    stencil.set_fusion(k)
    oldk = stencil.get_fusion()
    stencil.set_fusion(k, ht2, u2)
    try:
        return _decomposed_run(grid, T, PX, PY, overlap, priority, busy)
    finally:
        stencil.set_fusion(k, oldk["rows_per_wave"] or -1, oldk["rows_in_flight"])
        stencil.set_fusion(old["steps_per_pass"], old["rows_per_wave"], old["rows_in_flight"])


@pytest.mark.parametrize("shape", [(4, 8), (5, 8), (7, 260), (64, 64), (129, 260), (300, 1028), (1000, 516)])
def test_fused_single_tile(gpu, oracle_mod, shape):
    X, Y = shape
    g = oracle_mod.init_uniform(X, Y, seed=X + 3 * Y)
    for T in (1, 2, 3, 6):
        got = _run_fused(g, T)
        assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, T))), (shape, T)


@pytest.mark.parametrize("ht2,u2", [(1, 1), (3, 2), (16, 4), (64, 8), (7, 8)])
def test_fused_tuning_is_bit_neutral(gpu, oracle_mod, ht2, u2):
    g = oracle_mod.init_uniform(517, 1540, seed=9)
    got = _run_fused(g, 4, ht2=ht2, u2=u2)
    assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, 4)))


@pytest.mark.parametrize("overlap", [0, 1])
@pytest.mark.parametrize("pxpy", [(2, 1), (1, 2), (2, 2), (2, 4), (4, 2), (3, 3)])
def test_fused_decomposed(gpu, oracle_mod, pxpy, overlap):
    PX, PY = pxpy
    g = oracle_mod.init_uniform(64 * PX, 128 * PY, seed=PX * 7 + PY)
    for T in (5, 8):
        got = _run_fused(g, T, PX, PY, overlap)
        assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, T))), (pxpy, T)


def test_fused_tiny_and_fallback_tiles(gpu, oracle_mod):
    g = oracle_mod.init_uniform(8, 16, seed=21)     # 4x8 tiles at 2x2: smallest fused tile
    assert np.array_equal(bits(_run_fused(g, 7, 2, 2)), bits(oracle_mod.stencil(g, 7)))
    g = oracle_mod.init_uniform(6, 8, seed=22)      # 3x4 tiles: single-step fallback
    assert np.array_equal(bits(_run_fused(g, 7, 2, 2)), bits(oracle_mod.stencil(g, 7)))
    g = stencil_init = oracle_mod.init_edges(256, 256)   # config 1 through the fused path
    got = _run_fused(g, 32, 2, 2)
    assert np.array_equal(bits(got), bits(oracle_mod.stencil_decomposed(stencil_init, 32, 2, 2)))


def test_fused_full_size_8192(gpu, oracle_mod):
    g = oracle_mod.init_uniform(8192, 8192, seed=43)
    got = _run_fused(g, 4)
    assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, 4)))


# ------------------------------------------ K = 3..12 steps per pass (deep) --
@pytest.mark.parametrize("k", [3, 4, 5, 6, 7, 8, 9, 10, 11, 12])
@pytest.mark.parametrize("shape", [(1, 4), (2, 8), (5, 8), (9, 12), (17, 260), (64, 64), (129, 500),
                                   (300, 1028), (1000, 516)])
def test_deep_single_tile(gpu, oracle_mod, k, shape):
    X, Y = shape
    g = oracle_mod.init_uniform(X, Y, seed=X + 5 * Y + k)
    for T in (1, k - 1, k, k + 3, 2 * k + 1):
        got = _run_fused(g, T, k=k)
        assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, T))), (k, shape, T)


@pytest.mark.parametrize("k", [3, 4, 7, 8, 12])
@pytest.mark.parametrize("ht,u", [(1, 2), (5, 4), (16, 8), (32, 2), (100, 8)])
def test_deep_tuning_is_bit_neutral(gpu, oracle_mod, k, ht, u):
    g = oracle_mod.init_uniform(517, 1540, seed=11)
    got = _run_fused(g, 2 * k, ht2=ht, u2=u, k=k)
    assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, 2 * k)))


def test_deep_config1_and_edges(gpu, oracle_mod):
    g = oracle_mod.init_edges(256, 256)
    assert np.array_equal(bits(_run_fused(g, 32, k=4)), bits(oracle_mod.stencil(g, 32)))
    assert np.array_equal(bits(_run_fused(g, 32, k=8)), bits(oracle_mod.stencil(g, 32)))


def test_deep_full_size_8192(gpu, oracle_mod):
    g = oracle_mod.init_uniform(8192, 8192, seed=44)
    got = _run_fused(g, 8, k=4)
    assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, 8)))


def test_bench_config_full_size_default_plan(gpu, oracle_mod):
    """BASELINE config 2 exactly as bench.py runs it: 8192^2 fp32, the default
    K = 20 and automatic geometry, T = 12 (one K = 12 pass), 20 (one pass of
    the rotating-ring sweep: the driver's --steps 20) and 25 (13 + 12),
    bit-exact vs the oracle."""
    from smi_amd import LocalGroup, stencil
    assert stencil.get_fusion()["steps_per_pass"] == 20
    g = oracle_mod.init_uniform(8192, 8192, seed=1000)
    comm = LocalGroup(1).comm(0)
    want = g
    done = 0
    for T in (12, 20, 25):
        want = oracle_mod.stencil(want, T - done)
        done = T
        t = torch.from_numpy(g).cuda()
        res = stencil.run(comm, t, T, 1, 1)
        torch.cuda.synchronize()
        assert np.array_equal(bits(res.cpu().numpy()), bits(want)), T
        del t, res
    comm.finalize()


@pytest.mark.parametrize("T", list(range(1, 27)))
def test_remainder_plan_every_step_count(gpu, oracle_mod, T):
    """Every step count 1..26 under the default K = 12 (K-step passes, then
    one remainder pass of 3..11 steps, or a pair / single step)."""
    from smi_amd import stencil
    g = oracle_mod.init_uniform(203, 780, seed=T)
    ph = stencil.plan(203, 780, 1, 1, 0, T)["phases"]
    assert sum(k * n for k, n in ph) == T
    assert np.array_equal(bits(_run_fused(g, T, k=12)), bits(oracle_mod.stencil(g, T)))


@pytest.mark.parametrize("T", [5, 13, 14, 23, 31])
@pytest.mark.parametrize("pxpy", [(2, 2), (1, 3)])
def test_remainder_plan_decomposed(gpu, oracle_mod, T, pxpy):
    """Multi-rank runs whose plan ends in a remainder pass (depth-r halos from
    the same staging as depth 12) or a pair / single step."""
    PX, PY = pxpy
    g = oracle_mod.init_uniform(48 * PX, 64 * PY, seed=T + PX)
    for overlap in (0, 1):
        got = _run_fused(g, T, PX, PY, overlap, k=12)
        assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, T))), (T, pxpy, overlap)


def test_clipped_k_on_small_tiles(gpu, oracle_mod):
    """Tiles smaller than 24 x 24 in a multi-rank run clip K to half the
    smaller side (here 10 x 16 tiles: K = 5) instead of dropping to pairs."""
    from smi_amd import stencil
    assert stencil.plan(10, 16, 2, 2, 0, 23)["phases"] == [(5, 3), (4, 2)]
    g = oracle_mod.init_uniform(20, 32, seed=5)
    assert np.array_equal(bits(_run_fused(g, 23, 2, 2, k=12)), bits(oracle_mod.stencil(g, 23)))


@pytest.mark.parametrize("overlap", [0, 1])
@pytest.mark.parametrize("k", [3, 4, 8, 12])
@pytest.mark.parametrize("pxpy", [(2, 1), (1, 2), (2, 2), (2, 4), (3, 3)])
def test_deep_decomposed(gpu, oracle_mod, k, pxpy, overlap):
    """K-step passes with depth-K halos and K x K corner blocks, then the
    pair and single-step phases for the remainder (T = 2K+3)."""
    PX, PY = pxpy
    g = oracle_mod.init_uniform(72 * PX, 136 * PY, seed=PX * 11 + PY + k)
    for T in (k, 2 * k + 3):
        got = _run_fused(g, T, PX, PY, overlap, k=k)
        assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, T))), (k, pxpy, T)


@pytest.mark.parametrize("k", [3, 7, 10, 12])
@pytest.mark.parametrize("bands", [(0, 1), (0, 3), (64, 1), (500, 2), (65536, 1)])
def test_band_tuning_is_bit_neutral(gpu, oracle_mod, k, bands):
    """Wave slots the interior leaves to the band kernel and the exchange
    (none .. more than the GPU holds) and the interior's rounds of resident
    waves change scheduling only: a 3x3 decomposition (one interior rank with
    all eight neighbours) and the 2x4 of the 8-GPU run stay bit-exact, with
    and without overlap.  K = 7 and 10 have column bands (KC = 8, 12) wider
    than K."""
    from smi_amd import stencil
    reserve, rounds = bands
    old = stencil.get_bands()
    stencil.set_bands(reserve, rounds)
    try:
        assert stencil.get_bands() == dict(reserve_waves=reserve, interior_rounds=rounds)
        for PX, PY, X, Y in ((3, 3, 3 * 61, 3 * 140), (2, 4, 2 * 96, 4 * 128)):
            g = oracle_mod.init_uniform(X, Y, seed=k + reserve % 97 + PX)
            for T in (k, 2 * k + 1):
                for overlap in (1, 0):
                    got = _run_fused(g, T, PX, PY, overlap, k=k)
                    assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, T))), (k, bands, PX, PY, T, overlap)
    finally:
        stencil.set_bands(old["reserve_waves"], old["interior_rounds"])


@pytest.mark.parametrize("k", [4, 8, 12])
def test_deep_decomposed_small_tiles(gpu, oracle_mod, k):
    # exactly 2K x 2K tiles (smallest deep tile), ring blocks larger than tiles
    g = oracle_mod.init_uniform(4 * k, 6 * k, seed=k)
    assert np.array_equal(bits(_run_fused(g, 3 * k + 1, 2, 3, k=k)), bits(oracle_mod.stencil(g, 3 * k + 1)))
    # tiles below 2K clip K (or fall back to pairs/singles below 6 x 8)
    g = oracle_mod.init_uniform(2 * k - 4, 4 * k, seed=k + 1)
    assert np.array_equal(bits(_run_fused(g, 2 * k, 2, 2, k=k)), bits(oracle_mod.stencil(g, 2 * k)))
    # config 1 (256^2, 2x2, 32 steps) through the deep path
    g = oracle_mod.init_edges(256, 256)
    assert np.array_equal(bits(_run_fused(g, 32, 2, 2, k=k)), bits(oracle_mod.stencil_decomposed(g, 32, 2, 2)))


# ------------------------- K = 13..20 steps per pass (rotating-ring sweep) --
# stencild.h: single tiles and multi-rank interiors (beside bandk_kernel /
# bandl_kernel<K>); a sweep rectangle shorter than 4K rows clips K to 12.
RING_SHAPES = [(52, 8), (80, 260), (129, 500), (300, 1028), (1000, 516), (257, 2060), (96, 4)]


@pytest.mark.parametrize("k", list(range(13, 21)))
@pytest.mark.parametrize("shape", RING_SHAPES)
def test_ring_single_tile(gpu, oracle_mod, k, shape):
    """Every deep K on tiles with one strip (narrower than a window), edge
    strips on both sides, several interior strips, tall and short row blocks;
    T = k (one pass), k + 3 and 2k + 1 (balanced passes of mixed depth)."""
    from smi_amd import stencil
    X, Y = shape
    g = oracle_mod.init_uniform(X, Y, seed=X + 7 * Y + k)
    for T in (k, k + 3, 2 * k + 1):
        got = _run_fused(g, T, k=k)
        assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, T))), (k, shape, T)
    old = stencil.get_fusion()
    stencil.set_fusion(k)
    try:
        ph = stencil.plan(X, Y, 1, 1, 0, k)["phases"]
    finally:
        stencil.set_fusion(old["steps_per_pass"])
    if X >= 4 * k and Y >= 8:
        assert ph == [(k, 1)], ph   # one deep pass
    elif Y < 8:
        assert ph == [(1, k)], ph   # below 4 x 8: single steps
    else:
        assert max(kk for kk, _ in ph) <= 12 and sum(kk * n for kk, n in ph) == k, ph


@pytest.mark.parametrize("k", [14, 20])
@pytest.mark.parametrize("geom", [(0, 0, 0), (8, 8, 0), (16, 0, 512), (0, 12, 3000), (3, 4, 64)])
def test_ring_geometry_is_bit_neutral(gpu, oracle_mod, k, geom):
    """The edge-strip / bottom-block weights and the wave count of the
    rotating-ring sweep change scheduling only."""
    from smi_amd import stencil
    old = stencil.get_deep()
    stencil.set_deep(*geom)
    try:
        g = oracle_mod.init_uniform(611, 1236, seed=k + geom[0])
        got = _run_fused(g, 2 * k + 1, k=k)
        assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, 2 * k + 1))), (k, geom)
    finally:
        stencil.set_deep(old["ce16"], old["rev16"], old["waves"])


def test_ring_config1_edges_and_decomposed(gpu, oracle_mod):
    """The reference grid (0 interior, 1 on the edges) through K = 16 / 20,
    single tile and as the 2x2 emulator program (128^2 tiles: interiors of
    88 rows, deep enough for K = 20)."""
    g = oracle_mod.init_edges(256, 256)
    for k in (16, 20):
        assert np.array_equal(bits(_run_fused(g, 32, k=k)), bits(oracle_mod.stencil(g, 32)))
        assert np.array_equal(bits(_run_fused(g, 32, 2, 2, k=k)), bits(oracle_mod.stencil_decomposed(g, 32, 2, 2)))


@pytest.mark.parametrize("overlap", [0, 1])
@pytest.mark.parametrize("k", [13, 16, 20])
@pytest.mark.parametrize("pxpy", [(2, 1), (1, 2), (2, 2), (3, 3), (2, 4)])
def test_ring_decomposed(gpu, oracle_mod, k, pxpy, overlap):
    """Multi-rank K-step passes with the rotating-ring interior, the depth-K
    band kernel, depth-K halos and K x KC corner blocks (tiles 136 x 264: the
    interior keeps >= 4K rows), then the remainder phases (T = 2K + 3)."""
    from smi_amd import stencil
    PX, PY = pxpy
    g = oracle_mod.init_uniform(136 * PX, 264 * PY, seed=PX * 13 + PY + k)
    old = stencil.get_fusion()
    stencil.set_fusion(k)
    try:
        assert stencil.plan(136, 264, PX, PY, 0, k)["phases"] == [(k, 1)]
    finally:
        stencil.set_fusion(old["steps_per_pass"])
    for T in (k, 2 * k + 3):
        got = _run_fused(g, T, PX, PY, overlap, k=k)
        assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, T))), (k, pxpy, T)


@pytest.mark.parametrize("priority,busy", [(-1, False), (-1, True), (0, True)])
@pytest.mark.parametrize("k", [13, 20])
def test_ring_decomposed_caller_stream(gpu, oracle_mod, k, priority, busy):
    """The caller's stream at the highest priority (the interior runs on it)
    or at normal priority (the communicator's interior stream, joined to it),
    with the tile still being produced on it when the run is enqueued: the
    K-step passes' host-observed join and the stream joins are bit-neutral
    (2x2 and 2x4 ranks, T = 2K + 3)."""
    for PX, PY in ((2, 2), (2, 4)):
        g = oracle_mod.init_uniform(136 * PX, 264 * PY, seed=PX * 7 + PY + k)
        T = 2 * k + 3
        got = _run_fused(g, T, PX, PY, 1, k=k, priority=priority, busy=busy)
        assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, T))), (k, PX, PY, priority, busy)


@pytest.mark.parametrize("k", [16, 20])
@pytest.mark.parametrize("bands", [(0, 1), (4, 1), (64, 1), (500, 1)])
def test_ring_band_reserve_is_bit_neutral(gpu, oracle_mod, k, bands):
    """Wave slots reserved for the band kernel come off the rotating-ring
    interior's round of waves and cap the lean band kernel's grid (4: one
    workgroup whose four waves walk every segment in turn): scheduling
    only."""
    from smi_amd import stencil
    old = stencil.get_bands()
    stencil.set_bands(*bands)
    try:
        g = oracle_mod.init_uniform(3 * 140, 3 * 264, seed=k + bands[0] % 97)
        for overlap in (1, 0):
            got = _run_fused(g, k + 1, 3, 3, overlap, k=k)
            assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, k + 1))), (k, bands, overlap)
    finally:
        stencil.set_bands(old["reserve_waves"], old["interior_rounds"])


@pytest.mark.parametrize("k", [13, 14, 17, 20])
@pytest.mark.parametrize("pxpy", [(1, 2), (2, 1), (3, 3), (2, 4)])
def test_band_kernel_choice_is_bit_neutral(gpu, oracle_mod, k, pxpy):
    """The lean band kernel (bandl_kernel: KS = ceil(K/7) staged walks through
    LDS, <= 64 VGPRs, one workgroup per CU) and the one-wave-per-segment
    kernel (bandk_kernel) give the same bits, both equal to the oracle;
    global edges on every side of some rank (the copy rule inside the band
    walks), tiles 137 x 268 (ragged band segments)."""
    from smi_amd import stencil
    PX, PY = pxpy
    g = oracle_mod.init_uniform(137 * PX, 268 * PY, seed=k * 7 + PX * 3 + PY)
    want = bits(oracle_mod.stencil(g, k + 2))
    old = stencil.get_band_kernel()
    try:
        for lean in (1, 0):
            stencil.set_band_kernel(lean)
            got = _run_fused(g, k + 2, PX, PY, 1, k=k)
            assert np.array_equal(bits(got), want), (k, pxpy, lean)
    finally:
        stencil.set_band_kernel(old)


@pytest.mark.parametrize("k,pxpy,steps", [(20, (2, 2), 62), (13, (1, 3), 29), (12, (3, 1), 37)])
def test_join_mode_is_bit_neutral(gpu, oracle_mod, k, pxpy, steps):
    """smi_stencil_set_join: the host-observed pass join (1, default) and the
    device-side stream wait per pass (0) give the same bits, both equal to
    the oracle -- several K-step passes plus the remainder phases, so that
    both joins are crossed many times."""
    from smi_amd import stencil
    PX, PY = pxpy
    g = oracle_mod.init_uniform(200 * PX, 264 * PY, seed=k * 11 + PX)
    want = bits(oracle_mod.stencil(g, steps))
    old = stencil.get_join()
    try:
        for join in (1, 0):
            stencil.set_join(join)
            got = _run_fused(g, steps, PX, PY, 1, k=k)
            assert np.array_equal(bits(got), want), (k, pxpy, join)
    finally:
        stencil.set_join(old)


def test_ring_full_size_8192_driver_config(gpu, oracle_mod):
    """BASELINE config 2 at the driver's --steps 20 with K = 20: one pass of
    the rotating-ring sweep over 8192^2, bit-exact vs the oracle."""
    g = oracle_mod.init_uniform(8192, 8192, seed=1000)
    got = _run_fused(g, 20, k=20)
    assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, 20)))


# ------------------------------------------ special values through every path --
def _special_grid(X, Y, seed):
    """Uniform grid salted with the values IEEE fp32 treats specially: signed
    zeros, subnormals, the largest finite values, infinities and NaN."""
    rng = np.random.default_rng(seed)
    g = (rng.random((X, Y), dtype=np.float32) * 2 - 1).astype(np.float32)
    salt = np.array([0.0, -0.0, 1e-40, -1e-40, 1.4e-45, 1.17549435e-38, 3.4e38, -3.4e38],
                    dtype=np.float32)
    idx = rng.integers(0, X * Y, size=X * Y // 7)
    g.reshape(-1)[idx] = salt[rng.integers(0, len(salt), size=len(idx))]
    # a patch of tiny values whose averages go subnormal and back
    g[X // 3:X // 3 + 5, Y // 4:Y // 4 + 40] = np.float32(3e-38)
    # a few isolated non-finite cells (they spread one cell per step), one on
    # a global edge, one next to a tile boundary of a 2x2 decomposition
    for (r, c), v in zip([(5, 7), (X - 1, Y // 3), (X // 2 - 1, Y // 2), (X - 9, Y - 3)],
                         [np.nan, np.inf, -np.inf, np.nan]):
        g[r, c] = v
    return g


def _same(a, b):
    """Bit-identical, except that any NaN matches any NaN (payload propagation
    is not part of the reference's contract)."""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(bits(np.where(na, 0, a)), bits(np.where(nb, 0, b)))


@pytest.mark.parametrize("k", [1, 2, 4, 12, 16, 20])
@pytest.mark.parametrize("pxpy", [(1, 1), (2, 2)])
def test_special_values_bit_exact(gpu, oracle_mod, k, pxpy):
    PX, PY = pxpy
    g = _special_grid(96 * PX, 264 * PY, seed=k + 7 * PX)
    for T in (1, k + 1, 2 * k + 3):
        got = _run_fused(g, T, PX, PY, k=k)
        assert _same(got, oracle_mod.stencil(g, T)), (k, pxpy, T)


def test_special_values_single_steps(gpu, oracle_mod):
    g = _special_grid(70, 132, seed=3)
    assert _same(run_steps(g, 5), oracle_mod.stencil(g, 5))


# ------------------------------------- the K-step sweep's scaled-level guard --
def _guard_grid(X, Y, seed):
    """Uniform [0,1) grid with (a) cells at the edges of the scaled walk's
    range -- +-2^-100 and the largest float below 2^101, which it accepts --
    including a patch of +-2^-100(1 + j 2^-23) whose cancellations drive the
    levels down to multiples of 2^-147, and (b) a few isolated cells outside
    it (below 2^-100, subnormal, above 2^101), so that only the waves whose
    cones hold them walk their blocks again with the exact arithmetic."""
    rng = np.random.default_rng(seed)
    g = rng.random((X, Y), dtype=np.float32)
    lo = np.float32(2.0 ** -100)
    hi = np.nextafter(np.float32(2.0 ** 101), np.float32(0))
    r0, c0 = X // 5, Y // 6
    j = np.arange(64 * 48, dtype=np.float32).reshape(64, 48)
    sgn = np.where((j.astype(np.int64) % 2) == 0, 1, -1).astype(np.float32)
    g[r0:r0 + 64, c0:c0 + 48] = sgn * lo * (np.float32(1) + (j % 5) * np.float32(2.0 ** -23))
    g[X // 2, Y // 2] = hi
    g[X // 2 + 3, Y // 2 - 7] = -hi
    g[3 * X // 4, Y // 3] = lo
    for (r, c), v in zip([(X // 8, 7 * Y // 8), (7 * X // 8, Y // 8), (X - 20, Y - 300), (40, Y // 2)],
                         [1e-35, 1e-40, 3e30, -np.float32(2.0 ** 101)]):
        g[r, c] = v
    return g


@pytest.mark.parametrize("pxpy", [(1, 1), (2, 2)])
def test_scaled_guard_mixed_blocks(gpu, oracle_mod, pxpy):
    PX, PY = pxpy
    g = _guard_grid(1536, 2048, seed=11 + PX)
    for T in (12, 27):
        got = _run_fused(g, T, PX, PY, k=12)
        assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, T))), (pxpy, T)


@pytest.mark.parametrize("k", [3, 7, 12, 13, 16, 20])
def test_scaled_guard_every_k(gpu, oracle_mod, k):
    g = _guard_grid(700, 1028, seed=k)
    assert np.array_equal(bits(_run_fused(g, 2 * k + 1, k=k)), bits(oracle_mod.stencil(g, 2 * k + 1)))


@pytest.mark.parametrize("seed", range(10))
def test_scaled_guard_fuzz(gpu, oracle_mod, seed):
    """Random tiles whose magnitudes span 2^-135 .. 2^110 with mixed signs and
    zeros, in patches, so that within one pass some waves stay in the scaled
    range and others re-walk their blocks exactly; every K, bit-exact."""
    rng = np.random.default_rng(100 + seed)
    X, Y = int(rng.integers(60, 400)), 4 * int(rng.integers(20, 200))
    k = int(rng.integers(3, 21))
    g = rng.random((X, Y), dtype=np.float32)
    for _ in range(int(rng.integers(1, 6))):  # patches of scaled magnitudes
        r0, c0 = int(rng.integers(0, X)), int(rng.integers(0, Y))
        h, w = int(rng.integers(1, 40)), int(rng.integers(1, 80))
        e = rng.integers(-135, 111, size=(min(h, X - r0), min(w, Y - c0)))
        sgn = rng.choice(np.array([-1.0, 1.0, 0.0], np.float32), size=e.shape, p=[0.45, 0.45, 0.1])
        g[r0:r0 + h, c0:c0 + w] = (sgn * np.ldexp(rng.random(e.shape) + 0.5, e)).astype(np.float32)
    T = int(rng.integers(k, 3 * k + 2))
    assert np.array_equal(bits(_run_fused(g, T, k=k)), bits(oracle_mod.stencil(g, T))), (X, Y, k, T)


@pytest.mark.parametrize("k", [13, 16, 20])
@pytest.mark.parametrize("pxpy", [(2, 2), (1, 3), (3, 1)])
def test_band_special_values(gpu, oracle_mod, k, pxpy):
    """Decomposed K >= 13 passes (the lean band kernel beside the rotating-ring
    interior, whose waves walk scaled levels under their input guard) on
    tiles salted with signed zeros, subnormals, the largest finite values,
    infinities and NaN, which also reach the bands through the halos:
    bit-exact (NaN payloads aside) vs the oracle."""
    PX, PY = pxpy
    g = _special_grid(6 * k + 20 * PX, 268 * PY, seed=k * 5 + PX)
    for T in (k, 2 * k + 3):
        got = _run_fused(g, T, PX, PY, k=k)
        assert _same(got, oracle_mod.stencil(g, T)), (k, pxpy, T)


@pytest.mark.parametrize("seed", range(8))
def test_band_scaled_guard_fuzz(gpu, oracle_mod, seed):
    """Decomposed tiles with patches of magnitudes 2^-135 .. 2^110 (mixed
    signs, zeros) straddling the internal tile boundaries -- the band
    kernel's inputs and the halos -- so that within one pass some interior
    waves pass the scaled-level guard and others walk exactly next to the
    band kernel's exact walks; K = 13..20, bit-exact vs the oracle."""
    rng = np.random.default_rng(500 + seed)
    PX, PY = [(2, 2), (1, 2), (2, 1), (3, 2), (2, 3), (1, 3), (3, 1), (2, 2)][seed]
    k = int(rng.integers(13, 21))
    xl = 6 * k + int(rng.integers(0, 60))
    yl = 4 * int(rng.integers(40, 90))
    X, Y = xl * PX, yl * PY
    g = rng.random((X, Y), dtype=np.float32)
    bounds = [(r, None) for r in range(xl, X, xl)] + [(None, c) for c in range(yl, Y, yl)]
    for _ in range(int(rng.integers(3, 8))):
        br, bc = bounds[int(rng.integers(0, len(bounds)))]
        r0 = (br - int(rng.integers(0, 2 * k))) if br is not None else int(rng.integers(0, X - 8))
        c0 = (bc - int(rng.integers(0, 2 * k))) if bc is not None else int(rng.integers(0, Y - 8))
        r0, c0 = max(r0, 0), max(c0, 0)
        h, w = int(rng.integers(1, 3 * k)), int(rng.integers(1, 3 * k))
        e = rng.integers(-135, 111, size=(min(h, X - r0), min(w, Y - c0)))
        sgn = rng.choice(np.array([-1.0, 1.0, 0.0], np.float32), size=e.shape, p=[0.45, 0.45, 0.1])
        g[r0:r0 + h, c0:c0 + w] = (sgn * np.ldexp(rng.random(e.shape) + 0.5, e)).astype(np.float32)
    T = int(rng.integers(k, 2 * k + 3))
    got = _run_fused(g, T, PX, PY, k=k)
    assert np.array_equal(bits(got), bits(oracle_mod.stencil(g, T))), (PX, PY, xl, yl, k, T)


def test_profiling_entries_distinct(gpu, oracle_mod):
    """smi_prof_list counts distinct (kernel, tag) pairs, also for the
    max_entries = 0 size query profiling.entries() starts with: a 41-step
    run (passes of 11 + 10 + 10 + 10 steps) records four launches and lists
    two pairs."""
    import ctypes
    from smi_amd import LocalGroup, _lib, profiling, stencil
    comm = LocalGroup(1).comm(0)
    t = torch.from_numpy(oracle_mod.init_uniform(256, 512, seed=3)).cuda()
    profiling.reset()
    profiling.enable(True)
    old = stencil.get_fusion()
    stencil.set_fusion(12)
    try:
        stencil.run(comm, t, 3 * 12 + 5, 1, 1)
    finally:
        stencil.set_fusion(old["steps_per_pass"])
    torch.cuda.synchronize()
    profiling.enable(False)
    n = ctypes.c_int()
    _lib.call("smi_prof_list", None, None, 0, ctypes.byref(n))
    ents = profiling.entries()
    assert n.value == len(ents) == len(set(ents)), ents
    assert sorted(ents) == [(profiling.SWEEPK, 10), (profiling.SWEEPK, 11)], ents
    assert profiling.read_tag(profiling.SWEEPK, 10)[1] == 3
    profiling.reset()
    comm.finalize()
