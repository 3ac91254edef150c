"""gesummv parity on the GPU.

Contract: bit-exact vs the oracle's restatement of the row-streamed fold of
examples/kernels/gesummv_rank0.cl:53-203 (our build's order; the emulator's
FP contraction is not knowable here), and accepted by the reference host's
own check (rel. err < 1e-4, examples/host/gesummv_smi.cpp:40-46,299-313).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


# m spans: one chunk, odd chunk counts (a lone last tile), slab (64-chunk)
# boundaries +-1, several full slabs
@pytest.mark.parametrize("shape", [(1, 64), (5, 128), (17, 192), (128, 1024), (64, 4096), (3, 33 * 64),
                                   (7, 65 * 64), (9, 127 * 64), (4, 129 * 64), (6, 3 * 64 * 64)])
def test_gemv_rows_matches_oracle(gpu, oracle_mod, shape):
    from smi_amd import gesummv
    n, m = shape
    rng = np.random.default_rng(n * m)
    A = (rng.random((n, m), dtype=np.float32) * 2 - 1)
    B = (rng.random((n, m), dtype=np.float32) * 2 - 1)
    x = (rng.random(m, dtype=np.float32) * 2 - 1)
    want = oracle_mod.gesummv(A, B, x, 1.5, 0.5)
    got = gesummv.gemv_rows(torch.from_numpy(A).cuda(), torch.from_numpy(B).cuda(),
                            torch.from_numpy(x).cuda(), 1.5, 0.5).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_gemv_rows_strided_and_single_matrix(gpu, oracle_mod):
    """lda > m (a column window of a wider matrix) and the A-only form
    (rank 0 of the reference with beta = 0, gesummv_smi.cpp:224)."""
    from smi_amd import gesummv
    n, m, lda = 13, 130 * 64, 130 * 64 + 4
    rng = np.random.default_rng(5)
    W = rng.random((n, lda), dtype=np.float32) * 2 - 1
    x = rng.random(m, dtype=np.float32) * 2 - 1
    A = torch.from_numpy(W).cuda()[:, :m]
    got = gesummv.gemv_rows(A, A, torch.from_numpy(x).cuda(), 1.25, -0.75).cpu().numpy()
    want = oracle_mod.gesummv(W[:, :m], W[:, :m], x, 1.25, -0.75)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    got1 = gesummv.gemv_rows(A, None, torch.from_numpy(x).cuda(), 1.25, 0.0).cpu().numpy()
    want1 = oracle_mod.gesummv(W[:, :m], np.zeros((n, m), np.float32), x, 1.25, 0.0)
    assert np.array_equal(got1, want1)


def test_reference_pattern(gpu, oracle_mod):
    from smi_amd import gesummv
    n, m = 256, 512
    A = gesummv.reference_matrix(n, m)
    x = gesummv.reference_vector(m)
    got = gesummv.gemv_rows(torch.from_numpy(A).cuda(), torch.from_numpy(A).cuda(),
                            torch.from_numpy(x).cuda(), 2.0, 3.0).cpu().numpy()
    assert oracle_mod.gesummv_reference_check(got, A, A, x, 2.0, 3.0)
    assert np.array_equal(got, oracle_mod.gesummv(A, A, x, 2.0, 3.0))


@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
def test_distributed_gesummv(gpu, oracle_mod, nranks):
    from smi_amd import LocalGroup, gesummv
    n, m = 203, 640
    rng = np.random.default_rng(nranks)
    A = rng.random((n, m), dtype=np.float32)
    B = rng.random((n, m), dtype=np.float32)
    x = rng.random(m, dtype=np.float32)
    root = nranks - 1

    def fn(comm):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            r0, r1 = gesummv.row_range(n, comm.size, comm.rank)
            y = gesummv.gesummv(comm, torch.from_numpy(A[r0:r1].copy()).cuda(),
                                torch.from_numpy(B[r0:r1].copy()).cuda(), torch.from_numpy(x).cuda(),
                                n, 1.5, 0.5, root=root)
            s.synchronize()
            return None if y is None else y.cpu().numpy()

    got = LocalGroup(nranks).run(fn)[root]
    want = oracle_mod.gesummv(A, B, x, 1.5, 0.5)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
