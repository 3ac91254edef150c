"""C++ host programs on the C ABI (hosts/*.cpp): the reference's own host
programs restated without Python in the loop.

* hosts/stencil_smi_host.cpp -- examples/host/stencil_smi.cpp:126-413:
  grid, SplitMemory, one smi_init_local rank thread per tile,
  smi_stencil_run, CombineMemory, Reference() + the 1e-4 * mean check.
* hosts/reduce_benchmark.cpp -- microbenchmarks/host/reduce_benchmark.cpp:
  19-158 with the app of microbenchmarks/kernels/reduce.cl (every rank sends
  rank + 1; the root checks n(n+1)/2), bulk smi_reduce and the per-element
  SMI_Reduce API.

The GPU tests run the binaries as child processes (never exec) and check the
stencil result bit for bit against the committed golden hash of BASELINE
config 1 and against the oracle.
"""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "hosts", "_build")
GOLDEN = os.path.join(ROOT, "tests", "golden", "golden.json")


def _exe(name):
    path = os.path.join(BIN, name)
    if not os.path.exists(path):
        pytest.fail(f"{path} missing: build with python smi_amd/build.py --hosts (or __graft_entry__.build())")
    return path


def _run(args, timeout=120):
    return subprocess.run(args, capture_output=True, text=True, timeout=timeout)


def test_hosts_build_and_fail_loudly_without_gpu():
    """On the build host: both hosts compile against include/ + libsmi_amd.so
    and, with no GPU, stop at the first C-ABI call with SMI_ERR_NO_DEVICE's
    text and exit code 2 (no silent fallback)."""
    import torch
    from smi_amd import build
    build.build_hosts()
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible: the GPU tests run the hosts")
    for args in ([_exe("stencil_smi_host"), "256", "256", "2", "2", "32"],
                 [_exe("reduce_benchmark"), "-n", "16", "-r", "0", "-i", "1", "-p", "2"]):
        r = _run(args)
        assert r.returncode == 2, r.stdout + r.stderr
        assert "no GPU visible" in r.stderr


def _golden_config1():
    with open(GOLDEN) as f:
        gold = json.load(f)
    return next(c["sha256"] for c in gold["stencil"]
                if c["init"] == "edges" and (c["X"], c["Y"], c["T"]) == (256, 256, 32) and c.get("PX") == 2)


@pytest.mark.gpu
@pytest.mark.parametrize("pxpy", [(2, 2), (1, 1), (1, 4)])
def test_stencil_host_config1_matches_golden(tmp_path, pxpy):
    """BASELINE config 1 (256^2, 32 steps, reference init) through the C++
    host: the reference's own acceptance check passes (exit 0, "Successfully
    verified result.") and the result is bit-identical to the committed
    golden hash of the rank-decomposed emulator program."""
    out = tmp_path / "res.f32"
    r = _run([_exe("stencil_smi_host"), "256", "256", str(pxpy[0]), str(pxpy[1]), "32", "--out", str(out)])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Successfully verified result." in r.stdout
    assert hashlib.sha256(out.read_bytes()).hexdigest() == _golden_config1()


@pytest.mark.gpu
def test_stencil_host_deep_passes_vs_oracle(tmp_path):
    """A tile big enough for the rotating-ring sweep and the lean band kernel
    (2x4 ranks of 512x512, 40 steps = two K = 20 passes): bit-exact vs the
    oracle's rank-decomposed program, reference check passed."""
    import oracle
    out = tmp_path / "res.f32"
    r = _run([_exe("stencil_smi_host"), "1024", "2048", "2", "4", "40", "--out", str(out)])
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.fromfile(out, dtype=np.float32).reshape(1024, 2048)
    want = oracle.stencil(oracle.init_edges(1024, 2048), 40)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("mode,n,ranks,runs", [("bulk", 1 << 20, 4, 5), ("bulk", 4096, 8, 3),
                                               ("element", 512, 4, 2)])
def test_reduce_benchmark_host_kat(tmp_path, mode, n, ranks, runs):
    """reduce.cl's known answer (rank + 1 from every rank, n(n+1)/2 on the
    root) on every element of every run, and the reference harness's
    statistics file."""
    dat = tmp_path / "smi_reduce.dat"
    r = _run([_exe("reduce_benchmark"), "-n", str(n), "-r", str(ranks - 1), "-i", str(runs), "-p", str(ranks),
              "-m", mode, "-o", str(dat)])
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("Result is Ok!") == runs
    assert "Conf interval 99" in r.stdout
    lines = dat.read_text().splitlines()
    assert lines[0].startswith("#SMI Reduce") and len([ln for ln in lines if not ln.startswith("#")]) == runs
