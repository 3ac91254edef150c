"""C++ host programs on the C ABI (hosts/*.cpp): the reference's own host
programs restated without Python in the loop.

* hosts/stencil_smi_host.cpp -- examples/host/stencil_smi.cpp:126-413:
  grid, SplitMemory, one smi_init_local rank thread per tile,
  smi_stencil_run, CombineMemory, Reference() + the 1e-4 * mean check.
* hosts/reduce_benchmark.cpp -- microbenchmarks/host/reduce_benchmark.cpp:
  19-158 with the app of microbenchmarks/kernels/reduce.cl (every rank sends
  rank + 1; the root checks n(n+1)/2), bulk smi_reduce and the per-element
  SMI_Reduce API.

* hosts/broadcast_benchmark.cpp -- microbenchmarks/host/broadcast_benchmark.cpp:
  20-166 with broadcast.cl (the root sends 0..n-1, every other rank checks
  element i == i), bulk smi_bcast and the per-element SMI_Bcast API.
* hosts/gesummv_smi_host.cpp -- examples/host/gesummv_smi.cpp:48-351: the
  A = B = i, x = 1 pattern, smi_gesummv row-sharded, the rel. 1e-4 check.
* hosts/bandwidth_benchmark.cpp / latency_benchmark.cpp -- the point-to-point
  microbenchmarks (microbenchmarks/host/{bandwidth,latency}_benchmark.cpp with
  kernels/{bandwidth,latency}_{0,1}.cl): two ports of n doubles 0.1f + i, and
  an int ping-pong incremented on every round trip; element and bulk forms.
* hosts/kmeans_smi_host.cpp -- examples/host/kmeans_smi.cpp:41-311: the
  reference generator (libstdc++ minstd_rand0, seed 5) on rank 0, smi_bcast +
  smi_scatter, one smi_kmeans per rank; centroids against the committed
  golden fixtures and the oracle.

Every host runs its ranks either as threads of one process (in-process
group) or as one process per rank (--rank/--size/--uid, smi_init over RCCL,
hosts/host_rt.h) -- the one-process-per-GPU deployment of an 8-GPU node.
On a one-GPU box every rank process gets its own NCCL_HOSTID (RCCL refuses
two ranks on one device of one host), so the bytes move over RCCL's socket
transport, as in tests/test_rccl_multiproc_gpu.py.

The GPU tests run the binaries as child processes (never exec) and check the
stencil result bit for bit against the committed golden hash of BASELINE
config 1 and against the oracle.
"""
import hashlib
import json
import os
import signal
import subprocess
import time

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


# a launcher's variables select the hosts' one-process-per-rank mode
# (hosts/host_rt.h): the threads-mode runs start without them
_LAUNCHER_VARS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE",
                  "OMPI_COMM_WORLD_LOCAL_RANK", "PMI_RANK", "PMI_SIZE", "SLURM_PROCID", "SLURM_NTASKS")


def _clean_env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in _LAUNCHER_VARS}
    env.update(extra)
    return env


def _run(args, timeout=120):
    return subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=_clean_env())


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
                 [_exe("reduce_benchmark"), "-n", "16", "-r", "0", "-i", "1", "-p", "2"],
                 [_exe("broadcast_benchmark"), "-n", "16", "-r", "0", "-i", "1", "-p", "2"],
                 [_exe("gesummv_smi_host"), "-n", "64", "-m", "64", "-a", "1", "-c", "1", "-r", "1"],
                 [_exe("bandwidth_benchmark"), "-k", "1", "-r", "1", "-i", "1"],
                 [_exe("latency_benchmark"), "-n", "4", "-r", "1", "-i", "1"],
                 [_exe("kmeans_smi_host"), "64", "1", "-p", "2", "-q"]):
        r = _run(args)
        assert r.returncode == 2, r.stdout + r.stderr
        assert "no GPU visible" in r.stderr


def test_hosts_process_mode_fails_loudly_without_gpu(tmp_path):
    """The one-process-per-rank launch stops at its first C-ABI call too
    (rank 0's smi_get_unique_id) with exit code 2, and leaves no id file."""
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible: the GPU tests run the hosts")
    uid = tmp_path / "uid"
    r = _run([_exe("stencil_smi_host"), "256", "256", "1", "2", "32", "--rank", "0", "--size", "2", "--uid", str(uid)])
    assert r.returncode == 2, r.stdout + r.stderr
    assert "smi_get_unique_id" in r.stderr and not uid.exists()
    r = _run([_exe("stencil_smi_host"), "256", "256", "1", "2", "32", "--rank", "2", "--size", "2", "--uid", str(uid)])
    assert r.returncode == 1  # a malformed launch is a usage error


def test_hosts_take_ranks_from_a_launcher_environment(tmp_path):
    """Without --rank a launcher's environment (torchrun's RANK / WORLD_SIZE,
    Open MPI's OMPI_COMM_WORLD_*, PMI_*, SLURM_*) selects one process per
    rank: with no GPU, rank 0 stops at smi_get_unique_id (exit 2); a rank
    outside the job is a usage error (exit 1)."""
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible: the GPU tests run the hosts")
    base = _clean_env()
    args = [_exe("stencil_smi_host"), "256", "256", "1", "2", "32"]
    for envs in ({"RANK": "0", "WORLD_SIZE": "2", "MASTER_PORT": "29999"},
                 {"OMPI_COMM_WORLD_RANK": "0", "OMPI_COMM_WORLD_SIZE": "2"},
                 {"PMI_RANK": "0", "PMI_SIZE": "2"}):
        r = subprocess.run(args, env=dict(base, TMPDIR=str(tmp_path), **envs), capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 2 and "smi_get_unique_id" in r.stderr, (envs, r.stdout + r.stderr)
    r = subprocess.run(args, env=dict(base, RANK="3", WORLD_SIZE="2"), capture_output=True, text=True, timeout=120)
    assert r.returncode == 1, r.stdout + r.stderr


def _launch_ranks(args, world, tmp_path, timeout=240, stall=None):
    """One process per rank (--rank/--size/--uid), started with subprocess;
    every rank is killed once one fails or the time limit passes.  Returns
    (exit codes, outputs).  stall = (rank, every_s, for_s): that rank's
    process is stopped (SIGSTOP) for for_s every every_s seconds while the
    job runs -- a host descheduled at arbitrary points."""
    import torch
    ngpu = torch.cuda.device_count()  # does not initialise the GPU on this image
    uid = tmp_path / f"uid_{world}_{time.monotonic_ns()}"
    procs = []
    for r in range(world):
        env = _clean_env(HSA_ENABLE_IPC_MODE_LEGACY="0")
        if ngpu < world:
            env.update(NCCL_HOSTID=f"smi-host-test-{r}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
        procs.append(subprocess.Popen(args + ["--rank", str(r), "--size", str(world), "--uid", str(uid)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    t_end = time.monotonic() + timeout
    lines0 = []
    if stall:
        # stop the victim only once the runs are under way (rank 0 has printed
        # its first run time): a stop inside the HIP runtime's start-up makes
        # it find no device
        import threading
        reader = threading.Thread(target=lambda: lines0.extend(iter(procs[0].stdout.readline, "")), daemon=True)
        reader.start()
        while not any(ln.startswith("run ") for ln in lines0) and procs[0].poll() is None:
            if time.monotonic() > t_end:
                break
            time.sleep(0.002)
    t_stall = time.monotonic() + (stall[1] if stall else 0)
    while any(p.poll() is None for p in procs):
        failed = any(p.poll() not in (None, 0) for p in procs)
        if failed or time.monotonic() > t_end:
            for p in procs:
                if p.poll() is None:
                    p.kill()
            break
        if stall and time.monotonic() >= t_stall and procs[stall[0]].poll() is None:
            victim = procs[stall[0]]
            victim.send_signal(signal.SIGSTOP)
            time.sleep(stall[2])
            victim.send_signal(signal.SIGCONT)
            t_stall = time.monotonic() + stall[1]
        time.sleep(0.005 if stall else 0.05)
    if stall:
        reader.join(timeout=30)
        outs = ["".join(lines0)] + [p.communicate()[0] for p in procs[1:]]
        procs[0].wait()
    else:
        outs = [p.communicate()[0] for p in procs]
    return [p.returncode for p in procs], outs


def _log(rcs, outs):
    return "\n".join(f"--- rank {r} (rc {rc})\n{o[-3000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))


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


@pytest.mark.gpu
@pytest.mark.parametrize("pxpy", [(2, 2), (1, 2)])
def test_stencil_host_processes_config1_matches_golden(tmp_path, pxpy):
    """BASELINE config 1 through the C++ host with one process per rank over
    RCCL (smi_get_unique_id -> file -> smi_init; tiles scattered from and
    gathered to rank 0): the reference check passes on rank 0 and the result
    is bit-identical to the golden hash."""
    out = tmp_path / "res.f32"
    world = pxpy[0] * pxpy[1]
    rcs, outs = _launch_ranks([_exe("stencil_smi_host"), "256", "256", str(pxpy[0]), str(pxpy[1]), "32",
                               "--out", str(out)], world, tmp_path)
    assert all(rc == 0 for rc in rcs), _log(rcs, outs)
    assert "Successfully verified result." in outs[0]
    assert hashlib.sha256(out.read_bytes()).hexdigest() == _golden_config1()
    assert not list(tmp_path.glob("uid_*"))  # rank 0 removed the id file after smi_init


@pytest.mark.gpu
def test_stencil_host_processes_deep_passes_vs_oracle(tmp_path):
    """A 2x2 grid of 512x512 tiles in four rank processes, 40 steps = two
    K = 20 passes (rotating-ring interior, lean band kernel, the depth-20
    exchange over RCCL, the host-observed pass join): bit-exact vs the
    oracle, reference check passed."""
    import oracle
    out = tmp_path / "res.f32"
    rcs, outs = _launch_ranks([_exe("stencil_smi_host"), "1024", "1024", "2", "2", "40", "--init", "uniform",
                               "--repeat", "2", "--out", str(out)], 4, tmp_path)
    assert all(rc == 0 for rc in rcs), _log(rcs, outs)
    got = np.fromfile(out, dtype=np.float32).reshape(1024, 1024)
    # the host's uniform grid: std::mt19937(1234) + uniform_real_distribution
    # is not numpy's, so regenerate it from the host itself at T = 0
    out0 = tmp_path / "init.f32"
    r = _run([_exe("stencil_smi_host"), "1024", "1024", "1", "1", "0", "--init", "uniform", "--out", str(out0)])
    assert r.returncode == 0, r.stdout + r.stderr
    g0 = np.fromfile(out0, dtype=np.float32).reshape(1024, 1024)
    want = oracle.stencil(g0, 40)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
def test_stencil_host_processes_with_a_stopped_rank(tmp_path):
    """Rank 1's host is stopped (SIGSTOP) for 20 ms every 50 ms while two rank
    processes run 30 repeats of 400 steps (20 K = 20 passes) on 4096x4096
    tiles: the host-observed pass join (smi_stencil_run enqueues interior(t)
    only after seeing band(t-1) finish) must not depend on the host keeping
    up -- the result stays bit-exact vs the oracle.  The run times rank 0
    prints show what the stalls cost the job."""
    import oracle
    out = tmp_path / "res.f32"
    args = [_exe("stencil_smi_host"), "4096", "8192", "1", "2", "400", "--init", "uniform", "--repeat", "30",
            "--out", str(out)]
    rcs, outs = _launch_ranks(args, 2, tmp_path, stall=(1, 0.05, 0.02))
    assert all(rc == 0 for rc in rcs), _log(rcs, outs)
    runs = [float(ln.split()[2]) for ln in outs[0].splitlines() if ln.startswith("run ")]
    print("run times (s):", runs)
    assert len(runs) == 30
    print("stalled runs, median (s):", sorted(runs)[15])
    got = np.fromfile(out, dtype=np.float32).reshape(4096, 8192)
    out0 = tmp_path / "init.f32"
    r = _run([_exe("stencil_smi_host"), "4096", "8192", "1", "1", "0", "--init", "uniform", "--out", str(out0)])
    assert r.returncode == 0, r.stdout + r.stderr
    want = oracle.stencil(np.fromfile(out0, dtype=np.float32).reshape(4096, 8192), 400)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("world,mode,n", [(2, "bulk", 1 << 20), (4, "bulk", 4096), (2, "element", 256)])
def test_reduce_benchmark_processes_kat(tmp_path, world, mode, n):
    """reduce.cl's known answer with one process per rank over RCCL."""
    rcs, outs = _launch_ranks([_exe("reduce_benchmark"), "-n", str(n), "-r", "0", "-i", "3", "-m", mode],
                              world, tmp_path)
    assert all(rc == 0 for rc in rcs), _log(rcs, outs)
    assert outs[0].count("Result is Ok!") == 3 and "Conf interval 99" in outs[0]


@pytest.mark.gpu
@pytest.mark.parametrize("mode,n,ranks,root", [("bulk", 1 << 20, 4, 0), ("bulk", 1000, 3, 2),
                                               ("element", 512, 4, 1)])
def test_broadcast_benchmark_host_kat(tmp_path, mode, n, ranks, root):
    """broadcast.cl's check (element i arrives as i) on every non-root rank of
    every run, threads as ranks, and the harness's statistics file."""
    dat = tmp_path / "smi_broadcast.dat"
    r = _run([_exe("broadcast_benchmark"), "-n", str(n), "-r", str(root), "-i", "3", "-p", str(ranks),
              "-m", mode, "-o", str(dat)])
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("Result is Ok!") == 3 * (ranks - 1) and "Error" not in r.stdout
    assert "Average bandwidth (Gbit/s)" in r.stdout
    lines = dat.read_text().splitlines()
    assert lines[0].startswith("#SMI Broadcast") and len([ln for ln in lines if not ln.startswith("#")]) == 3


@pytest.mark.gpu
@pytest.mark.parametrize("world,mode,n", [(2, "bulk", 1 << 20), (4, "bulk", 100000), (2, "element", 256)])
def test_broadcast_benchmark_processes_kat(tmp_path, world, mode, n):
    """The same with one process per rank over RCCL."""
    rcs, outs = _launch_ranks([_exe("broadcast_benchmark"), "-n", str(n), "-r", "0", "-i", "3", "-m", mode],
                              world, tmp_path)
    assert all(rc == 0 for rc in rcs), _log(rcs, outs)
    assert sum(o.count("Result is Ok!") for o in outs) == 3 * (world - 1)


def _oracle_gesummv_pattern(n, m, alpha, beta):
    import oracle
    A = np.repeat(np.arange(n, dtype=np.float32)[:, None], m, axis=1)
    return oracle.gesummv(A, A, np.ones(m, dtype=np.float32), alpha, beta)


@pytest.mark.gpu
@pytest.mark.parametrize("ranks,n,m", [(2, 1024, 2048), (8, 4096, 8192), (3, 1000, 4096)])
def test_gesummv_host_reference_pattern(tmp_path, ranks, n, m):
    """gesummv_smi's own test (A = B = i, x = 1, rel. 1e-4 vs sgemv) through
    the C++ host, threads as ranks: "OK!!!", and y bit-identical to the
    oracle's restatement of the row fold."""
    y = tmp_path / "y.f32"
    r = _run([_exe("gesummv_smi_host"), "-n", str(n), "-m", str(m), "-a", "1.5", "-c", "0.5", "-r", "3",
              "-p", str(ranks), "-y", str(y)])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK!!!" in r.stdout
    got = np.fromfile(y, dtype=np.float32)
    assert np.array_equal(got.view(np.uint32), _oracle_gesummv_pattern(n, m, 1.5, 0.5).view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_gesummv_host_processes(tmp_path, world):
    """The same with one process per rank over RCCL (y chunks streamed to
    rank 0 over the transport)."""
    y = tmp_path / "y.f32"
    n, m = 2048, 4096
    rcs, outs = _launch_ranks([_exe("gesummv_smi_host"), "-n", str(n), "-m", str(m), "-a", "2", "-c", "-0.25",
                               "-r", "2", "-y", str(y)], world, tmp_path)
    assert all(rc == 0 for rc in rcs), _log(rcs, outs)
    assert "OK!!!" in outs[0]
    got = np.fromfile(y, dtype=np.float32)
    assert np.array_equal(got.view(np.uint32), _oracle_gesummv_pattern(n, m, 2.0, -0.25).view(np.uint32))


# ------------------------------------------------ BASELINE configs 3-5 as rank processes --
@pytest.mark.gpu
def test_config3_stencil_16384_processes(tmp_path):
    """BASELINE config 3 (16384^2 fp32 as 2x2 tiles of 8192^2, the halo
    exchange over RCCL) with one process per rank: two K = 20 passes,
    bit-exact vs the oracle and the reference check on rank 0."""
    import oracle
    out = tmp_path / "res.f32"
    rcs, outs = _launch_ranks([_exe("stencil_smi_host"), "16384", "16384", "2", "2", "40", "--init", "uniform",
                               "--out", str(out)], 4, tmp_path, timeout=400)
    assert all(rc == 0 for rc in rcs), _log(rcs, outs)
    assert "Successfully verified result." in outs[0]
    got = np.fromfile(out, dtype=np.float32).reshape(16384, 16384)
    out0 = tmp_path / "init.f32"
    r = _run([_exe("stencil_smi_host"), "16384", "16384", "1", "1", "0", "--init", "uniform", "--out", str(out0)])
    assert r.returncode == 0, r.stdout + r.stderr
    want = oracle.stencil(np.fromfile(out0, dtype=np.float32).reshape(16384, 16384), 40)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("host", ["reduce_benchmark", "broadcast_benchmark"])
def test_config4_256mib_processes(tmp_path, host):
    """BASELINE config 4 at its largest message (256 MiB of fp32) across four
    rank processes: the reduce.cl / broadcast.cl known answers on every
    element of every run."""
    rcs, outs = _launch_ranks([_exe(host), "-n", str(64 << 20), "-r", "0", "-i", "2"], 4, tmp_path, timeout=400)
    assert all(rc == 0 for rc in rcs), _log(rcs, outs)
    assert sum(o.count("Result is Ok!") for o in outs) == (2 if host == "reduce_benchmark" else 6)
    assert not any("Error" in o for o in outs)


@pytest.mark.gpu
def test_config5_gesummv_32768_8_processes(tmp_path):
    """BASELINE config 5 (gesummv 32768^2 fp32, rows sharded over 8 ranks,
    y chunks streamed to the root) with one process per rank: the
    reference's rel. 1e-4 check on every row, y bit-identical to the oracle
    on a sample of rows."""
    import oracle
    n = m = 32768
    y = tmp_path / "y.f32"
    rcs, outs = _launch_ranks([_exe("gesummv_smi_host"), "-n", str(n), "-m", str(m), "-a", "1.5", "-c", "0.5",
                               "-r", "2", "-y", str(y)], 8, tmp_path, timeout=400)
    assert all(rc == 0 for rc in rcs), _log(rcs, outs)
    assert "OK!!!" in outs[0]
    got = np.fromfile(y, dtype=np.float32)
    rows = np.array(sorted({0, 1, 4095, 4096, 16384, 32767} | set(range(7, n, 4099))))
    A = np.repeat(rows.astype(np.float32)[:, None], m, axis=1)
    want = oracle.gesummv(A, A, np.ones(m, dtype=np.float32), 1.5, 0.5)
    assert np.array_equal(got[rows].view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
def test_stencil_host_under_torchrun(tmp_path):
    """The C++ host launched like the reference's (mpirun -np N), here by
    torchrun --no-python: ranks from RANK / WORLD_SIZE, the id file named by
    MASTER_PORT, --fake-host for two ranks on one GPU.  BASELINE config 1 as
    1x2 ranks, bit-identical to the golden hash."""
    import socket
    import sys
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    out = tmp_path / "res.f32"
    env = _clean_env(TMPDIR=str(tmp_path), HSA_ENABLE_IPC_MODE_LEGACY="0", NCCL_SOCKET_IFNAME="lo",
                     NCCL_IB_DISABLE="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--no-python", "--nnodes", "1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port", str(port),
                        _exe("stencil_smi_host"), "256", "256", "1", "2", "32", "--fake-host", "--out", str(out)],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "Successfully verified result." in r.stdout
    assert hashlib.sha256(out.read_bytes()).hexdigest() == _golden_config1()


# ------------------------------------------------ point-to-point microbenchmarks --
@pytest.mark.gpu
@pytest.mark.parametrize("mode,kb,ranks,recv", [("bulk", 4096, 2, 1), ("bulk", 64, 3, 2), ("element", 256, 2, 1)])
def test_bandwidth_benchmark_host(tmp_path, mode, kb, ranks, recv):
    """bandwidth_0/1.cl: two ports of doubles 0.1f + i from rank 0 to the
    receiver, every element checked every run; threads as ranks."""
    dat = tmp_path / "bw.dat"
    r = _run([_exe("bandwidth_benchmark"), "-k", str(kb), "-r", str(recv), "-i", "3", "-p", str(ranks), "-m", mode,
              "-o", str(dat)])
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("Result is Ok!") == 3 and "Average bandwidth (Gbit/s)" in r.stdout
    assert dat.read_text().startswith("#SMI Bandwidth")


@pytest.mark.gpu
@pytest.mark.parametrize("mode,n,ranks,recv", [("element", 200, 2, 1), ("element", 50, 3, 2), ("bulk", 100, 2, 1)])
def test_latency_benchmark_host(tmp_path, mode, n, ranks, recv):
    """latency_0/1.cl: an int ping-pong incremented on every round trip,
    checked on rank 0 every run; threads as ranks."""
    r = _run([_exe("latency_benchmark"), "-n", str(n), "-r", str(recv), "-i", "3", "-p", str(ranks), "-m", mode])
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("Result is Ok!") == 3 and "One-way latency (usec)" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("host,args", [("bandwidth_benchmark", ["-k", "1024", "-r", "1", "-i", "3"]),
                                       ("bandwidth_benchmark", ["-k", "8", "-r", "1", "-i", "2", "-m", "element"]),
                                       ("latency_benchmark", ["-n", "100", "-r", "1", "-i", "3"]),
                                       ("latency_benchmark", ["-n", "50", "-r", "1", "-i", "2", "-m", "bulk"])])
def test_p2p_benchmarks_processes(tmp_path, host, args):
    """The same over RCCL with one process per rank."""
    rcs, outs = _launch_ranks([_exe(host)] + args, 2, tmp_path)
    assert all(rc == 0 for rc in rcs), _log(rcs, outs)
    assert sum(o.count("Result is Ok!") for o in outs) == int(args[args.index("-i") + 1])


# ------------------------------------------------------------------ kmeans_smi --
def _golden_kmeans():
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)["kmeans"]


def test_kmeans_host_usage_errors():
    """Usage errors exit 1 before any GPU work."""
    exe = _exe("kmeans_smi_host")
    assert _run([exe]).returncode == 1
    assert _run([exe, "64", "1", "-w", "5", "-p", "2"]).returncode == 1   # 64 dims % 5
    assert _run([exe, "63", "1", "-p", "2"]).returncode == 1              # 63 % 2 ranks


@pytest.mark.gpu
def test_kmeans_host_generator_overrun_stops():
    """A num_points for which the reference's inclusive
    uniform_int_distribution(0, num_points) picks one past the end of its
    input (kmeans_smi.cpp:141-146; 8 points): exit 1, nothing read."""
    r = _run([_exe("kmeans_smi_host"), "hardware", "8", "1", "-p", "1", "-q"])
    assert r.returncode == 1 and "past the end" in r.stderr, r.stdout + r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("case", [0, 1])
def test_kmeans_host_golden(tmp_path, case):
    """The committed kmeans fixtures (tests/golden/golden.json: 2048 points on
    8 ranks with W = 16, 10 iterations; 1536 points on 3 ranks with W = 1, 6
    iterations), ranks as threads: final centroids bit-identical."""
    g = _golden_kmeans()[case]
    out = tmp_path / "cen.f32"
    r = _run([_exe("kmeans_smi_host"), "emulator", str(g["num_points"]), str(g["iterations"]), "-k",
              str(g["clusters"]), "-d", str(g["dims"]), "-w", str(g["width"]), "-p", str(g["ranks"]), "-o", str(out)])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Final centroids:" in r.stdout and r.stdout.count("Finished in") == g["ranks"]
    assert hashlib.sha256(out.read_bytes()).hexdigest() == g["sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_kmeans_host_processes_vs_oracle(tmp_path, world):
    """One process per rank over RCCL: 4096 points of the reference generator,
    W = 16, 6 iterations, bit-identical to the oracle's rank-order program."""
    import oracle
    out = tmp_path / "cen.f32"
    rcs, outs = _launch_ranks([_exe("kmeans_smi_host"), "4096", "6", "-q", "-o", str(out)], world, tmp_path)
    assert all(rc == 0 for rc in rcs), _log(rcs, outs)
    _, pts, cen0 = oracle.kmeans_reference_data(4096, 8, 64)
    want = oracle.kmeans(pts, cen0, 6, ranks=world, width=16)
    got = np.fromfile(out, dtype=np.float32).reshape(want.shape)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
