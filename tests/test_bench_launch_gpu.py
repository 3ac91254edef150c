"""bench.py launches its own ranks (reference: `mpirun -np 8
./stencil_smi_host`, README.md:96): `bench.py --gpus 2` with no WORLD_SIZE
starts two child processes, and the parent prints rank 0's one JSON line.
On a one-GPU box --fake-host puts both ranks on GPU 0 with their own
NCCL_HOSTID (RCCL over sockets): the numbers are meaningless, the launch,
the halo exchange over the production RCCL transport and the line are not.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_self_launch_two_ranks(gpu):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--fake-host", "--steps", "24",
                        "--warmup", "2", "--no-aux", "--warmup-ms", "5", "--tile", "2048", "--launch-timeout", "150"],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=200)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 24 and d["value"] > 0
    assert d["config"]["decomposition"] == [1, 2] and d["config"]["fake_host"]
    assert d["config"]["launch"].startswith("self")
    assert d["roofline"]["kernels"], d["roofline"]
    # repetition statistics of the timed plan (max over ranks per run)
    r = d["repeats"]
    assert r["runs"] >= 5 and 0 < r["min"] <= r["median"] <= r["max"] and r["stddev"] >= 0, r
    # the timed plan re-run from the seeded inputs and checked per rank on its
    # light cone against the oracle, verdict agreed by both ranks
    p = d["parity"]
    assert p["checked"] and p["bit_exact"] and p["mismatches"] == 0, p
    assert p["cells"] == 2 * 2048 * 2048 and p["steps"] == 24 and p["same_plan_as_timed"], p
