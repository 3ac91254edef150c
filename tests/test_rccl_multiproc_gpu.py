"""The production RCCL transport under pytest: 2 and 4 fresh child processes
(tests/rccl_worker.py), one rank each, through smi_init -- bulk reduce/bcast
(incl. pipelined pieces), p2p, scatter/gather, gesummv, the decomposed stencil
(K = 1, 2, 12, overlap on and off) and the element-granular channels, every
case bit-exact vs the oracle.  The reference runs its known-answer tests the
same way, one process per rank (test/CMakeLists.txt:48-88, mpirun -np 8).

On a one-GPU box every child gets its own NCCL_HOSTID in its environment
before it starts (RCCL refuses two ranks on one device of one host), so the
bytes move over RCCL's socket transport; on a multi-GPU node each rank takes
its own device and RCCL picks xGMI.  The parent never touches the GPU
itself and never execs: the children are started with subprocess and killed
if they outlive the time limit.
"""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(world, timeout=240):
    import torch
    ngpu = torch.cuda.device_count()  # does not initialise the GPU on this image
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ)
        env.update(RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r % max(1, ngpu)),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        if ngpu < world:
            env.update(NCCL_HOSTID=f"smi-test-host-{r}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "rccl_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs, rcs = [], []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            out, _ = p.communicate()
            out += "\n<killed: time limit>"
        outs.append(out)
        rcs.append(p.returncode)
    return rcs, outs


@pytest.mark.parametrize("world", [2, 4])
def test_rccl_multiprocess_parity(gpu, world):
    rcs, outs = _launch(world)
    log = "\n".join(f"--- rank {r} (rc {rc})\n{o[-4000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    print(log)
    assert all(rc == 0 for rc in rcs), log
    assert "RCCL MULTIPROC PASS" in outs[0], log
    cases = sum(o.count(" CASE ") for o in outs)
    assert cases >= 30 and not any("MISMATCH" in o for o in outs), log
