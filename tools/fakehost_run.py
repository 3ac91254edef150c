#!/usr/bin/env python3
"""Run a script as one rank of a multi-process RCCL job on a ONE-GPU box.

RCCL refuses two ranks on the same device of one host ("Duplicate GPU
detected"), so each rank gets its own NCCL_HOSTID; RCCL then carries the
bytes over its socket transport on loopback.  Functional rehearsal of the
multi-process path only -- timings are meaningless.  Launch with
torch.distributed.run:  ... tools/fakehost_run.py bench.py --gpus 2 ...
"""
import os
import runpy
import sys

os.environ["NCCL_HOSTID"] = f"smi-fakehost-{os.environ.get('RANK', '0')}"
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
os.environ.setdefault("NCCL_IB_DISABLE", "1")
# every rank maps to the one visible GPU
os.environ["LOCAL_RANK"] = "0"
script = sys.argv[1]
sys.argv = sys.argv[1:]
sys.path.insert(0, os.path.dirname(os.path.abspath(script)))
runpy.run_path(script, run_name="__main__")
