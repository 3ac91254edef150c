#!/bin/bash
# Round-2: pipelined reduce/bcast, transport split, RCCL multi-process tests, configs at size, then all GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_collectives_gpu.py -x -q --timeout 200 --timeout-method thread > $O/coll.log 2>&1 || { echo "collectives failed"; tail -40 $O/coll.log; exit 1; }
tail -1 $O/coll.log
timeout -k 10 600 python -u -m pytest tests/test_rccl_multiproc_gpu.py -x -q -s --timeout 550 --timeout-method thread > $O/rccl.log 2>&1 || { echo "rccl failed"; tail -60 $O/rccl.log; exit 1; }
tail -1 $O/rccl.log
timeout -k 10 600 python -u -m pytest tests/test_configs_at_size_gpu.py -x -v --timeout 300 --timeout-method thread > $O/configs.log 2>&1 || { echo "configs failed"; tail -40 $O/configs.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/configs.log | tail -12
