#!/bin/bash
# Phase-end join on the host too: rehearsal, real RCCL, caller's stream at
# normal (library interior stream) and highest priority, 20 and 60 passes,
# alternating; then the multi-rank stencil GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$1; mkdir -p $O
step() { echo "=== $1"; shift; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; exit $rc; fi; }
step warm timeout -k 10 300 python -u -c 'print("importing torch", flush=True); import torch; torch.zeros(1).cuda(); print("warm", flush=True)'
G="REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_LEAN=1 REHEARSAL_OVERLAP=1 REHEARSAL_PROF=0 REHEARSAL_TRANSPORT=rccl"
for r in 1 2; do
  for spec in normal:REHEARSAL_PASSES=20 high:REHEARSAL_PASSES=20,REH_STREAM_PRIO=high normal_p60:REHEARSAL_PASSES=60; do
    name=${spec%%:*}; envs=$(echo ${spec#*:} | tr ',' ' ')
    step reh_$name bash -c "env $G $envs timeout -k 10 240 python -u tools/rehearsal.py 8192 20 >> $O/reh_$name.jsonl 2>> $O/reh_$name.err"
  done
done
python3 - $O <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/reh_*.jsonl")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(os.path.basename(f)[4:-6], "eff", d["efficiency"], "med", d["efficiency_median"], "alone", d["ms_per_step_alone"], "rank", d["runs_chronological"])
PY
step tests bash -c "timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_stencil_gpu.py tests/test_rccl_multiproc_gpu.py tests/test_hosts.py > $O/tests.log 2>&1"
tail -2 $O/tests.log
echo ALLDONE
