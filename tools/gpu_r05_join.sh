#!/bin/bash
# Round-5 host-observed pass join (stencil_run.cpp join_band): interior-rank
# rehearsal A/B with the join on (SMI_HOST_JOIN=1, the default) and off
# (stream wait packet), real RCCL exchange and in-process transport,
# alternating; one kernel trace with the join on; then the stencil GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$1; mkdir -p $O
step() { echo "=== $1"; shift; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; exit $rc; fi; }
step warm timeout -k 10 300 python -u -c 'print("importing torch", flush=True); import torch; torch.zeros(1).cuda(); print("warm", flush=True)'
G="REHEARSAL_PASSES=20 REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_LEAN=1 REHEARSAL_OVERLAP=1 REHEARSAL_PROF=0"
for r in 1 2; do
  for spec in rccl_j1:REHEARSAL_TRANSPORT=rccl,SMI_HOST_JOIN=1 rccl_j0:REHEARSAL_TRANSPORT=rccl,SMI_HOST_JOIN=0 transport_j1:SMI_HOST_JOIN=1 transport_j0:SMI_HOST_JOIN=0; do
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
            print(os.path.basename(f), d["efficiency"], d.get("efficiency_median"), d["ms_per_step_alone"], d["ms_per_step_interior_rank"])
PY
step traces bash -c "env REH_K=20 REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_PASSES=20 REHEARSAL_LEAN=1 bash tools/gpu_trace_reh.sh $1/tr rccl_j1:REHEARSAL_TRANSPORT=rccl 'rccl_j0:REHEARSAL_TRANSPORT=rccl SMI_HOST_JOIN=0' > $O/traces.log 2>&1"
grep '^{' $O/traces.log || true
step tests bash -c "timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_stencil_gpu.py tests/test_rccl_multiproc_gpu.py tests/test_hosts.py tests/test_bench_launch_gpu.py > $O/tests.log 2>&1"
tail -3 $O/tests.log
echo ALLDONE
