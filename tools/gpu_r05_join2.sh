#!/bin/bash
# Round-5 host-observed join, second pass: rehearsal A/B (join on / off) with
# the garbage collector off in the timed runs (and one series with it on),
# median-to-median efficiency, 20- and 60-pass runs.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$1; mkdir -p $O
step() { echo "=== $1"; shift; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; exit $rc; fi; }
step warm timeout -k 10 300 python -u -c 'print("importing torch", flush=True); import torch; torch.zeros(1).cuda(); print("warm", flush=True)'
G="REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_LEAN=1 REHEARSAL_OVERLAP=1 REHEARSAL_PROF=0"
for r in 1 2; do  # r05_join3: one stream for every run
  for spec in rccl_j1:REHEARSAL_TRANSPORT=rccl,SMI_HOST_JOIN=1 rccl_j0:REHEARSAL_TRANSPORT=rccl,SMI_HOST_JOIN=0 rccl_j1_gc:REHEARSAL_TRANSPORT=rccl,SMI_HOST_JOIN=1,REHEARSAL_GC=1 transport_j1:SMI_HOST_JOIN=1 transport_j0:SMI_HOST_JOIN=0 rccl_j1_p60:REHEARSAL_TRANSPORT=rccl,SMI_HOST_JOIN=1,REHEARSAL_PASSES=60 rccl_j0_p60:REHEARSAL_TRANSPORT=rccl,SMI_HOST_JOIN=0,REHEARSAL_PASSES=60; do
    name=${spec%%:*}; envs=$(echo ${spec#*:} | tr ',' ' ')
    step reh_$name bash -c "env REHEARSAL_PASSES=20 $G $envs timeout -k 10 240 python -u tools/rehearsal.py 8192 20 >> $O/reh_$name.jsonl 2>> $O/reh_$name.err"
  done
done
python3 - $O <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/reh_*.jsonl")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(os.path.basename(f)[4:-6], "eff", d["efficiency"], "med", d["efficiency_median"], "alone", d["alone_runs_ms_per_step"], "rank", d["runs_chronological"])
PY
echo ALLDONE
