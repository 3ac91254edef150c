#!/bin/bash
# Which hardware queue the interior's stream lands on (HIP maps streams onto
# GPU_MAX_HW_QUEUES queues; RCCL creates streams of its own): rehearsal with
# the real RCCL exchange, one stream for all runs, created late (after the
# communicator, default), early, at high priority, or with 8 / 16 HW queues.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$1; mkdir -p $O
step() { echo "=== $1"; shift; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; exit $rc; fi; }
step warm timeout -k 10 300 python -u -c 'print("importing torch", flush=True); import torch; torch.zeros(1).cuda(); print("warm", flush=True)'
G="REHEARSAL_PASSES=20 REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_LEAN=1 REHEARSAL_OVERLAP=1 REHEARSAL_PROF=0 REHEARSAL_TRANSPORT=rccl"
for spec in late:X=1 early:REH_STREAM_EARLY=1 high:REH_STREAM_PRIO=high q8:GPU_MAX_HW_QUEUES=8 q16:GPU_MAX_HW_QUEUES=16 early_j0:REH_STREAM_EARLY=1,SMI_HOST_JOIN=0 transport_late:REHEARSAL_TRANSPORT=inproc transport_early:REHEARSAL_TRANSPORT=inproc,REH_STREAM_EARLY=1; do
  name=${spec%%:*}; envs=$(echo ${spec#*:} | tr ',' ' ')
  step reh_$name bash -c "env $G $envs timeout -k 10 240 python -u tools/rehearsal.py 8192 20 >> $O/reh_$name.jsonl 2>> $O/reh_$name.err"
done
python3 - $O <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/reh_*.jsonl")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(os.path.basename(f)[4:-6], d["exchange"][:12], "eff", d["efficiency"], "med", d["efficiency_median"], "rank", d["runs_chronological"])
PY
echo ALLDONE
