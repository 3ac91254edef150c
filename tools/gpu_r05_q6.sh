#!/bin/bash
# Does the band kernel's dispatch (comm stream at the highest priority) delay
# the next interior at the pass boundary?  Rehearsal with the comm stream at
# the highest (default) and the lowest priority, real RCCL exchange, caller's
# stream at the highest priority; kernel traces of both.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$1; mkdir -p $O
step() { echo "=== $1"; shift; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; exit $rc; fi; }
step warm timeout -k 10 300 python -u -c 'print("importing torch", flush=True); import torch; torch.zeros(1).cuda(); print("warm", flush=True)'
G="REHEARSAL_PASSES=20 REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_LEAN=1 REHEARSAL_OVERLAP=1 REHEARSAL_PROF=0 REHEARSAL_TRANSPORT=rccl REH_STREAM_PRIO=high"
for r in 1 2; do
  for spec in comm_high:X=1 comm_low:SMI_COMM_LOW_PRIORITY=1; do
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
step traces bash -c "env REH_K=20 REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_PASSES=20 REHEARSAL_LEAN=1 bash tools/gpu_trace_reh.sh $1/tr 'comm_high:REHEARSAL_TRANSPORT=rccl REH_STREAM_PRIO=high' 'comm_low:REHEARSAL_TRANSPORT=rccl REH_STREAM_PRIO=high SMI_COMM_LOW_PRIORITY=1' > $O/traces.log 2>&1"
grep '^{' $O/traces.log || true
echo ALLDONE
