#!/bin/bash
# Does a wait packet on a highest-priority stream serialise the pass?  The
# caller's stream at the highest priority with the host-observed join on and
# off, next to the normal-priority caller (the library's interior stream).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$1; mkdir -p $O
step() { echo "=== $1"; shift; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; exit $rc; fi; }
step warm timeout -k 10 300 python -u -c 'print("importing torch", flush=True); import torch; torch.zeros(1).cuda(); print("warm", flush=True)'
G="REHEARSAL_PASSES=20 REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_LEAN=1 REHEARSAL_OVERLAP=1 REHEARSAL_PROF=0 REHEARSAL_TRANSPORT=rccl"
for r in 1 2; do
  for spec in high_j1:REH_STREAM_PRIO=high high_j0:REH_STREAM_PRIO=high,SMI_HOST_JOIN=0 normal_j1:X=1 normal_j0:SMI_HOST_JOIN=0 transport_normal_j0:REHEARSAL_TRANSPORT=inproc,SMI_HOST_JOIN=0 transport_high_j0:REHEARSAL_TRANSPORT=inproc,SMI_HOST_JOIN=0,REH_STREAM_PRIO=high; do
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
            print(os.path.basename(f)[4:-6], d["exchange"][:12], "eff", d["efficiency"], "med", d["efficiency_median"], "alone", d["ms_per_step_alone"], "rank", d["runs_chronological"])
PY
echo ALLDONE
