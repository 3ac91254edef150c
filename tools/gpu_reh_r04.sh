#!/bin/bash
# Interior-rank rehearsal at K = 20 without profiling (the production launch
# path), lean vs one-wave-per-segment band kernel, both exchange models,
# three alternating repetitions, into gpurun_out/<tag>/rehearsal.jsonl.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$1; mkdir -p $O
G="REHEARSAL_PASSES=20 REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_LEAN=1,0 REHEARSAL_OVERLAP=1 REHEARSAL_PROF=0"
for rep in 1 2 3; do
  for x in fused transport; do
    F=""; [ $x = fused ] && F="SMI_LOOPBACK_FUSED=1"
    echo "=== rep $rep $x"
    env $G $F timeout -k 10 300 python -u tools/rehearsal.py 8192 20 >> $O/rehearsal.jsonl 2>> $O/rehearsal.err
    rc=$?; if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; exit $rc; fi
  done
done
python3 -c "
import json
for l in open('$O/rehearsal.jsonl'):
    d=json.loads(l); print(d['exchange'], d['band_kernel'], d['ms_per_step_alone'], d['ms_per_step_interior_rank'], d['efficiency'])"
echo ALLDONE
