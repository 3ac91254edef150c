#!/bin/bash
# interior-rank rehearsal: ring workgroup size x interior wave budget (overlap on)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for nt in 256 128 64; do
  for pct in 100 85 70; do
    SMI_RING_THREADS=$nt SMI_INTERIOR_PCT=$pct SMI_LOOPBACK_FUSED=1 REHEARSAL_ROUNDS=1,2 timeout -k 10 120 python tools/rehearsal.py 8192 12 > $O/r_${nt}_${pct}.jsonl 2>>$O/err.log || exit 1
    grep '"overlap": 1' $O/r_${nt}_${pct}.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('nt=$nt pct=$pct rounds',d['rounds'],'eff',d['efficiency'],'ring',d['ring_avg_ms'],'int',d['interior_avg_ms'])"
  done
done
