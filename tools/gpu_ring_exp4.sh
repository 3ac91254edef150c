#!/bin/bash
# repeat: base vs low-priority comm stream (LDS ring), rounds 2 and 3
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for i in 1 2; do
for cfg in base lowprio; do
  if [ $cfg = lowprio ]; then E=SMI_COMM_LOW_PRIORITY=1; else E=X=1; fi
  env $E SMI_LOOPBACK_FUSED=1 REHEARSAL_ROUNDS=2,3 timeout -k 10 150 python tools/rehearsal.py 8192 12 > $O/${cfg}_$i.jsonl 2>>$O/err.log || exit 1
  grep '"overlap": 1' $O/${cfg}_$i.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$cfg $i rounds',d['rounds'],'eff',d['efficiency'],'ring',d['ring_avg_ms'],'int',d['interior_avg_ms'])"
done
done
