#!/bin/bash
# comm-stream priority x enqueue order on the interior-rank rehearsal (LDS ring)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
run() {  # name, env...
  local name=$1; shift
  env "$@" SMI_LOOPBACK_FUSED=1 REHEARSAL_ROUNDS=1,2 timeout -k 10 150 python tools/rehearsal.py 8192 12 > $O/$name.jsonl 2>>$O/err.log || exit 1
  grep '"overlap": 1' $O/$name.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$name rounds',d['rounds'],'eff',d['efficiency'],'ring',d['ring_avg_ms'],'int',d['interior_avg_ms'])"
}
run base X=1
run lowprio SMI_COMM_LOW_PRIORITY=1
run intfirst SMI_INTERIOR_FIRST=1
run both SMI_COMM_LOW_PRIORITY=1 SMI_INTERIOR_FIRST=1
