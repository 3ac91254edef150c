#!/bin/bash
# ring-kernel timing experiments on the rehearsal build (overlap off: ring timed alone)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for m in 0 1 2 4 7; do
  SMI_RING_EXP=$m SMI_LOOPBACK_FUSED=1 REHEARSAL_ROUNDS=1 timeout -k 10 120 python tools/rehearsal.py 8192 12 > $O/ring_exp_$m.jsonl 2>>$O/err.log || exit 1
  echo "mode $m: $(grep '"overlap": 0' $O/ring_exp_$m.jsonl | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ring_avg_ms"], d["interior_avg_ms"])')"
done
