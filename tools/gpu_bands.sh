#!/bin/bash
# band-sweep ring: multi-rank parity (both ring modes) + interior-rank rehearsal (both modes)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_stencil_gpu.py tests/test_configs_at_size_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "decomposed or config3 or special or guard or halo or remainder or clipped" > $O/tests_bands.log 2>&1 || { tail -30 $O/tests_bands.log; exit 1; }
tail -1 $O/tests_bands.log
SMI_RING_MODE=0 timeout -k 10 400 python -u -m pytest tests/test_stencil_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "decomposed or special or guard" > $O/tests_lds.log 2>&1 || { tail -30 $O/tests_lds.log; exit 1; }
tail -1 $O/tests_lds.log
for m in 1 0; do
  SMI_RING_MODE=$m SMI_LOOPBACK_FUSED=1 REHEARSAL_ROUNDS=1,2 timeout -k 10 150 python tools/rehearsal.py 8192 12 > $O/rehearsal_mode$m.jsonl 2>>$O/err.log || exit 1
  grep '"overlap": 1' $O/rehearsal_mode$m.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('ring mode $m rounds',d['rounds'],'eff',d['efficiency'],'ring',d['ring_avg_ms'],'int',d['interior_avg_ms'],'alone',d['ms_per_step_alone'],'rank',d['ms_per_step_interior_rank'])"
done
