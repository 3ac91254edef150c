#!/bin/bash
# gemv split variants vs one-wave-per-row, fold stride sensitivity, gesummv + reduce parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for v in 0 2 3 1; do
  SMI_GEMV_VARIANT=$v timeout -k 10 200 python tools/exp/gemv_fold.py > $O/exp_v$v.jsonl 2> $O/exp_v$v.err || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gesummv_gpu.py tests/test_configs_at_size_gpu.py tests/test_collectives_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; cat $O/exp_v*.jsonl; tail -3 $O/tests.log; exit $rc
