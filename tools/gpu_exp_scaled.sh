#!/bin/bash
# scaled vs exact K=12 sweep (sweepbench, bit-checked), copy calibration, stencil GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for i in 1 2; do
  for v in lib exact; do
    timeout -k 5 60 tools/sweepbench/bin/sweepbench_$v 8192 0 200 >> $O/sb.jsonl 2>> $O/sb.err || { echo "sweepbench $v failed rc=$?"; tail -5 $O/sb.err; exit 1; }
  done
done
timeout -k 10 60 python tools/exp/copy_rate.py >> $O/sb.jsonl 2>> $O/sb.err || exit 1
cat $O/sb.jsonl
timeout -k 10 600 python -u -m pytest tests/test_stencil_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
