#!/bin/bash
# Round-2 first pass: stencil parity (new K-step sweep), tuning table, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_stencil_gpu.py -x -q --timeout 300 --timeout-method thread > $O/stencil_tests.log 2>&1 || { echo "stencil tests failed"; tail -30 $O/stencil_tests.log; exit 1; }
tail -3 $O/stencil_tests.log
timeout -k 10 200 python -u tools/tune_deep.py 8192 20 12,10,8 -1,73,100,145,199,289 > $O/tune_release.jsonl 2>&1 || exit 1
SMI_LIB_VARIANT=exp_d3 timeout -k 10 120 python -u tools/tune_deep.py 8192 20 12,8 -1,100,145,199 > $O/tune_d3.jsonl 2>&1 || exit 1
SMI_LIB_VARIANT=exp_d9 timeout -k 10 120 python -u tools/tune_deep.py 8192 20 12,8 -1,100,145,199 > $O/tune_d9.jsonl 2>&1 || exit 1
cat $O/tune_*.jsonl
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-aux --no-cpu-baseline > $O/bench_20_5.json 2> $O/bench_20_5.err || exit 1
timeout -k 10 200 python bench.py --no-aux --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || exit 1
cat $O/bench_20_5.json $O/bench_default.json
