#!/bin/bash
# Round-2: restored register-ring sweep (global edges in-kernel) -- parity, sweepbench, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_stencil_gpu.py -x -q --timeout 300 --timeout-method thread > $O/stencil_tests.log 2>&1 || { echo "stencil tests failed"; tail -40 $O/stencil_tests.log; exit 1; }
tail -2 $O/stencil_tests.log
for v in "lib 8192 -1" "k8 8192 -1" "lib 8192 120" "lib 8192 170"; do
  timeout -k 5 60 tools/sweepbench/bin/sweepbench_${v%% *} ${v#* } >> $O/sb.jsonl 2>> $O/sb.err || { echo "sb failed $v"; exit 1; }
done
cat $O/sb.jsonl
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-aux --no-cpu-baseline > $O/bench_20_5.json 2> $O/bench_20_5.err || { tail $O/bench_20_5.err; exit 1; }
timeout -k 10 120 python bench.py --no-aux --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
for f in bench_20_5 bench_default; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['ms_per_step'],[(k['kernel'][:16],k['launches'],k['total_ms']) for k in d['roofline']['kernels']])"; done
