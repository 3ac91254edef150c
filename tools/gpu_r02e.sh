#!/bin/bash
# Round-2 (re-entry): full GPU suite on the committed K-step rework, smoke, benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || { tail $O/bench_20_5.err; exit 1; }
timeout -k 10 200 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
for f in bench_20_5 bench_default; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['ms_per_step'],d['roofline']['frac'],[(k['kernel'][:16],k['launches'],k['total_ms']) for k in d['roofline']['kernels']])"; done
