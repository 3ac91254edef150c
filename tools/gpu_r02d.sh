#!/bin/bash
# Round-2: single-path fast sweep + global-edge bands in the ring kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_stencil_gpu.py -x -q --timeout 300 --timeout-method thread > $O/stencil_tests.log 2>&1 || { echo "stencil tests failed"; tail -40 $O/stencil_tests.log; exit 1; }
tail -2 $O/stencil_tests.log
timeout -k 10 200 python -u tools/tune_deep.py 8192 20 12,10,8 -1,82,100,127 > $O/tune_release.jsonl 2>&1 || exit 1
SMI_LIB_VARIANT=exp_g1 timeout -k 10 120 python -u tools/tune_deep.py 8192 20 12 -1 > $O/tune_g1.jsonl 2>&1 || exit 1
SMI_LIB_VARIANT=exp_g3 timeout -k 10 120 python -u tools/tune_deep.py 8192 20 12 -1 > $O/tune_g3.jsonl 2>&1 || exit 1
cat $O/tune_*.jsonl | grep -v amdgpu.ids
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-aux --no-cpu-baseline > $O/bench_20_5.json 2> $O/bench_20_5.err || exit 1
timeout -k 10 120 python bench.py --no-aux --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || exit 1
for f in bench_20_5 bench_default; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['ms_per_step'],[(k['kernel'][:16],k['launches'],k['total_ms']) for k in d['roofline']['kernels']])"; done
