#!/bin/bash
# Full GPU pass into gpurun_out/<tag>: every -m gpu test, smoke, the bench at
# the driver's settings and at its defaults, rocprofv3 kernel stats of the
# default bench command, FETCH/WRITE/SQ counter passes on the K=12 sweep and
# FETCH/WRITE on K=10 passes (the driver's --steps 20 plan).  Afterwards, on
# the CPU: tools/pmc_summarize.py pmc ... profiles/pmc_stencil_sweep.json 12|10
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$1
mkdir -p $O
step() {  # step <name> <cmd...>: stop at the first failing step
  echo "=== $1"; shift
  "$@"; rc=$?
  if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; exit $rc; fi
}
step tests bash -c "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }"
tail -1 $O/gpu_tests.log
step smoke bash -c "timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1"
step bench_20_5 bash -c "timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err"
step bench_default bash -c "timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err"
cd /tmp && export TMPDIR=/tmp
step rocprof_stats timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python $R/bench.py --no-aux --no-cpu-baseline > $R/$O/bench_prof.json 2> $R/$O/bench_prof.err
step pmc_fetch timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_f -o run -- python $R/bench.py --steps 48 --warmup 12 --no-cpu-baseline --no-aux > $R/$O/pmc_f.log 2>&1
step pmc_write timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_w -o run -- python $R/bench.py --steps 48 --warmup 12 --no-cpu-baseline --no-aux > $R/$O/pmc_w.log 2>&1
step pmc_sq timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $R/$O/sq -o run -- python $R/bench.py --steps 48 --warmup 12 --no-cpu-baseline --no-aux > $R/$O/sq.log 2>&1
step pmc_fetch_k10 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_f10 -o run -- python $R/tools/pmc_sweep.py 8192 10 10 > $R/$O/pmc_f10.log 2>&1
step pmc_write_k10 timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_w10 -o run -- python $R/tools/pmc_sweep.py 8192 10 10 > $R/$O/pmc_w10.log 2>&1
cd $R
for f in bench_20_5 bench_default; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['ms_per_step'],d['roofline'].get('hbm_frac'),[(k['kernel'][:16],k['launches'],k['total_ms']) for k in d['roofline']['kernels']])"; done
echo ALLDONE
