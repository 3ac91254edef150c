#!/bin/bash
# Round-4 GPU pass into gpurun_out/<tag>: the rotating-ring sweep's tests (or
# TESTS="<pytest args>"), the bench at the driver's command and at its
# defaults, and rocprofv3 kernel stats of the driver's command.
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
DRV="--gpus 1 --steps 20 --warmup 5"
T=${TESTS:-tests/test_stencil_gpu.py}
KX=${KEXPR:-ring or bench_config}
if [ "$T" != "none" ]; then
  step tests bash -c "timeout -k 10 900 python -u -m pytest $T -k '$KX' -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }"
  tail -1 $O/gpu_tests.log
fi
step bench_driver bash -c "timeout -k 10 200 python bench.py $DRV > $O/bench_driver.json 2> $O/bench_driver.err"
step bench_default bash -c "timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err"
if [ -n "$PROF" ]; then
cd /tmp && export TMPDIR=/tmp
step rocprof_driver timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_driver -o run -- python3 $R/bench.py $DRV > $R/$O/bench_prof_driver.json 2> $R/$O/bench_prof_driver.err
cd $R
fi
for f in bench_driver bench_default; do python -c "import json;d=json.load(open('$O/$f.json'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r['frac'],r['kernel_avg_ms'],r.get('kernels_share_of_timed_region'),d.get('parity',{}).get('bit_exact'),[(k['kernel'][:16],k['launches'],k['total_ms']) for k in r['kernels']])"; done
echo ALLDONE
