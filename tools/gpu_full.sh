#!/bin/bash
# Full GPU pass into gpurun_out/<tag>: every -m gpu test, smoke, the bench at
# the driver's own command (--gpus 1 --steps 20 --warmup 5) and at its
# defaults, rocprofv3 kernel stats of the driver's command and FETCH/WRITE
# counter passes of the same command (its sweepk<10> passes), plus the same
# for the default command's sweepk<12>, an SQ pass, and the interior-rank
# rehearsal (one-kernel exchange and in-process transport) with a kernel trace.  Afterwards, on the
# CPU: tools/pmc_summarize.py driver|pmc ... into profiles/ (see DESIGN.md §7).
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
if [ -z "$SKIP_TESTS" ]; then
step tests bash -c "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }"
tail -1 $O/gpu_tests.log
step smoke bash -c "timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1"
fi
step bench_driver bash -c "timeout -k 10 200 python bench.py $DRV > $O/bench_driver.json 2> $O/bench_driver.err"
step bench_default bash -c "timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err"
cd /tmp && export TMPDIR=/tmp
step rocprof_driver timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_driver -o run -- python3 $R/bench.py $DRV > $R/$O/bench_prof_driver.json 2> $R/$O/bench_prof_driver.err
step pmc_fetch_driver timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_f_driver -o run -- python3 $R/bench.py $DRV --no-aux --no-cpu-baseline > $R/$O/pmc_f_driver.log 2>&1
step pmc_write_driver timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_w_driver -o run -- python3 $R/bench.py $DRV --no-aux --no-cpu-baseline > $R/$O/pmc_w_driver.log 2>&1
step rocprof_default timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_default -o run -- python3 $R/bench.py --no-aux --no-cpu-baseline > $R/$O/bench_prof_default.json 2> $R/$O/bench_prof_default.err
step pmc_fetch_k12 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_f12 -o run -- python3 $R/bench.py --steps 48 --warmup 12 --no-cpu-baseline --no-aux > $R/$O/pmc_f12.log 2>&1
step pmc_write_k12 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_w12 -o run -- python3 $R/bench.py --steps 48 --warmup 12 --no-cpu-baseline --no-aux > $R/$O/pmc_w12.log 2>&1
step pmc_sq timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $R/$O/sq -o run -- python3 $R/bench.py $DRV --no-cpu-baseline --no-aux > $R/$O/sq.log 2>&1
cd $R
G="REHEARSAL_PASSES=40 REHEARSAL_OVERLAP=1 REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0"
step rehearsal bash tools/gpu_reh_grid.sh $1/rehearsal "copy:$G SMI_LOOPBACK_FUSED=1" "transport:$G" "copy_b:$G SMI_LOOPBACK_FUSED=1" "transport_b:$G"
step rehearsal_trace bash tools/gpu_trace_reh.sh $1/rehearsal "copy:$G SMI_LOOPBACK_FUSED=1"
for f in bench_driver bench_default; do python -c "import json;d=json.load(open('$O/$f.json'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r['frac'],r.get('hbm_frac'),r['kernel_avg_ms'],[(k['kernel'][:16],k['launches'],k['total_ms']) for k in r['kernels']])"; done
echo ALLDONE
