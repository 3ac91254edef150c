#!/bin/bash
# One GPU session on the box: gpu.sh TAG STEP [STEP ...] runs the steps in
# order into gpurun_out/TAG and stops at the first that fails (a failing GPU
# step ends the call: nothing else touches the GPU after it).  Steps:
#   warm      import torch + load the library (the first import pages in)
#   tests     every -m gpu test (TESTS / KEXPR narrow it), then smoke()
#   smoke     smoke() alone
#   bench     bench.py at the driver's command -> bench_driver.json
#   default   bench.py at its defaults          -> bench_default.json
#   prof      rocprofv3 --kernel-trace --stats of the driver's command
#   pmc       FETCH_SIZE / WRITE_SIZE / SQ passes of the driver's command
#   reh       the interior-rank rehearsal (tools/rehearsal.py; REH_ENV adds
#             settings), against the bench step's lone tile when it ran
#   trace     kernel traces of the rehearsal, one per case (TRACE_CASES)
#   stall     rehearsal with a host that falls behind every 10th pass
#             (STALL_US), host join vs wait packets
#   fake      bench.py --gpus 2/4/8 --fake-host with parity (FAKE_N)
#   hosts     the C++ hosts' tests (tests/test_hosts.py)
#   p2p       tools/p2p_sweep.sh + a kernel trace of the 256 MiB bulk copy
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=$1; shift
O=$R/gpurun_out/$TAG; mkdir -p $O
DRV="--gpus 1 --steps 20 --warmup 5"
fail() { echo "=== FAILED $1 rc=$2"; exit $2; }
summ() { python3 -c "import json;d=json.load(open('$1'));r=d['roofline'];print('$(basename $1)',d['value'],d['ms_per_step'],r['frac'],r['kernel_avg_ms'],r.get('kernels_share_of_timed_region'),d.get('parity',{}).get('bit_exact'))"; }
for st in "$@"; do
  echo "=== $st"
  case $st in
  warm)
    timeout -k 10 300 python -u -c 'print("importing torch", flush=True); import torch; torch.zeros(1).cuda(); import smi_amd; smi_amd.load(build_if_missing=False); print("warm", flush=True)' || fail $st $?
    ;;
  tests)
    timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu ${KEXPR:+-k "$KEXPR"} -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
    rc=$?; tail -5 $O/gpu_tests.log; [ $rc -eq 0 ] || fail $st $rc
    timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || fail smoke $?
    tail -1 $O/smoke.log
    ;;
  smoke)
    timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || fail $st $?
    tail -1 $O/smoke.log
    ;;
  hosts)
    timeout -k 10 600 python -u -m pytest tests/test_hosts.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/hosts.log 2>&1
    rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/hosts.log | tail -30; [ $rc -eq 0 ] || fail $st $rc
    ;;
  bench)
    timeout -k 10 200 python bench.py $DRV > $O/bench_driver.json 2> $O/bench_driver.err || fail $st $?
    summ $O/bench_driver.json
    ;;
  default)
    timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || fail $st $?
    summ $O/bench_default.json
    ;;
  prof)
    (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver -o run -- python3 $R/bench.py $DRV > $O/bench_prof_driver.json 2> $O/bench_prof_driver.err) || fail $st $?
    grep -h sweepd $O/prof_driver/*kernel_stats.csv | head -3
    ;;
  pmc)
    cd /tmp; export TMPDIR=/tmp
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- python3 $R/bench.py $DRV --no-aux --no-cpu-baseline --no-parity > $O/pmc_f.log 2>&1 || fail pmc_fetch $?
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- python3 $R/bench.py $DRV --no-aux --no-cpu-baseline --no-parity > $O/pmc_w.log 2>&1 || fail pmc_write $?
    timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/sq -o run -- python3 $R/bench.py $DRV --no-cpu-baseline --no-aux --no-parity > $O/sq.log 2>&1 || fail pmc_sq $?
    cd $R
    ;;
  reh)
    lone=""
    [ -f $O/bench_default.json ] && lone=$(python3 -c "import json;d=json.load(open('$O/bench_default.json'));print(8192*8192/d['value']/1e6)")
    env BENCH_LONE_MS_PER_STEP=$lone $REH_ENV timeout -k 10 400 python -u tools/rehearsal.py 8192 ${REH_K:-20} >> $O/reh.jsonl 2>> $O/reh.err || fail $st $?
    tail -1 $O/reh.jsonl | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('bench lone',d['bench_lone_ms_per_step']);[print(c,v['ms_per_step_min'],v['ms_per_step_median'],v.get('efficiency_min'),v.get('efficiency_median'),v.get('efficiency_vs_bench_median'),v.get('interior_avg_ms')) for c,v in d['cases'].items()]"
    ;;
  stall)
    # what a host that falls behind costs: SMI_REH_STALL_US of busy host time
    # every 10th pass, host join (1) vs wait packets (0)
    for j in 1 0; do for us in ${STALL_US:-0 50 100 200 500}; do
      env REHEARSAL_CASES=alone,full REHEARSAL_REPS=${STALL_REPS:-3} SMI_HOST_JOIN=$j SMI_REH_STALL_US=$us timeout -k 10 200 python -u tools/rehearsal.py 8192 20 > $O/stall_j${j}_$us.json 2> $O/stall_j${j}_$us.err || fail stall_j${j}_$us $?
      python3 -c "import json;d=json.load(open('$O/stall_j${j}_$us.json'));c=d['cases'];print('join $j stall_us $us', c['alone']['ms_per_step_median'], c['full']['ms_per_step_median'], c['full']['efficiency_median'])"
    done; done
    ;;
  trace)
    for c in ${TRACE_CASES:-alone full bands xchg bare}; do
      (cd /tmp && env TMPDIR=/tmp REHEARSAL_CASES=$c REHEARSAL_REPS=1 REHEARSAL_PASSES=${TRACE_PASSES:-100} REHEARSAL_WARM_MS=50 $REH_ENV timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$c -o run -- python3 $R/tools/rehearsal.py 8192 ${REH_K:-20} > $O/trace_$c.log 2>&1) || fail trace_$c $?
      python3 $R/tools/pass_timeline.py $O/trace_$c/run_kernel_trace.csv 60 > $O/timeline_$c.txt
      echo "$c $(tail -1 $O/timeline_$c.txt)"
    done
    ;;
  fake)
    for n in ${FAKE_N:-2 4 8}; do
      timeout -k 10 500 python bench.py --gpus $n --fake-host --steps 20 --warmup 5 --no-aux > $O/bench_fake$n.json 2> $O/bench_fake$n.err || fail fake$n $?
      python3 -c "import json;d=json.load(open('$O/bench_fake$n.json'));print('fake$n',d['value'],d['config']['decomposition'],d['parity']['bit_exact'],d['parity']['cells'])"
    done
    ;;
  p2p)
    timeout -k 10 900 bash tools/p2p_sweep.sh $O/p2p || fail $st $?
    (cd /tmp && TMPDIR=/tmp timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_p2p -o run -- $R/hosts/_build/bandwidth_benchmark -k 262144 -r 1 -i 10 -p 2 > $O/prof_p2p.log 2>&1) || fail prof_p2p $?
    grep -h multicopy $O/prof_p2p/*kernel_stats.csv | head -2
    ;;
  *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo ALLDONE
