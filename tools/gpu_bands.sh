#!/bin/bash
# Band-kernel / CU-partition check on one GPU into gpurun_out/<tag>: the
# multi-rank stencil parity tests, then the interior-rank rehearsal
# (tools/rehearsal.py, rehearsal build) with a one-copy-kernel exchange for
# every (rounds, band CUs, CU-mask layout, profiling markers) setting, no
# exchange, and the in-process transport, and a kernel trace of one rehearsal.
#   ROUNDS, BAND_CUS, LAYOUTS, PROFS: comma lists; TRACE_CUS: band CUs of the trace
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
if [ -z "$SKIP_TESTS" ]; then
step tests bash -c "timeout -k 10 600 python -u -m pytest tests/test_stencil_gpu.py tests/test_bench_launch_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k '${TESTS_K:-decomposed or band or special or guard or remainder or clipped or config1 or launch}' > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }"
tail -1 $O/tests.log
fi
for lay in ${LAYOUTS:-0}; do
  for prof in ${PROFS:-1}; do
    step reh_fused_l${lay}_p${prof} bash -c "SMI_REH_MASK_LAYOUT=$lay REHEARSAL_PROF=$prof SMI_LOOPBACK_FUSED=1 REHEARSAL_ROUNDS=${ROUNDS:-1,2} REHEARSAL_BAND_CUS=${BAND_CUS:-0} REHEARSAL_BANDFUSION=${FUSIONS:-1:12:0} REHEARSAL_OVERLAP=1 timeout -k 10 300 python tools/rehearsal.py 8192 12 >> $O/rehearsal_fused.jsonl 2>>$O/rehearsal.err"
  done
done
step reh_noxchg bash -c "SMI_LOOPBACK_NOXCHG=1 REHEARSAL_PROF=${PROFS%% *} REHEARSAL_ROUNDS=${ROUNDS:-1,2} REHEARSAL_BAND_CUS=${BAND_CUS:-0} REHEARSAL_BANDFUSION=${FUSIONS:-1:12:0} REHEARSAL_OVERLAP=1 timeout -k 10 150 python tools/rehearsal.py 8192 12 > $O/rehearsal_noxchg.jsonl 2>>$O/rehearsal.err"
step reh_transport bash -c "REHEARSAL_PROF=${PROFS%% *} REHEARSAL_ROUNDS=${ROUNDS:-1,2} REHEARSAL_BAND_CUS=${BAND_CUS:-0} REHEARSAL_BANDFUSION=${FUSIONS:-1:12:0} REHEARSAL_OVERLAP=1,0 timeout -k 10 200 python tools/rehearsal.py 8192 12 > $O/rehearsal_transport.jsonl 2>>$O/rehearsal.err"
cd /tmp && export TMPDIR=/tmp
step trace env SMI_LOOPBACK_FUSED=1 REHEARSAL_PROF=0 REHEARSAL_ROUNDS=${TRACE_ROUNDS:-2} REHEARSAL_BAND_CUS=0 REHEARSAL_BANDFUSION=${TRACE_FUSION:-1:12:0} REHEARSAL_OVERLAP=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- python $R/tools/rehearsal.py 8192 12 > $R/$O/trace.log 2>&1
cd $R
python - <<PY
import json
for f in ("fused", "noxchg", "transport"):
    for l in open("$O/rehearsal_%s.jsonl" % f):
        d = json.loads(l)
        print(f, "rounds", d["rounds"], "cus", d["band_cus"], "fusion", d["band_fusion"], "layout", d["mask_layout"], "prof", d["prof"],
              "ov", d["overlap"], "eff", d["efficiency"], "band", d["band_avg_ms"], "int", d["interior_avg_ms"],
              "alone", d["ms_per_step_alone"])
PY
python tools/pass_timeline.py $O/trace/run_kernel_trace.csv 10
