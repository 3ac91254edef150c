#!/bin/bash
# Kernel traces of interior-rank rehearsals (no profiling markers) into
# gpurun_out/<tag>/trace_<name>: one rocprofv3 --kernel-trace run per
# setting "name:env..." given as arguments, then the per-pass timeline.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}
  envs=${spec#*:}
  echo "=== $name ($envs)"
  env $envs REHEARSAL_PROF=0 REHEARSAL_OVERLAP=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$name -o run -- python $R/tools/rehearsal.py 8192 ${REH_K:-12} > $O/trace_$name.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; tail -5 $O/trace_$name.log; exit $rc; fi
  grep '^{' $O/trace_$name.log
  python $R/tools/pass_timeline.py $O/trace_$name/run_kernel_trace.csv 8
done
