#!/bin/bash
# Run GPU steps in order; stop at the first step whose exit status is not a
# plain pass/fail (crash, abort, fault, timeout).  Usage: gpu_session.sh "cmd1" "cmd2" ...
mkdir -p gpurun_out
i=0
for cmd in "$@"; do
  i=$((i+1))
  echo "=== step $i: $cmd"
  bash -c "$cmd"
  rc=$?
  echo "=== step $i rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: step $i exited with $rc"
    exit $rc
  fi
done
