#!/bin/bash
# wpsbench runs: gpu_wps.sh <outdir> "<PxL> <n> <ht>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
for spec in "$@"; do
  set -- $spec
  timeout -k 5 60 tools/sweepbench/bin/wps_$1 $2 $3 ${4:-100} >> $O/wps.jsonl 2>> $O/wps.err
  rc=$?
  if [ $rc -gt 1 ]; then echo "FAILED rc=$rc: $spec"; tail -5 $O/wps.err; exit 1; fi
done
cat $O/wps.jsonl
