#!/bin/bash
# sweepbench runs: gpu_sb.sh <outdir> "<variant> <n> <ht>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
for spec in "$@"; do
  set -- $spec
  timeout -k 5 60 tools/sweepbench/bin/sweepbench_$1 $2 $3 ${4:-200} >> $O/sb.jsonl 2>> $O/sb.err
  rc=$?  # 1 = bit mismatch (expected for the timing-only variants); anything else stops the run
  if [ $rc -gt 1 ]; then echo "FAILED rc=$rc: $spec"; tail -5 $O/sb.err; exit 1; fi
done
cat $O/sb.jsonl
