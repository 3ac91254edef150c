#!/bin/bash
# Sweep-kernel variants (tools/sweepbench/bin/*, built on the CPU by
# tools/sweepbench/build.sh) on one GPU into gpurun_out/<tag>/sweepbench.jsonl:
# each checks its pass bit for bit against K one-step launches, then times
# back-to-back passes.  Usage: gpu_sweepbench.sh <tag> [binary-name ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$1
shift
mkdir -p $O
names=("$@")
if [ ${#names[@]} -eq 0 ]; then names=($(ls tools/sweepbench/bin | sed 's/^sweepbench_//')); fi
for n in "${names[@]}"; do
  for rep in 1 2; do
    timeout -k 10 60 tools/sweepbench/bin/sweepbench_$n 8192 -1 200 300 >> $O/sweepbench.jsonl 2>> $O/sweepbench.err
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "sweepbench_$n rc=$rc: stopping"; exit $rc; fi
  done
done
python -c "
import json
for l in open('$O/sweepbench.jsonl'):
    d = json.loads(l); print(d['variant'], 'K', d['K'], 'mism', d['mismatches'], 'med', d['ms_med'], 'GCells', d['GCells'])"
