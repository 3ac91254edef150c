#!/bin/bash
# power.sh OUTDIR : socket power and clocks while the K = 20 sweep runs back
# to back (read-only rocm-smi queries), idle first, then the library's
# geometry (d20: equal blocks) and the balanced halves (u20, fo = 176)
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; mkdir -p $out
sample() {  # label
  for i in 1 2 3 4; do
    echo "== $1 sample $i" >> $out/power.log
    timeout -k 5 20 rocm-smi --showpower --showclocks --showmaxpower --json >> $out/power.log 2>&1
    echo >> $out/power.log
    sleep 0.5
  done
}
sample idle
for spec in d20:XB_KERNEL=d u20:XB_KERNEL=u,XB_FO=176 u20:XB_KERNEL=u,XB_FO=128; do
  v=${spec%%:*}; e=$(echo ${spec#*:} | tr ',' ' ')
  env $e timeout -k 10 60 tools/xbench/bin/xbench_$v 8192 60000 2000 >> $out/xb.jsonl 2>> $out/xb.err &
  pid=$!
  sleep 2.5
  sample "$spec"
  wait $pid || { echo "$spec rc=$?"; exit 1; }
done
echo ALLDONE
