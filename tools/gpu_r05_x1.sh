#!/bin/bash
# Round-5 shared-start sweep (stencilx.h) vs the rotating-ring sweep
# (stencild.h) in tools/xbench, the stream-ordering variants of
# tools/streambench, and the counter list of this box.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$1; mkdir -p $O
B=tools/xbench/bin
step() { echo "=== $1"; shift; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; exit $rc; fi; }
step d20 bash -c "timeout -k 10 120 $B/xbench_d20 8192 100 200 >> $O/x.jsonl 2>> $O/x.err"
for dc in 20 30 40; do
  step x20_$dc bash -c "XB_DCONE=$dc timeout -k 10 120 $B/xbench_x20 8192 100 200 >> $O/x.jsonl 2>> $O/x.err"
done
step x16 bash -c "timeout -k 10 120 $B/xbench_x16 8192 100 200 >> $O/x.jsonl 2>> $O/x.err"
step d20b bash -c "timeout -k 10 120 $B/xbench_d20 8192 100 200 >> $O/x.jsonl 2>> $O/x.err"
cat $O/x.jsonl
head -20 $O/x.err
step streambench bash -c "timeout -k 10 120 tools/streambench/streambench 200 > $O/streambench.jsonl 2> $O/streambench.err"
cat $O/streambench.jsonl
step counters bash -c "cd /tmp && timeout -k 10 60 rocprofv3 --list-avail > $R/$O/counters.txt 2>&1"
grep -iE "icache|ifetch|SQC_" $O/counters.txt | head -30
echo ALLDONE
