#!/bin/bash
# power.sh TAG CMD...: socket power and clocks (read-only rocm-smi queries)
# while CMD runs in the background -- idle first, then one sample every
# ~0.5 s until CMD exits -- into gpurun_out/TAG/power.log; CMD's stdout goes
# to gpurun_out/TAG/power_cmd.out.  Example (the K = 20 sweep back to back):
#   tools/power.sh pw python bench.py --steps 200000 --warmup 0 --no-cpu-baseline --no-parity --no-aux
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; shift; mkdir -p $out
sample() {  # label
  echo "== $1 $(date +%s.%N)" >> $out/power.log
  timeout -k 5 20 rocm-smi --showpower --showclocks --json >> $out/power.log 2>&1
  echo >> $out/power.log
}
sample idle
timeout -k 10 300 "$@" > $out/power_cmd.out 2> $out/power_cmd.err &
pid=$!
sleep 3
while kill -0 $pid 2> /dev/null; do
  sample load
  sleep 0.5
done
wait $pid || { echo "command rc=$?"; exit 1; }
echo ALLDONE
