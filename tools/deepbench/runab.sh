# runab.sh OUTDIR ROUNDS variant... : interleaved repeated timing runs (A/B on one box)
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; shift; rounds=$1; shift
mkdir -p $out
for i in $(seq $rounds); do
  for b in "$@"; do
    timeout -k 10 60 tools/deepbench/bin/deepbench_$b 8192 100 200 >> $out/ab.jsonl 2>> $out/ab_err.log; rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$b rc=$rc"; exit 1; fi
  done
done
python3 tools/deepbench/absum.py $out/ab.jsonl
