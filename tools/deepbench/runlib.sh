# runlib.sh OUTDIR : the library's K=10 / K=12 sweeps through tools/sweepbench (same-box baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; mkdir -p $out
for b in lib10 lib12; do timeout -k 10 60 tools/sweepbench/bin/sweepbench_$b 8192 -1 100 200 >> $out/res.jsonl 2>> $out/err_$b.log || exit 1; done
tail -2 $out/res.jsonl
