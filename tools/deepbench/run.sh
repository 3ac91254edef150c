# run.sh OUTDIR variant... : run deepbench variants (bit check + timing), one JSON line each
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; shift
mkdir -p $out
for b in "$@"; do
  timeout -k 10 60 tools/deepbench/bin/deepbench_$b 8192 100 200 >> $out/res.jsonl 2>> $out/err_$b.log; rc=$?
  echo "$b rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
done
cat $out/res.jsonl
for b in "$@"; do echo "== $b"; head -12 $out/err_$b.log; done
