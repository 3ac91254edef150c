# runpmc.sh OUTDIR variant : SQ counters of one deepbench variant (its own rocprofv3 pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $out/sq_$2 -o run -- $GRAFT_REPO_ROOT/tools/deepbench/bin/deepbench_$2 8192 20 10 > $out/sq_$2.log 2>&1
