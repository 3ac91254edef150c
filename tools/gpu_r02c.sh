#!/bin/bash
# Round-2: memory-side experiments on the K=12 sweep (cache policy, walk
# direction) + FETCH/WRITE/SQ counter passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r02c
mkdir -p $O
for v in exp_noedge exp_noedge_nt exp_noedge_onedir; do
  SMI_LIB_VARIANT=$v timeout -k 10 120 python -u tools/tune_deep.py 8192 20 12 -1 2>&1 | grep -v amdgpu.ids >> $O/tune.jsonl || exit 1
done
cat $O/tune.jsonl
cd /tmp && export TMPDIR=/tmp
for v in release exp_noedge exp_noedge_onedir exp_noedge_nt; do
  if [ $v = release ]; then unset SMI_LIB_VARIANT; else export SMI_LIB_VARIANT=$v; fi
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f_$v -o run -- python $R/tools/pmc_sweep.py 8192 12 10 > $O/pmc_f_$v.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w_$v -o run -- python $R/tools/pmc_sweep.py 8192 12 10 > $O/pmc_w_$v.log 2>&1 || exit 1
done
export SMI_LIB_VARIANT=exp_noedge
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/sq_noedge -o run -- python $R/tools/pmc_sweep.py 8192 12 10 > $O/sq.log 2>&1 || exit 1
find $O -name "*counter_collection.csv" | head
