#!/bin/bash
# SQ / HBM counter passes on sweepbench variants: gpu_sbprof.sh <outdir> <variant> ...
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1; shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  B=$R/tools/sweepbench/bin/sweepbench_$v
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/sq1_$v -o run -- $B 8192 -1 10 10 > $O/sq1_$v.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM --output-format csv -d $O/sq2_$v -o run -- $B 8192 -1 10 10 > $O/sq2_$v.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$v -o run -- $B 8192 -1 10 10 > $O/f_$v.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$v -o run -- $B 8192 -1 10 10 > $O/w_$v.log 2>&1 || exit 1
done
find $O -name "*counter_collection.csv" | head -20
