#!/bin/bash
# Full GPU pass: parity tests, bench, kernel-trace stats, two PMC passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_session.sh \
 "timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1" \
 "timeout -k 10 200 python bench.py > gpurun_out/bench.json 2>gpurun_out/bench.err" \
 "cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python $R/bench.py > $R/gpurun_out/bench_prof.json 2>$R/gpurun_out/bench_prof.err" \
 "cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_f -o run -- python $R/bench.py --steps 48 --warmup 12 --no-cpu-baseline --no-aux > $R/gpurun_out/pmc_f.log 2>&1" \
 "cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_w -o run -- python $R/bench.py --steps 48 --warmup 12 --no-cpu-baseline --no-aux > $R/gpurun_out/pmc_w.log 2>&1" \
 "cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $R/gpurun_out/sq -o run -- python $R/bench.py --steps 48 --warmup 12 --no-cpu-baseline --no-aux > $R/gpurun_out/sq.log 2>&1"
