#!/bin/bash
# Round-4 profiles of the driver's command into gpurun_out/<tag>: rocprofv3
# --kernel-trace --stats, FETCH_SIZE and WRITE_SIZE passes (one counter
# group per run, MI355X_MICROARCH.md "HBM"), and SQ counters.  Afterwards, on
# the CPU: tools/pmc_summarize.py driver|pmc into profiles/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
step() { echo "=== $1"; shift; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; exit $rc; fi; }
DRV="--gpus 1 --steps 20 --warmup 5"
cd /tmp && export TMPDIR=/tmp
step rocprof_driver timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver -o run -- python3 $R/bench.py $DRV > $O/bench_prof_driver.json 2> $O/bench_prof_driver.err
step pmc_fetch timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- python3 $R/bench.py $DRV --no-aux --no-cpu-baseline --no-parity > $O/pmc_f.log 2>&1
step pmc_write timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- python3 $R/bench.py $DRV --no-aux --no-cpu-baseline --no-parity > $O/pmc_w.log 2>&1
step pmc_sq timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/sq -o run -- python3 $R/bench.py $DRV --no-cpu-baseline --no-aux --no-parity > $O/sq.log 2>&1
echo ALLDONE
