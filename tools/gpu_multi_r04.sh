#!/bin/bash
# Round-4 multi-rank checks on one GPU into gpurun_out/<tag>: the
# interior-rank rehearsal (K = 20 rotating-ring interior vs K = 12), and
# bench.py --gpus 2 / 8 --fake-host (RCCL over sockets; functional, with the
# parity check of the timed plan on every rank's light cone).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$1; mkdir -p $O
step() { echo "=== $1"; shift; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; exit $rc; fi; }
G="REHEARSAL_PASSES=20 REHEARSAL_OVERLAP=1 REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0"
step reh_copy bash -c "env $G SMI_LOOPBACK_FUSED=1 timeout -k 10 200 python -u tools/rehearsal.py 8192 20 12 > $O/rehearsal_copy.jsonl 2> $O/rehearsal_copy.err"
step reh_transport bash -c "env $G timeout -k 10 200 python -u tools/rehearsal.py 8192 20 12 > $O/rehearsal_transport.jsonl 2> $O/rehearsal_transport.err"
cat $O/rehearsal_*.jsonl | python3 -c "import json,sys;[print(d['K'],d['exchange'],d['ms_per_step_alone'],d['ms_per_step_interior_rank'],d['efficiency'],d['band_avg_ms'],d['interior_avg_ms']) for d in map(json.loads,sys.stdin)]"
step fake2 bash -c "timeout -k 10 300 python bench.py --gpus 2 --fake-host --steps 20 --warmup 5 --no-aux > $O/bench_fake2.json 2> $O/bench_fake2.err"
step fake8 bash -c "timeout -k 10 600 python bench.py --gpus 8 --fake-host --steps 20 --warmup 5 --no-aux > $O/bench_fake8.json 2> $O/bench_fake8.err"
for f in bench_fake2 bench_fake8; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['config']['plan'],d['parity'])"; done
echo ALLDONE
