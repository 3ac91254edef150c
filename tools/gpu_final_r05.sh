#!/bin/bash
# Round-5 final GPU pass into gpurun_out/<tag>: every -m gpu test + smoke, the
# bench at the driver's command and its defaults with rocprofv3 kernel stats,
# PMC (FETCH / WRITE / SQ) of the driver's command, the faithful interior-rank
# rehearsal (real RCCL kernel with the caller's stream at normal and at the
# highest priority, 20 and 60 passes; RCCL-footprint stand-in; in-process
# transport) with a kernel trace of the RCCL run
# and bench --gpus 2 / 4 / 8 --fake-host with parity.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
T=$1
O=gpurun_out/$T; mkdir -p $O
step() { echo "=== $1"; shift; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; exit $rc; fi; }
echo "=== warm"
timeout -k 10 300 python -u -c 'print("importing torch", flush=True); import torch; torch.zeros(1).cuda(); import smi_amd; smi_amd.load(build_if_missing=False); print("warm", flush=True)' || exit 1
[ -n "$SKIP_TESTS" ] || step tests bash tools/gpu_tests.sh $T
step bench env TESTS=none PROF=1 bash tools/gpu_r04.sh $T
bash tools/gpu_prof_r04.sh $T/prof > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
G="REHEARSAL_PASSES=20 REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_LEAN=1 REHEARSAL_OVERLAP=1 REHEARSAL_PROF=0"
for spec in rccl:REHEARSAL_TRANSPORT=rccl rccl_high:REHEARSAL_TRANSPORT=rccl,REH_STREAM_PRIO=high rccl_p60:REHEARSAL_TRANSPORT=rccl,REHEARSAL_PASSES=60 heavy16:SMI_LOOPBACK_HEAVY=16 transport:X=1; do
  name=${spec%%:*}; envs=$(echo ${spec#*:} | tr ',' ' ')
  step reh_$name bash -c "env $G $envs timeout -k 10 240 python -u tools/rehearsal.py 8192 20 > $O/reh_$name.jsonl 2> $O/reh_$name.err"
  grep '^{' $O/reh_$name.jsonl | python3 -c "import json,sys;[print('$name',d['exchange'][:40],d['ms_per_step_alone'],d['ms_per_step_interior_rank'],d['efficiency'],d['efficiency_median'],d['runs_chronological']) for d in map(json.loads,sys.stdin)]"
done
step traces bash -c "env REH_K=20 REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_PASSES=20 REHEARSAL_LEAN=1 bash tools/gpu_trace_reh.sh $T/tr rccl:REHEARSAL_TRANSPORT=rccl > $O/traces.log 2>&1"
grep '^{' $O/traces.log || true
for n in 2 4 8; do
  step fake$n bash -c "timeout -k 10 500 python bench.py --gpus $n --fake-host --steps 20 --warmup 5 --no-aux > $O/bench_fake$n.json 2> $O/bench_fake$n.err"
  python3 -c "import json;d=json.load(open('$O/bench_fake$n.json'));print('fake$n',d['value'],d['config']['decomposition'],d['parity']['bit_exact'],d['parity']['cells'])"
done
echo ALLDONE
