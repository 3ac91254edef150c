#!/bin/bash
# Round-5 interior-rank rehearsal with a faithful exchange
# into gpurun_out/<tag>: K = 20, lean band kernel, profiling off; exchange as
# the in-process transport, one light copy kernel, one copy kernel with
# rcclGenericKernel's footprint (8 / 16 / 32 workgroups) and the real RCCL
# kernel (one-rank communicator, self send/recv); kernel traces of the
# RCCL-footprint and real-RCCL runs with their per-pass timelines.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$1; mkdir -p $O
step() { echo "=== $1"; shift; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; exit $rc; fi; }
step warm timeout -k 10 300 python -u -c 'print("importing torch", flush=True); import torch; torch.zeros(1).cuda(); print("warm", flush=True)'
G="REHEARSAL_PASSES=20 REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_LEAN=1 REHEARSAL_OVERLAP=1 REHEARSAL_PROF=0"
for spec in transport: copy:SMI_LOOPBACK_FUSED=1 heavy8:SMI_LOOPBACK_HEAVY=8 heavy16:SMI_LOOPBACK_HEAVY=16 heavy32:SMI_LOOPBACK_HEAVY=32 rccl:REHEARSAL_TRANSPORT=rccl; do
  name=${spec%%:*}; envs=${spec#*:}
  step reh_$name bash -c "env $G $envs timeout -k 10 240 python -u tools/rehearsal.py 8192 20 > $O/reh_$name.jsonl 2> $O/reh_$name.err"
  python3 -c "import json,sys;[print('$name',d['exchange'],d['ms_per_step_alone'],d['ms_per_step_interior_rank'],d['efficiency'],d['runs_ms_per_step']) for d in map(json.loads,open('$O/reh_$name.jsonl'))]"
done
step traces bash -c "env REH_K=20 REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_PASSES=20 REHEARSAL_LEAN=1 bash tools/gpu_trace_reh.sh $1/tr heavy16:SMI_LOOPBACK_HEAVY=16 rccl:REHEARSAL_TRANSPORT=rccl copy:SMI_LOOPBACK_FUSED=1 > $O/traces.log 2>&1"
grep '^{' $O/traces.log
step smoke bash -c "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1"
cat $O/smoke.log
step bench bash -c "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err"
python3 -c "import json;d=json.load(open('$O/bench_driver.json'));r=d['roofline'];c=d['cpu_baseline'];print('bench',d['value'],r['kernel_avg_ms'],r['share_of_timed_region'],d['parity']['bit_exact'],d['config']['lib_srchash'][:16],'cpu',c['value'],c['cores'],c.get('affinity_cpus'),c['legs'].get('all_affinity_cpus'))"
echo ALLDONE
