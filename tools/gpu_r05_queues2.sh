#!/bin/bash
# Round-5 interior stream + host-observed join, measured: interior-rank
# rehearsal with the real RCCL exchange and the in-process transport, the
# caller's stream at normal priority (the library's own interior stream) or
# at the highest (used as it is), join on / off, 20 and 60 passes; a kernel
# trace; then the multi-rank GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$1; mkdir -p $O
step() { echo "=== $1"; shift; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; exit $rc; fi; }
step warm timeout -k 10 300 python -u -c 'print("importing torch", flush=True); import torch; torch.zeros(1).cuda(); print("warm", flush=True)'
G="REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_LEAN=1 REHEARSAL_OVERLAP=1 REHEARSAL_PROF=0"
for r in 1 2; do
  for spec in rccl_normal:REHEARSAL_TRANSPORT=rccl rccl_high:REHEARSAL_TRANSPORT=rccl,REH_STREAM_PRIO=high rccl_high_j0:REHEARSAL_TRANSPORT=rccl,REH_STREAM_PRIO=high,SMI_HOST_JOIN=0 transport_normal:X=1 rccl_normal_p60:REHEARSAL_TRANSPORT=rccl,REHEARSAL_PASSES=60 rccl_high_p60:REHEARSAL_TRANSPORT=rccl,REH_STREAM_PRIO=high,REHEARSAL_PASSES=60; do
    name=${spec%%:*}; envs=$(echo ${spec#*:} | tr ',' ' ')
    step reh_$name bash -c "env REHEARSAL_PASSES=20 $G $envs timeout -k 10 240 python -u tools/rehearsal.py 8192 20 >> $O/reh_$name.jsonl 2>> $O/reh_$name.err"
  done
done
python3 - $O <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/reh_*.jsonl")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(os.path.basename(f)[4:-6], d["exchange"][:12], "eff", d["efficiency"], "med", d["efficiency_median"], "alone", d["ms_per_step_alone"], "rank", d["runs_chronological"])
PY
step traces bash -c "env REH_K=20 REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_PASSES=20 REHEARSAL_LEAN=1 bash tools/gpu_trace_reh.sh $1/tr rccl_normal:REHEARSAL_TRANSPORT=rccl 'rccl_high:REHEARSAL_TRANSPORT=rccl REH_STREAM_PRIO=high' > $O/traces.log 2>&1"
grep '^{' $O/traces.log || true
step tests bash -c "timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_stencil_gpu.py tests/test_rccl_multiproc_gpu.py tests/test_hosts.py tests/test_bench_launch_gpu.py tests/test_configs_at_size_gpu.py > $O/tests.log 2>&1"
tail -3 $O/tests.log
step bench bash -c "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err"
python3 -c "import json;d=json.load(open('$O/bench_driver.json'));print('bench',d['value'],d['repeats']['median'],d['roofline']['kernel_avg_ms'],d['parity']['bit_exact'],d['config']['lib_srchash'][:16])"
step fake2 bash -c "timeout -k 10 300 python bench.py --gpus 2 --fake-host --steps 20 --warmup 5 --no-aux > $O/bench_fake2.json 2> $O/bench_fake2.err"
python3 -c "import json;d=json.load(open('$O/bench_fake2.json'));print('fake2',d['value'],d['repeats'],d['parity']['bit_exact'])"
echo ALLDONE
