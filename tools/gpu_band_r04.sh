#!/bin/bash
# Round-4 lean band kernel checks on one GPU into gpurun_out/<tag>: its GPU
# tests, the interior-rank rehearsal at K = 20 with the lean and the
# one-wave-per-segment band kernel (both exchange models), and the timed
# region overhead probe.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$1; mkdir -p $O
step() { echo "=== $1"; shift; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; exit $rc; fi; }
step tests bash -c "timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_stencil_gpu.py -k 'band_kernel_choice or ring_decomposed or ring_band_reserve or ring_full_size' > $O/tests.log 2>&1"
tail -3 $O/tests.log
G="REHEARSAL_PASSES=20 REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_LEAN=1,0"
step reh_copy bash -c "env $G REHEARSAL_OVERLAP=1 SMI_LOOPBACK_FUSED=1 timeout -k 10 300 python -u tools/rehearsal.py 8192 20 > $O/rehearsal_copy.jsonl 2> $O/rehearsal_copy.err"
step reh_transport bash -c "env $G REHEARSAL_OVERLAP=1 timeout -k 10 300 python -u tools/rehearsal.py 8192 20 > $O/rehearsal_transport.jsonl 2> $O/rehearsal_transport.err"
step reh_noprof bash -c "env $G REHEARSAL_OVERLAP=1 REHEARSAL_PROF=0 SMI_LOOPBACK_FUSED=1 timeout -k 10 300 python -u tools/rehearsal.py 8192 20 > $O/rehearsal_noprof.jsonl 2> $O/rehearsal_noprof.err"
cat $O/rehearsal_*.jsonl | python3 -c "import json,sys;[print(d['K'],d['exchange'],d['band_kernel'],d['prof'],d['ms_per_step_alone'],d['ms_per_step_interior_rank'],d['efficiency'],d['band_avg_ms'],d['interior_avg_ms']) for d in map(json.loads,sys.stdin)]"
step traces bash -c "env REH_K=20 REHEARSAL_ROUNDS=1 REHEARSAL_RESERVE=0 REHEARSAL_PASSES=20 SMI_LOOPBACK_FUSED=1 bash tools/gpu_trace_reh.sh $1/tr lean:REHEARSAL_LEAN=1 wide:REHEARSAL_LEAN=0 > $O/traces.log 2>&1"
grep '^{' $O/traces.log
step ovh bash -c "timeout -k 10 120 python -u tools/overhead_r04.py 20 > $O/ovh20.json 2> $O/ovh20.err"
cat $O/ovh20.json
step bench bash -c "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err"
python3 -c "import json;d=json.load(open('$O/bench_driver.json'));r=d['roofline'];print('bench',d['value'],r['kernel_avg_ms'],r['share_of_timed_region'],d['parity']['bit_exact'])"
step fake2 bash -c "timeout -k 10 300 python bench.py --gpus 2 --fake-host --steps 20 --warmup 5 --no-aux > $O/bench_fake2.json 2> $O/bench_fake2.err"
python3 -c "import json;d=json.load(open('$O/bench_fake2.json'));print('fake2',d['value'],d['parity'])"
echo ALLDONE
