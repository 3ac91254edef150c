#!/bin/bash
# Round-4 final GPU pass into gpurun_out/<tag>: every -m gpu test + smoke,
# both bench lines, then bench --gpus 4 / 8 --fake-host with parity.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
# a fresh box pages the image in at the first import torch (1-2 min without
# output): once, printing around it, before pytest's quiet collection
echo "=== warm"
timeout -k 10 300 python -u -c 'print("importing torch", flush=True); import torch; print("torch", flush=True); torch.zeros(1).cuda(); import smi_amd; smi_amd.load(build_if_missing=False); print("warm", flush=True)' || exit 1
bash tools/gpu_tests.sh $T || exit $?
TESTS=none bash tools/gpu_r04.sh $T || exit $?
O=gpurun_out/$T
for n in 4 8; do
  echo "=== fake$n"
  timeout -k 10 500 python bench.py --gpus $n --fake-host --steps 20 --warmup 5 --no-aux > $O/bench_fake$n.json 2> $O/bench_fake$n.err
  rc=$?; if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; grep -v amdgpu.ids $O/bench_fake$n.err | tail -5; exit $rc; fi
  python3 -c "import json;d=json.load(open('$O/bench_fake$n.json'));print('fake$n',d['value'],d['config']['decomposition'],d['parity']['bit_exact'],d['parity']['cells'])"
done
echo ALLDONE
