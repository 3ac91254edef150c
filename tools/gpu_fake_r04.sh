#!/bin/bash
# bench.py --gpus 4 / 8 --fake-host (RCCL over sockets on one GPU) with the
# parity check of the timed plan on every rank's light cone, into
# gpurun_out/<tag>.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
# a fresh box pages the image in at the first import torch (1-2 min, no
# output): do it once, in one process, before four or eight at a time
echo "=== warm"
timeout -k 10 300 python -u -c 'import torch; print("torch", flush=True); torch.zeros(1).cuda(); import smi_amd; smi_amd.load(); print("warm", flush=True)' || exit 1
echo "=== band tests"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_stencil_gpu.py -k 'band_kernel_choice or ring_decomposed or ring_band_reserve' > $O/band_tests.log 2>&1 || { tail -20 $O/band_tests.log; exit 1; }
tail -1 $O/band_tests.log
for n in 4 8; do
  echo "=== fake$n"
  timeout -k 10 500 python bench.py --gpus $n --fake-host --steps 20 --warmup 5 --no-aux > $O/bench_fake$n.json 2> $O/bench_fake$n.err
  rc=$?; if [ $rc -ne 0 ]; then echo "=== FAILED rc=$rc"; tail -5 $O/bench_fake$n.err; exit $rc; fi
  python3 -c "import json;d=json.load(open('$O/bench_fake$n.json'));print('fake$n',d['value'],d['config']['decomposition'],d['parity'])"
done
echo ALLDONE
