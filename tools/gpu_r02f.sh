#!/bin/bash
# Round-2: tuning table of the committed LDS-DMA sweep (K x row-block height)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02f
mkdir -p $O
timeout -k 10 300 python -u tools/tune_deep.py 8192 20 12,10,8,6 -1,64,82,100,127,145,199,289 > $O/tune_release.jsonl 2>&1 || { tail $O/tune_release.jsonl; exit 1; }
grep -v amdgpu.ids $O/tune_release.jsonl
