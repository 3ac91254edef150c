#!/bin/bash
# the round-2 (344fd23) and round-3 (749c50d) trees, built
# in ab/r02 and ab/r03 (git worktrees), benched alternately on one box with
# the driver's flags, 3 runs each, plus the round-4 tree.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1; mkdir -p $O
for i in 1 2 3; do
  for t in r02 r03 r04; do
    d=$R/ab/$t; [ $t = r04 ] && d=$R
    (cd $d && timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-aux --no-cpu-baseline $([ $t = r04 ] && echo --no-parity) > $O/${t}_$i.json 2> $O/${t}_$i.err) || { echo "$t run $i failed"; tail -5 $O/${t}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${t}_$i.json'));r=d['roofline'];print('$t',$i,d['value'],d['ms_per_step'],r['kernel_avg_ms'],r['launches'])"
  done
done
