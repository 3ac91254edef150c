#!/bin/bash
# element-channel throughput (C host, in-process transport) + a short bench with the new aux lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 240 tools/chanbench/chanbench 1000000 > $O/chanbench.jsonl 2> $O/chanbench.err || { echo "chanbench rc=$?"; tail $O/chanbench.err; exit 1; }
cat $O/chanbench.jsonl
timeout -k 10 300 python bench.py --steps 240 --warmup 24 > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], json.dumps(d['aux'].get('kernels')))"
