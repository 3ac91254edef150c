#!/bin/bash
# ab.sh OUTDIR rounds variant[:ENV=..]... : alternate xbench variants (bit check + timing)
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; rounds=$2; shift 2
mkdir -p $out
for r in $(seq $rounds); do
  for spec in "$@"; do
    v=${spec%%:*}; e=""; [ "$v" != "$spec" ] && e=${spec#*:}
    env $e timeout -k 10 60 tools/xbench/bin/xbench_$v 8192 100 200 >> $out/ab.jsonl 2>> $out/ab.err; rc=$?
    if [ $rc -ne 0 ]; then echo "$spec rc=$rc"; tail -3 $out/ab.err; exit 1; fi
  done
done
python3 - $out/ab.jsonl <<'PY'
import json, sys, collections
res = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l); res[(d["variant"], d["kernel"], d.get("wcone"), d.get("fo"))].append((d["ms_med"], d["ms_min"], d["mismatches"]))
for k, v in res.items():
    print(k, "med", sorted(x[0] for x in v), "min", min(x[1] for x in v), "mismatches", max(x[2] for x in v))
PY
