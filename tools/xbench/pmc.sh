#!/bin/bash
# pmc.sh OUTDIR variant... : instruction-cache and SQ counters of xbench
# variants, one rocprofv3 pass per counter group, summarised per kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/$1; shift; mkdir -p $out
for v in "$@"; do
  for grp in "ic:SQC_ICACHE_HITS SQC_ICACHE_MISSES" "if:SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH" \
             "sq:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES"; do
    g=${grp%%:*}; c=${grp#*:}
    timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $out/${v}_$g -o run -- $GRAFT_REPO_ROOT/tools/xbench/bin/xbench_$v 8192 10 10 > $out/${v}_$g.log 2>&1
    rc=$?; echo "$v $g rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $out/${v}_$g.log; exit $rc; fi
  done
done
python3 - "$out" "$@" <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
for v in sys.argv[2:]:
    tot = collections.defaultdict(float); n = collections.defaultdict(set)
    for f in glob.glob(f"{out}/{v}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            kn = r.get("Kernel_Name", "")
            if "sweep" not in kn: continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r.get("Dispatch_Id"))
    per = {k: tot[k] / max(1, len(n[k])) for k in tot}
    print(json.dumps({"variant": v, "per_dispatch": {k: round(x) for k, x in sorted(per.items())},
                      "icache_miss_rate": round(per.get("SQC_ICACHE_MISSES", 0) / max(1, per.get("SQC_ICACHE_HITS", 0) + per.get("SQC_ICACHE_MISSES", 0)), 4)}))
PY
