#!/bin/bash
# clock.sh OUTDIR variant : GPU clock during the sweep -- GRBM_GUI_ACTIVE /
# GRBM_COUNT per dispatch with the dispatch's own kernel-trace duration
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/$1; v=$2; mkdir -p $out
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $out/$v -o run -- $GRAFT_REPO_ROOT/tools/xbench/bin/xbench_$v 8192 20 20 > $out/$v.log 2>&1 || { tail -3 $out/$v.log; exit 1; }
python3 - "$out/$v" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
cnt = collections.defaultdict(dict); dur = {}
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "sweep" in r.get("Kernel_Name", ""):
            cnt[r["Dispatch_Id"]][r["Counter_Name"]] = cnt[r["Dispatch_Id"]].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "sweep" in r.get("Kernel_Name", ""):
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
rows = [(k, v, dur.get(k)) for k, v in cnt.items() if dur.get(k)]
for k, v, t in rows[-5:]:
    print({"dispatch": k, "ms": round(t * 1e3, 4), **{c: x for c, x in v.items()},
           "GUI_ACTIVE_GHz": round(v.get("GRBM_GUI_ACTIVE", 0) / t / 1e9, 3), "GRBM_COUNT_GHz": round(v.get("GRBM_COUNT", 0) / t / 1e9, 3)})
PY
