#!/bin/bash
# pmc_bytes.sh OUTDIR variant... : HBM bytes per sweep dispatch (FETCH_SIZE,
# WRITE_SIZE: one rocprofv3 pass each), corrected as MI355X_MICROARCH.md
# prescribes for gfx950 (FETCH_SIZE in KiB, doubled for 16-B/lane streaming
# reads; WRITE_SIZE in KiB, exact)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/$1; shift; mkdir -p $out
for v in "$@"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $out/${v}_$c -o run -- $GRAFT_REPO_ROOT/tools/xbench/bin/xbench_$v 8192 10 10 > $out/${v}_$c.log 2>&1
    rc=$?; echo "$v $c rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $out/${v}_$c.log; exit $rc; fi
  done
done
python3 - "$out" "$@" <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
for v in sys.argv[2:]:
    res = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        per = collections.defaultdict(float)
        for f in glob.glob(f"{out}/{v}_{c}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "sweep" in r.get("Kernel_Name", "") and r["Counter_Name"] == c:
                    per[r.get("Dispatch_Id")] += float(r["Counter_Value"])
        vals = sorted(per.values())
        res[c] = vals[len(vals) // 2] if vals else None
    f, w = res["FETCH_SIZE"], res["WRITE_SIZE"]
    mb = lambda kib: round(kib * 1024 / 1e6, 1) if kib else None
    print(json.dumps({"variant": v, "fetch_MB_raw": mb(f), "fetch_MB": mb(2 * f) if f else None, "write_MB": mb(w),
                      "hbm_MB": mb(2 * f + w) if f and w else None}))
PY
