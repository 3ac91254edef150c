#!/bin/bash
# big.sh OUTDIR : the K = 20 pass on one 16384^2 tile (1 GiB per buffer: the
# 256 MiB Infinity Cache cannot hold it) -- timing + bit check, then HBM
# bytes per dispatch (FETCH_SIZE / WRITE_SIZE passes), next to 8192^2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $out
for n in 16384 8192; do
  timeout -k 10 120 tools/xbench/bin/xbench_d20 $n 40 40 >> $out/time.jsonl 2>> $out/time.err || exit 1
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $out/n${n}_$c -o run -- $GRAFT_REPO_ROOT/tools/xbench/bin/xbench_d20 $n 5 5 > $out/n${n}_$c.log 2>&1
    rc=$?; echo "$n $c rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $out/n${n}_$c.log; exit $rc; fi
  done
done
cat $out/time.jsonl
python3 - "$out" <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
for n in (16384, 8192):
    res = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        per = collections.defaultdict(float)
        for f in glob.glob(f"{out}/n{n}_{c}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "sweep" in r.get("Kernel_Name", "") and r["Counter_Name"] == c:
                    per[r.get("Dispatch_Id")] += float(r["Counter_Value"])
        vals = sorted(per.values()); res[c] = vals[len(vals) // 2] if vals else None
    f, w = res["FETCH_SIZE"], res["WRITE_SIZE"]
    mb = lambda kib: round(kib * 1024 / 1e6, 1)
    comp = 8 * n * n / 1e6
    print(json.dumps({"n": n, "fetch_MB": mb(2 * f), "write_MB": mb(w), "hbm_MB": mb(2 * f + w), "compulsory_MB": comp,
                      "hbm_over_compulsory": round((2 * f + w) * 1024 / 1e6 / comp, 3)}))
PY
