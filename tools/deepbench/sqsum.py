"""Median SQ counters per sweepd dispatch from a rocprofv3 --pmc CSV."""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if "sweep" in r["Kernel_Name"]:
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
ds = sorted(agg, key=int)[2:]
med = {n: statistics.median(agg[d][n] for d in ds) for n in agg[ds[0]]}
for n, v in sorted(med.items()):
    print(f"{n:24s} {v:14.0f}")
w = med.get("SQ_WAVE_CYCLES", 0)
if w:
    for n in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        print(f"{n}/WAVE_CYCLES = {med[n] / w:.3f}")
    print(f"VALU per wave = {med['SQ_INSTS_VALU'] / med['SQ_WAVES']:.0f}")
