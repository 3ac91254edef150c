"""Per-variant median / min of the interleaved deepbench runs."""
import collections
import json
import statistics
import sys

runs = collections.defaultdict(list)
for line in open(sys.argv[1]):
    d = json.loads(line)
    runs[d["variant"]].append(d["ms_med"])
for v, ms in runs.items():
    print(f"{v:10s} n={len(ms)} med={statistics.median(ms):.5f} min={min(ms):.5f} max={max(ms):.5f}")
