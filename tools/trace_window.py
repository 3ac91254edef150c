#!/usr/bin/env python3
"""Average duration of the timed-region launches of a kernel from a rocprofv3
kernel trace, next to the HIP-event average the bench line reports.

  trace_window.py <run_kernel_trace.csv> <bench.json> <out.json> [kernel-substring]

bench.py's timed region is its last steps/K launches of the K-step sweep
(the warm-up launches come first); rocprofv3 --stats averages over all
launches, cold-clock warm-up included, so this picks the timed window."""
import csv
import json
import sys


def main():
    trace, bench, out = sys.argv[1:4]
    key = sys.argv[4] if len(sys.argv) > 4 else "sweepk_kernel"
    with open(bench) as f:
        line = [ln for ln in f if ln.startswith('{"metric"')][-1]
    b = json.loads(line)
    n = int(b["roofline"]["launches"])
    with open(trace) as f:
        d = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(f)
                   if key in r["Kernel_Name"])
    win = [(e - s) / 1e6 for s, e in d[-n:]] if n else []
    res = {"kernel": key, "launches_in_trace": len(d), "timed_launches": n,
           "rocprof_avg_ms_timed_window": round(sum(win) / max(len(win), 1), 5),
           "rocprof_avg_ms_all_launches": round(sum((e - s) / 1e6 for s, e in d) / max(len(d), 1), 5),
           "bench_hip_event_avg_ms": b["roofline"]["kernel_avg_ms"],
           "bench_value": b["value"], "bench_ms_per_step": b["ms_per_step"]}
    res["agreement"] = round(res["rocprof_avg_ms_timed_window"] / res["bench_hip_event_avg_ms"], 4)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
