#!/usr/bin/env python3
"""Per-pass timeline of a multi-rank (or loopback rehearsal) stencil run from a
rocprofv3 kernel trace: for the last N interior sweeps, when the band kernel
and the exchange ran relative to the interior of the same pass, and how long
each took (us).  Shows whether the bands overlap the interior or serialise.

  pass_timeline.py <run_kernel_trace.csv> [N]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    ev = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            kind = ("interior" if "sweepk_kernel" in name or "sweepd_kernel" in name or "sweepk_fused_kernel" in name
                    else "band" if "bandk_kernel" in name or "bandl_kernel" in name or "ringk" in name
                    else "xchg" if "copy" in name.lower() or "nccl" in name.lower() or "rccl" in name.lower() else None)
            if kind:
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind))
    ev.sort()
    ints = [e for e in ev if e[2] == "interior"]
    t0 = ints[-n][0] if len(ints) >= n else ev[0][0]
    print(f"{'kind':9s} {'start_us':>10s} {'end_us':>10s} {'dur_us':>8s}")
    for s, e, k in ev:
        if s >= t0 - 200_000:
            print(f"{k:9s} {(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f}")
    # each band / exchange launch against the interior it ran beside (the
    # one whose span contains its start): inside = it also ended before
    # that interior did
    import json
    rows = []
    for s, e, k in ev:
        if k == "interior" or s < t0:
            continue
        host = next((i for i in ints if i[0] <= s <= i[1]), None)
        rows.append((k, host is not None and e <= host[1], (e - host[1]) / 1e3 if host else None))
    def med(v):
        v = sorted(v)
        return round(v[len(v) // 2] / 1e3, 1) if v else None

    summ = {}
    for k in ("band", "xchg"):
        r = [x for x in rows if x[0] == k]
        if r:
            summ[k] = {"launches": len(r), "inside_interior": sum(1 for x in r if x[1]),
                       "max_overhang_us": round(max((x[2] for x in r if x[2] is not None), default=0.0), 1),
                       "duration_median_us": med([e - s for s, e, kk in ev if kk == k and s >= t0])}
    if len(ints) > 1:
        last = ints[-n:]
        per = (last[-1][1] - last[0][0]) / len(last) / 1e3
        durs = [e - s for s, e, _ in last]
        gaps = [b[0] - a[1] for a, b in zip(last, last[1:])]
        print(f"interior pass period over the last {len(last)}: {per:.1f} us; "
              f"interior duration avg {sum(durs) / len(last) / 1e3:.1f} us")
        summ["interior"] = {"period_us": round(per, 1), "passes": len(last),
                            "duration_avg_us": round(sum(durs) / len(last) / 1e3, 1),
                            "duration_median_us": med(durs), "duration_min_us": round(min(durs) / 1e3, 1),
                            "duration_max_us": round(max(durs) / 1e3, 1), "gap_median_us": med(gaps)}
    print(json.dumps(summ))


if __name__ == "__main__":
    main()
