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
            kind = ("interior" if "sweepk_kernel" in name or "sweepk_fused_kernel" in name else "band" if "bandk_kernel" in name or "ringk" in name
                    else "xchg" if "copy" in name.lower() or "nccl" in name.lower() else None)
            if kind:
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind))
    ev.sort()
    ints = [e for e in ev if e[2] == "interior"]
    t0 = ints[-n][0] if len(ints) >= n else ev[0][0]
    print(f"{'kind':9s} {'start_us':>10s} {'end_us':>10s} {'dur_us':>8s}")
    for s, e, k in ev:
        if s >= t0 - 200_000:
            print(f"{k:9s} {(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f}")
    if len(ints) > 1:
        last = ints[-n:]
        per = (last[-1][1] - last[0][0]) / len(last) / 1e3
        print(f"interior pass period over the last {len(last)}: {per:.1f} us; "
              f"interior duration avg {sum(e - s for s, e, _ in last) / len(last) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
