#!/usr/bin/env python3
"""Summarise rocprofv3 outputs into profiles/.

  pmc_summarize.py kt   <kernel_stats.csv> <out.json>
  pmc_summarize.py driver <kernel_stats.csv> <command> <out.json>
  pmc_summarize.py pmc  <fetch_counter_collection.csv> <write_counter_collection.csv> <cells> <out.json> [K]

With K >= 3 only the dispatches of sweepk_kernel<K> (K > 12: sweepd_kernel<K>) count, and the result is
merged into <out.json>'s "entries" (one per steps-per-launch), which is what
bench.py looks its roofline traffic up in.

HBM bytes per launch follow MI355X_MICROARCH.md "HBM": FETCH_SIZE/WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE counts half the bytes of a wide (16 B/lane)
coalesced streaming read, so it is doubled; WRITE_SIZE is exact for 16-B
streaming stores.
"""
import csv
import json
import sys

KERNEL = "sweep"  # matches sweep_kernel, sweep2_kernel and sweepk_kernel


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def counter_per_dispatch(path, name, kernel=KERNEL):
    vals = {}
    for r in rows(path):
        kn = r.get("Kernel_Name") or r.get("KernelName") or ""
        if kernel not in kn or "smi::" not in kn:
            continue
        if r.get("Counter_Name") != name:
            continue
        did = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[did] = vals.get(did, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    mode = sys.argv[1]
    if mode == "driver":
        # per-kernel averages of a --kernel-trace --stats run of `command`
        # (bench.py cites them next to its own HIP-event timing)
        ks = {}
        for r in rows(sys.argv[2]):
            name = r["Name"]
            short = name.split("(")[0].replace("void ", "").replace("smi::", "").strip()
            ks[short] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) * 1e-6,
                         "min_ms": float(r["MinNs"]) * 1e-6, "max_ms": float(r["MaxNs"]) * 1e-6,
                         "total_ms": float(r["TotalDurationNs"]) * 1e-6}
        json.dump({"command": sys.argv[3], "source": sys.argv[2], "kernels": ks}, open(sys.argv[4], "w"), indent=1)
        return
    if mode == "kt":
        out = []
        for r in rows(sys.argv[2]):
            out.append({k: r[k] for k in r})
        json.dump(out, open(sys.argv[3], "w"), indent=1)
        return
    cells = int(sys.argv[4])
    steps_per_launch = int(sys.argv[6]) if len(sys.argv) > 6 else 1
    kname = "sweepd_kernel" if steps_per_launch > 12 else "sweepk_kernel"  # K > 12: stencild.h
    kern = f"{kname}<{steps_per_launch}>" if steps_per_launch >= 3 else KERNEL
    fetch = counter_per_dispatch(sys.argv[2], "FETCH_SIZE", kern)
    write = counter_per_dispatch(sys.argv[3], "WRITE_SIZE", kern)
    f = sorted(fetch)[len(fetch) // 2]
    w = sorted(write)[len(write) // 2]
    d = {
        "kernel": {1: "sweep_kernel", 2: "sweep2_kernel"}.get(steps_per_launch, f"{kname}<{steps_per_launch}>"),
        "cells": cells,
        "dispatches": [len(fetch), len(write)],
        "FETCH_SIZE_KiB_median": f,
        "WRITE_SIZE_KiB_median": w,
        "read_bytes_corrected": 2 * f * 1024,
        "write_bytes": w * 1024,
        "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024,
        "steps_per_launch": steps_per_launch,
        "compulsory_bytes_per_launch": 8 * cells,
        "traffic_over_compulsory": round((2 * f * 1024 + w * 1024) / (8 * cells), 4),
        "cell_step_bytes_per_launch": 8 * cells * steps_per_launch,
        "source": [sys.argv[2], sys.argv[3]],
        "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 counts half of wide coalesced reads); "
                "compulsory = every cell read once and written once per pass",
    }
    try:
        old = json.load(open(sys.argv[5]))
    except (OSError, ValueError):
        old = {}
    entries = old.get("entries", [old] if "steps_per_launch" in old else [])
    entries = [e for e in entries if not (e.get("cells") == cells and e.get("steps_per_launch") == steps_per_launch)]
    entries.append(d)
    entries.sort(key=lambda e: (e["cells"], -e["steps_per_launch"]))
    json.dump({"entries": entries}, open(sys.argv[5], "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
