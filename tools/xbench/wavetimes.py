"""Summarise xbench per-wave stamps (SMI_X_WAVETIMES builds).

    python tools/xbench/wavetimes.py profiles/r05/xbench/wavetimes_clock_u_fo128.csv.gz ...

Each row is one wave of the last launch: its hardware place (XCC, SE, SH, CU,
SIMD, wave slot from HW_ID), the shader-clock cycle counter at the start and
end of its walk and, in the sweepu builds, the 100 MHz real-time counter at
both ends.  Per SIMD the two resident waves are split into the one with the
lower wave slot (dispatched first) and the other; the real-time stamps give
the shader clock each wave ran at (cycles / seconds).
"""
import sys

import pandas as pd


def summary(path: str) -> dict:
    d = pd.read_csv(path)
    d = d[d.end > 0].copy()
    d["cyc"] = d.end - d.start
    out = {"file": path, "waves": len(d)}
    key = ["xcc", "se", "sh", "cu", "simd"]
    first, second, span = [], [], []
    for _, s in d.groupby(key):
        if len(s) != 2:
            continue
        s = s.sort_values("wave_slot")
        first.append(s.iloc[0].cyc)
        second.append(s.iloc[1].cyc)
        span.append(max(s.end) - min(s.start))
    out["simds_with_two_waves"] = len(span)
    out["walk_kcycles_slot0_median"] = round(pd.Series(first).median() / 1e3, 1)
    out["walk_kcycles_slot1_median"] = round(pd.Series(second).median() / 1e3, 1)
    out["simd_span_kcycles_median"] = round(pd.Series(span).median() / 1e3, 1)
    out["simd_span_kcycles_max"] = round(max(span) / 1e3, 1)
    if "rstart" in d:
        rt = (d.rend - d.rstart) * 10e-9  # 100 MHz
        ghz = d.cyc / rt / 1e9
        out["clock_GHz_median"] = round(float(ghz.median()), 3)
        out["clock_GHz_min"] = round(float(ghz.min()), 3)
        out["clock_GHz_max"] = round(float(ghz.max()), 3)
        out["walk_us_median"] = round(float(rt.median()) * 1e6, 1)
        out["launch_walks_us"] = round((d.rend.max() - d.rstart.min()) * 0.01, 1)
    return out


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(summary(p))
