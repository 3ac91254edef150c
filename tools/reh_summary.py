#!/usr/bin/env python3
"""One line per rehearsal setting of a gpu_bands.sh output directory:
exchange model, rounds, band placement, overlap, us/step of the interior rank
and of the lone tile measured right before it, efficiency.
  reh_summary.py gpurun_out/<tag>"""
import json
import os
import sys

d = sys.argv[1]
for f in ("fused", "noxchg", "transport"):
    p = os.path.join(d, f"rehearsal_{f}.jsonl")
    if not os.path.exists(p):
        continue
    for line in open(p):
        r = json.loads(line)
        print(f"{f:9s} rounds {r['rounds']} cus {r.get('band_cus', 0):2d} fusion {r.get('band_fusion')} "
              f"ov {r['overlap']} {'NOBANDS ' if r.get('no_bands') else ''}loop {r['ms_per_step_interior_rank'] * 1e3:6.2f} us/step "
              f"alone {r['ms_per_step_alone'] * 1e3:6.2f} eff {r['efficiency']:.4f}")
