#!/usr/bin/env python3
"""Timing experiment (rehearsal build): cost of the global-edge variant of
the K-step sweep.  Runs the 8192^2 single tile with every wave on the normal
path (SMI_EDGE_FORCE=0), all waves on the edge variant (1) and none (2; wrong
results at the edges, timing only), and prints ms per step for each."""
import json
import os
import sys
import time

os.environ["SMI_LIB_VARIANT"] = "rehearsal"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import smi_amd  # noqa: E402
from smi_amd import stencil  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    steps = 120
    smi_amd.load(build_if_missing=False)
    comm = smi_amd.LocalGroup(1).comm(0)
    t = torch.rand((n, n), device="cuda")
    sc = torch.empty_like(t)
    s = torch.cuda.Stream()
    for force in (0, 1, 2, 0):
        os.environ["SMI_EDGE_FORCE"] = str(force)
        best = 1e9
        with torch.cuda.stream(s):
            stencil.run(comm, t, 24, 1, 1, sc)
            s.synchronize()
            for _ in range(5):
                t0 = time.perf_counter()
                stencil.run(comm, t, steps, 1, 1, sc)
                s.synchronize()
                best = min(best, (time.perf_counter() - t0) / steps * 1e3)
        print(json.dumps({"edge_force": force, "tile": n, "ms_per_step": round(best, 5),
                          "GCell_s": round(n * n / best / 1e6, 1)}), flush=True)
    os.environ.pop("SMI_EDGE_FORCE")
    comm.finalize()


if __name__ == "__main__":
    main()
