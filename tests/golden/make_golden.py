#!/usr/bin/env python3
"""Generate the committed golden fixtures from the CPU oracle.

The reference holds no bit-level stencil/gesummv vectors, so the
fixtures are the oracle's outputs on the reference's own problem shapes
(config 1: 256x256, 32 steps, edge-ones init, PX=PY=2) and seeded variants;
the oracle itself is pinned by tests/test_oracle.py.  GPU tests compare the
HIP path against these hashes without re-running the oracle.
Run:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle as o  # noqa: E402

CASES = [
    dict(init="edges", X=256, Y=256, T=32, PX=2, PY=2),      # BASELINE config 1
    dict(init="edges", X=256, Y=256, T=32),
    dict(init="uniform", seed=42, X=256, Y=256, T=32),
    dict(init="uniform", seed=42, X=512, Y=1024, T=10, PX=2, PY=4),
    dict(init="uniform", seed=7, X=1000, Y=1028, T=5),
]


def main():
    out = {"generator": "tests/golden/make_golden.py (oracle/smi_oracle.c)", "stencil": []}
    for c in CASES:
        g = o.init_edges(c["X"], c["Y"]) if c["init"] == "edges" else o.init_uniform(c["X"], c["Y"], c["seed"])
        if c.get("PX", 1) * c.get("PY", 1) > 1:
            r = o.stencil_decomposed(g, c["T"], c["PX"], c["PY"])
        else:
            r = o.stencil(g, c["T"])
        out["stencil"].append(dict(c, sha256=hashlib.sha256(r.tobytes()).hexdigest()))
    arr = o.stencil(o.init_uniform(64, 96, seed=42), 16)
    np.save(os.path.join(HERE, "stencil_uniform_64x96_T16.npy"), arr)
    # reduce: canonical-fold results for seeded inputs, n in {2,4,8}
    red = []
    for n in (2, 4, 8):
        rng = np.random.default_rng(100 + n)
        c = ((rng.random((n, 64)) * 2 - 1) * 1000).astype(np.float32)
        red.append(dict(n=n, seed=100 + n, inputs=c.tolist(),
                        fp32_add=o.reduce(c, o.SMI_FLOAT, o.SMI_ADD).view(np.uint32).tolist()))
    out["reduce"] = red
    # kmeans_smi on the reference host's own input (its generator, 8 clusters
    # x 64 dims, W = 16, 8 ranks as SMI_KMEANS_RANKS) and a W = 1 variant
    km = []
    for case in (dict(num_points=2048, ranks=8, width=16, iterations=10),
                 dict(num_points=1536, ranks=3, width=1, iterations=6)):
        _, pts, cen = o.kmeans_reference_data(case["num_points"], 8, 64)
        c = o.kmeans(pts, cen, case["iterations"], ranks=case["ranks"], width=case["width"])
        km.append(dict(case, clusters=8, dims=64, sha256=hashlib.sha256(c.tobytes()).hexdigest(),
                       centroid0=c[0].tolist()))
    out["kmeans"] = km
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
