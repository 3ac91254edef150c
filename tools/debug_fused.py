#!/usr/bin/env python3
"""Fused (two-step) multi-rank stencil: run cases in increasing complexity,
one process, stop at the first failure (diagnostic)."""
import os
import ctypes
import sys

os.environ.setdefault("SMI_LIB_VARIANT", "debug")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
import smi_amd  # noqa: E402
from smi_amd import stencil  # noqa: E402


def run(g, T, PX, PY, overlap):
    stencil.set_tuning(overlap=overlap)
    tiles = stencil.split_memory(g, PX, PY)

    def fn(comm):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            t = torch.from_numpy(tiles[comm.rank]).cuda()
            res = stencil.run(comm, t, T, PX, PY)
            s.synchronize()
            return res.cpu().numpy()

    return stencil.combine_memory(smi_amd.LocalGroup(PX * PY).run(fn), PX, PY)


def main():
    smi_amd.load()
    stencil.set_fusion(2)
    for PX, PY in ((2, 1), (1, 2), (2, 2)):
        for overlap in (0, 1):
            for T in (1, 2, 3, 4, 5):
                g = oracle.init_uniform(64 * PX, 128 * PY, seed=PX * 7 + PY)
                print(f"case {PX}x{PY} overlap={overlap} T={T} ...", flush=True)
                got = run(g, T, PX, PY, overlap)
                ok = np.array_equal(got.view(np.uint32), oracle.stencil(g, T).view(np.uint32))
                flags = ctypes.c_uint()
                if os.environ.get("SMI_LIB_VARIANT") == "debug":
                    smi_amd.load().smi_debug_oob(ctypes.byref(flags))
                print(f"   -> {'OK' if ok else 'MISMATCH'} oob_flags=0x{flags.value:x}", flush=True)
                if flags.value:
                    return 2
                if not ok:
                    bad = np.argwhere(got != oracle.stencil(g, T))
                    print("   first bad cells:", bad[:10].tolist(), flush=True)
                    return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
