#!/usr/bin/env python3
"""Short driver for rocprofv3 counter passes on the K-step sweep: warm-up,
then `passes` launches of K steps on an N x N tile (one launch per pass).

    python tools/pmc_sweep.py [N] [K] [passes]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import smi_amd  # noqa: E402
from smi_amd import stencil  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
k = int(sys.argv[2]) if len(sys.argv) > 2 else 12
passes = int(sys.argv[3]) if len(sys.argv) > 3 else 10
smi_amd.load()
comm = smi_amd.LocalGroup(1).comm(0)
a = torch.rand((n, n), device="cuda")
b = torch.empty_like(a)
stencil.set_fusion(k, -1)
stencil.run(comm, a, k * passes, 1, 1, b)
torch.cuda.synchronize()
comm.finalize()
print("ok", n, k, passes)
