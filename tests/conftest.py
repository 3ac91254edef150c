import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libsmi_amd.so)")


@pytest.fixture(scope="session")
def gpu():
    """The HIP library, loaded on a visible GPU.  On a GPU box a missing or
    broken library is an error, never a skip."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    import smi_amd
    lib = smi_amd.load()
    torch.cuda.set_device(0)
    return lib


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle
