"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` (run here, no GPU): oracle vs golden fixtures / the reference's compiled dense path,
host logic, the C-ABI library loads and exports every symbol of include/nfft4gp_amd.h, gloo ranks.
`-m gpu` (MI355X): parity of the HIP path against the oracle through the C ABI.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.init()
    return torch
