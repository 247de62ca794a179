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


# Under `pytest -m gpu -x` the hot path's oracle-parity files run first, so a failure in a peripheral
# test (the drop-in C link, a setup) cannot leave the north-star parity unreached. Files not listed
# keep their alphabetical order after these; test_dropin.py (compiles C, links oracle/_ref) runs last.
_FIRST = (
    "test_golden.py", "test_cpu_host.py",
    "test_gpu_configs.py", "test_gpu_golden.py", "test_gpu_nfft.py", "test_gpu_md.py",
    "test_gpu_dist.py", "test_gpu_layout.py", "test_gpu_multi.py", "test_gpu_solvers.py",
    "test_gpu_krylov.py", "test_gpu_dist_krylov.py", "test_gpu_slq_pairs.py",
)
_LAST = ("test_dropin.py",)


def _file_rank(item):
    name = os.path.basename(str(item.fspath))
    if name in _FIRST:
        return (0, _FIRST.index(name))
    if name in _LAST:
        return (2, _LAST.index(name))
    return (1, 0)


def pytest_collection_modifyitems(session, config, items):
    # stable sort: the order inside a file and among the middle files is unchanged
    items.sort(key=_file_rank)


@pytest.fixture(scope="session")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.init()
    return torch
