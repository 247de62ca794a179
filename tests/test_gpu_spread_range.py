"""Spread variant 2 (nfft_kernels.hip k_spread_range): workgroups over ranges of consecutive blocks, the
moment table accumulated over the range and folded once.  The moments are sums over points whatever their
block, so the matvec, the gradient matvec and PCG's fused-dot path equal the default spread's up to the
order of the LDS adds (1e-13 relative), for ragged last ranges and a row shard."""
import numpy as np
import pytest

import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / np.linalg.norm(np.asarray(b)))


@pytest.mark.parametrize("bpr", ["1", "3", "4", "7"])
def test_range_spread_matches_default(torch_cuda, monkeypatch, bpr):
    torch = torch_cuda
    rng = np.random.default_rng(int(bpr))
    n, d = 120000, 9  # B = 2032: 60 blocks, ragged last range for bpr 7
    X = rng.random((n, d))
    win = np.arange(d, dtype=np.int32)
    xd = torch.tensor(rng.random(n) - 0.5, device="cuda")
    ref = amd.NFFTAdditiveKernel(X, win, d, 1)
    assert ref.setup(amd.GAUSSIAN, 1.0, 0.2, 0.01) == 0
    y0, g0 = ref.matsymv(xd).cpu().numpy(), ref.gradmatsymv(xd).cpu().numpy()
    monkeypatch.setenv("NFFT4GP_AMD_SPREAD_VARIANT", "2")
    monkeypatch.setenv("NFFT4GP_AMD_SPREAD_BPR", bpr)
    op = amd.NFFTAdditiveKernel(X, win, d, 1)
    assert op.setup(amd.GAUSSIAN, 1.0, 0.2, 0.01) == 0
    assert rel(op.matsymv(xd).cpu().numpy(), y0) < 1e-13
    assert rel(op.gradmatsymv(xd).cpu().numpy(), g0) < 1e-13
    # PCG (fused (q, p) dot in the interpolation) takes the default spread's iterations within a few
    b = torch.tensor(rng.random(n) - 0.5, device="cuda")
    x1, x2 = torch.zeros_like(b), torch.zeros_like(b)
    _, _, _, it1 = amd.pcg(ref, b, x1, maxits=2000, tol=1e-6)
    _, _, _, it2 = amd.pcg(op, b, x2, maxits=2000, tol=1e-6)
    assert it1 > 0 and it2 > 0 and abs(it1 - it2) <= max(3, it1 // 20)
    # a row shard's spread + k_reduce_parts over the ranges' partial grids
    sh = amd.NFFTAdditiveKernel(X, win, d, 1, shard=(0, n // 3))
    assert sh.setup(amd.GAUSSIAN, 1.0, 0.2, 0.01) == 0
    monkeypatch.delenv("NFFT4GP_AMD_SPREAD_VARIANT")
    sh0 = amd.NFFTAdditiveKernel(X, win, d, 1, shard=(0, n // 3))
    assert sh0.setup(amd.GAUSSIAN, 1.0, 0.2, 0.01) == 0
    gsz = sh.shard_grid_size()
    xs = torch.tensor(np.asarray(xd.cpu().numpy()[: n // 3]), device="cuda")
    ga = sh.shard_spread(xs, torch.zeros(gsz, dtype=torch.float64, device="cuda")).cpu().numpy()
    gb = sh0.shard_spread(xs, torch.zeros(gsz, dtype=torch.float64, device="cuda")).cpu().numpy()
    assert rel(ga, gb) < 1e-13
