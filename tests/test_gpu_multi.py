"""Nfft4GPAmdAdditiveMatSymvMulti: the additive matvec on several device vectors, two per pass of the
interpolation over the layout (nfft_kernels.hip k_interp2).  Each column equals the single-vector
Nfft4GPAdditiveNFFTMatSymv to the matvec's run-to-run rounding (LDS atomics: 1e-13 relative), for an even
and an odd count, beta != 0, and multi-feature windows (served one vector at a time)."""
import ctypes as C

import numpy as np
import pytest

import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
from preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nv,nw,dw,beta,n", [(4, 16, 1, 0.0, 30000), (5, 16, 1, 0.7, 30000), (3, 2, 3, 0.0, 30000),
                                             (2, 9, 1, 0.0, 100000)],
                         ids=["even", "odd_beta", "md", "b2032"])
def test_multi_matches_single(torch_cuda, nv, nw, dw, beta, n):
    """Each column equals the single-vector matvec to 1e-15 (relative): the same spread per vector, and the
    two-vector interpolation adds in LDS with ds_add_f64 in the wave order."""
    import torch

    d = nw * dw
    rng = np.random.default_rng(nv)
    X = np.asfortranarray(rng.random((n, d)))
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), nw, dw)
    assert op.setup(amd.GAUSSIAN, f=1.1, l=0.3, mu=0.02) == 0
    if dw == 1:
        op.set_deterministic(True)  # the columns are then compared bit for bit below
    V = torch.tensor(rng.random((nv, n)) - 0.5, device="cuda")
    Y0 = torch.tensor(rng.random((nv, n)), device="cuda")
    Y1 = Y0.clone()
    Y2 = Y0.clone()
    for v in range(nv):
        op.matsymv(V[v], 1.3, beta, Y1[v])
    L = _lib.lib()
    assert L.Nfft4GPAmdAdditiveMatSymvMulti(op.h, n, nv, 1.3, V.data_ptr(), n, beta, Y2.data_ptr(), n) == 0
    torch.cuda.synchronize()
    rel = ((Y1 - Y2).norm(dim=1) / Y1.norm(dim=1)).max().item()
    assert rel < 1e-15, rel
    if dw == 1:  # the deterministic 1-D matvec: the columns are the single-vector matvecs bit for bit
        assert torch.equal(Y1, Y2)
    # host arrays and a short leading dimension are refused
    h = np.zeros(n)
    assert L.Nfft4GPAmdAdditiveMatSymvMulti(op.h, n, 1, 1.0, h.ctypes.data, n, 0.0, h.ctypes.data, n) != 0
    assert L.Nfft4GPAmdAdditiveMatSymvMulti(op.h, n, 2, 1.0, V.data_ptr(), n - 1, 0.0, Y2.data_ptr(), n) != 0


def test_multi_past_the_infinity_cache_is_bitwise(torch_cuda):
    """A layout past the 256 MB Infinity Cache (n = 4e6, 64 windows: ~1.4 GB): the single-vector matvec takes
    k_interp_hl (H rows staged in LDS) and the pair k_interp2; in deterministic mode both equal k_interp's bits."""
    import torch

    n, d = 4_000_000, 64
    rng = np.random.default_rng(41)
    X = rng.random((n, d))
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    del X
    assert op.setup(amd.GAUSSIAN, f=1.0, l=0.5, mu=0.01) == 0
    op.set_deterministic(True)
    V = torch.tensor(rng.random((2, n)) - 0.5, device="cuda")
    Y1 = torch.empty_like(V)
    Y2 = torch.empty_like(V)
    for v in range(2):
        op.matsymv(V[v], 0.9, 0.0, Y1[v])
    L = _lib.lib()
    assert L.Nfft4GPAmdAdditiveMatSymvMulti(op.h, n, 2, 0.9, V.data_ptr(), n, 0.0, Y2.data_ptr(), n) == 0
    torch.cuda.synchronize()
    assert torch.equal(Y1, Y2)
