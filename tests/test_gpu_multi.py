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
