"""Quadrature probes in pairs (krylov.hip lanczos_pair_dev): Nfft4GPLanczosQuadratureLogdet on this
library's additive operator runs caller-given probes two at a time, sharing each Lanczos step's matvec
through the two-vector interpolation.  Per-step printing (print_level 1) keeps the one-probe-at-a-time
loop, so the two paths are compared directly: loss and gradient to 1e-10 (the two-vector kernels sum in
another order: rounding-level differences), for an even and an odd probe count."""
import contextlib
import os

import numpy as np
import pytest

import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def quiet_stdout():
    fd = os.dup(1)
    null = os.open(os.devnull, os.O_WRONLY)
    os.dup2(null, 1)
    try:
        yield
    finally:
        os.dup2(fd, 1)
        os.close(null)
        os.close(fd)


@pytest.mark.parametrize("nvecs", [4, 5])
def test_paired_probes_equal_sequential(torch_cuda, nvecs):
    n, d, maxits = 30000, 8, 25
    rng = np.random.default_rng(nvecs)
    X = np.asfortranarray(rng.random((n, d)))
    y = rng.random(n) - 0.5
    win = np.arange(d, dtype=np.int32)
    R = np.asfortranarray(np.where(rng.random((n, nvecs)) < 0.5, -1.0, 1.0))
    op = amd.NFFTAdditiveKernel(X, win, d, 1)
    hyper = (1.0, 0.1, 0.05)
    loss_p, grad_p = amd.gp_loss(X, win, d, 1, y, hyper, maxits=maxits, nvecs=nvecs, rademacher=R, transform=3,
                                 op=op, print_level=-1)
    with quiet_stdout():
        loss_s, grad_s = amd.gp_loss(X, win, d, 1, y, hyper, maxits=maxits, nvecs=nvecs, rademacher=R,
                                     transform=3, op=op, print_level=1)
    assert np.isfinite(loss_p)
    assert loss_p == pytest.approx(loss_s, rel=1e-10)
    np.testing.assert_allclose(grad_p, grad_s, rtol=1e-9, atol=1e-12)
