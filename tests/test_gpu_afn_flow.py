"""Nfft4GPPrecondAFNSetup's decision logic (afn.c:161-489, MATLAB afn_setup.m) in one entry point
(Nfft4GPAmdPrecondAFNSetup, VERDICT r01 item 5 / ADVICE r01):
* estimated rank below max_k -> the rank-k Nystrom on the estimated landmarks (afn.c:294-304);
* estimated rank == max_k    -> the AFN with that rank and order;
* the AFN's factors break down -> a Nystrom on the same order (MATLAB's RAN fallback, afn_setup.m:93-98).
Each branch's apply equals the one built directly from the same rank and order (the rank estimation
draws libc rand(); both runs start from the same srand seed)."""
import ctypes

import numpy as np
import pytest

import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd

pytestmark = pytest.mark.gpu
libc = ctypes.CDLL(None)


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(b), 1e-300))


def additive_problem(n=20000, d=8, l=0.1, mu=0.01, seed=3):
    X = np.random.default_rng(seed).random((n, d))
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    assert op.setup(amd.GAUSSIAN, f=1.0, l=l, mu=mu) == 0
    return X, op


def test_low_rank_additive_kernel_switches_to_nystrom(torch_cuda):
    """1-D additive windows are low rank (config B's Gram is rank deficient at 256): the flow
    builds the rank-k Nystrom the reference would, not an AFN."""
    torch = torch_cuda
    # l = 0.5: low rank (at l = 0.1 the estimate reaches 256)
    X, op = additive_problem(l=0.5, mu=0.1)
    n = X.shape[0]
    libc.srand(807)
    k_est, perm = amd.afn_rank_estimate(X, 256, perm_opt="random", op=op)
    libc.srand(807)
    pre = amd.PrecondAFN(X, 256, perm_opt="random", op=op)
    assert pre.k == k_est
    assert 0 < k_est < 256, k_est
    assert pre.kind == "nystrom"
    direct = amd.NystromPrecond.from_additive(op, perm, k_est, k11="landmarks")
    r = torch.tensor(np.random.default_rng(4).random(n), device="cuda")
    z1 = pre.solve(torch.zeros_like(r), r).cpu().numpy()
    z2 = direct.solve(torch.zeros_like(r), r).cpu().numpy()
    assert rel(z1, z2) < 1e-12
    direct.free()
    pre.free()
    op.free()


def test_full_rank_plain_kernel_builds_the_afn(torch_cuda):
    """A short length scale on 3-D points: the estimate reaches max_k, so the AFN itself is built, equal to
    Nfft4GPAmdAfnSetupSchur with the estimated order."""
    torch = torch_cuda
    n, d, max_k = 6000, 3, 64
    X = np.random.default_rng(11).random((n, d))
    f, l, mu = 1.0, 0.05, 0.01
    libc.srand(99)
    k_est, perm = amd.afn_rank_estimate(X, max_k, f, l, mu, perm_opt="fps")
    assert k_est == max_k
    libc.srand(99)
    pre = amd.PrecondAFN(X, max_k, f, l, mu, perm_opt="fps", schur_lfil=20)
    assert pre.kind == "afn" and pre.k == max_k
    direct = amd.AfnPrecond.setup(X, max_k, f, l, mu, perm_opt="perm", perm=perm, schur_lfil=20)
    r = torch.tensor(np.random.default_rng(12).random(n), device="cuda")
    z1 = pre.solve(torch.zeros_like(r), r).cpu().numpy()
    z2 = direct.solve(torch.zeros_like(r), r).cpu().numpy()
    assert rel(z1, z2) < 1e-12
    direct.free()
    pre.free()


def test_predefined_rank_skips_estimation(torch_cuda):
    """max_k <= 0: rank -max_k in natural order, no estimation (afn.c:245-256), hence an AFN."""
    n, d = 3000, 3
    X = np.random.default_rng(21).random((n, d))
    pre = amd.PrecondAFN(X, -40, 1.0, 0.1, 0.01)
    assert pre.kind == "afn" and pre.k == 40
    k, perm, _ = amd.AfnPrecond.setup(X, 40, 1.0, 0.1, 0.01, perm_opt="identity").info()
    assert k == 40
    pre.free()


def test_breakdown_falls_back_to_nystrom(torch_cuda):
    """A11 = K11 + mu f^2 I with mu = -2 is indefinite, so the AFN's Cholesky breaks down; the flow then builds
    the Nystrom on the same order (MATLAB's RAN, afn_setup.m:93-98) instead of failing."""
    torch = torch_cuda
    X, op = additive_problem(n=4000, d=4, l=0.5, mu=-2.0)
    pre = amd.PrecondAFN(X, -48, op=op)
    assert pre.kind == "ran" and pre.k == 48
    direct = amd.NystromPrecond.from_additive(op, np.arange(X.shape[0], dtype=np.int32), 48, k11="landmarks")
    r = torch.tensor(np.random.default_rng(7).random(X.shape[0]), device="cuda")
    z1 = pre.solve(torch.zeros_like(r), r).cpu().numpy()
    z2 = direct.solve(torch.zeros_like(r), r).cpu().numpy()
    np.testing.assert_array_equal(np.isfinite(z1), np.isfinite(z2))
    ok = np.isfinite(z2)
    assert ok.any() and rel(z1[ok], z2[ok]) < 1e-12
    direct.free()
    pre.free()
    op.free()
