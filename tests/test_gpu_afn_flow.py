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


def _dense_additive(X, f, l):
    """f^2 (1/nw) sum_w exp(-(x_w - y_w)^2 / (2 l^2)) over 1-D windows and its l-derivative (kernels.c:3099-3494
    with kernels.c:680-1289 per window)."""
    n, d = X.shape
    K = np.zeros((n, n))
    dKl = np.zeros((n, n))
    for w in range(d):
        r2 = (X[:, w:w + 1] - X[:, w][None, :]) ** 2
        e = np.exp(-r2 / (2 * l * l))
        K += e
        dKl += e * r2 / l ** 3
    return f * f * K / d, f * f * dKl / d


def test_gradients_at_k_equal_n_use_the_full_rank_nystrom(torch_cuda):
    """with require_grad the k = n branch (afn.c:263-272, M = K + mu f^2 I) used to fail the whole
    setup.  It is now the rank-n Nystrom with gradients (kind 4), which is that matrix: apply, logdet, trace
    and dvp against the dense kernel."""
    torch = torch_cuda
    n, d, f, l, mu = 300, 6, 1.2, 0.05, 0.05
    X = np.random.default_rng(31).random((n, d))
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    assert op.setup(amd.GAUSSIAN, f=f, l=l, mu=mu) == 0
    pre = amd.PrecondAFN(X, -n, op=op, require_grad=True)
    assert pre.kind == "nystrom_full" and pre.k == n
    K, dKl = _dense_additive(X, f, l)
    M = K + mu * f * f * np.eye(n)
    r = np.random.default_rng(32).random(n)
    z = pre.solve(torch.zeros(n, dtype=torch.float64, device="cuda"),
                  torch.tensor(r, device="cuda")).cpu().numpy()
    assert rel(z, np.linalg.solve(M, r)) < 1e-8
    assert pre.logdet() == pytest.approx(np.linalg.slogdet(M)[1], rel=1e-8)
    Mi = np.linalg.inv(M)
    # the reference's Nystrom gradients (nys.c:175-474): dM/df = d(K1 K11^{-1} K1^T)/df of the noise-free
    # kernel (eta = mu f^2 is not differentiated in f), dM/dl likewise, dM/dmu = f^2 I.  At k = n the first
    # two equal 2 K / f and dK/dl only as far as K11 is numerically invertible (the additive kernel of 1-D
    # windows is not): 1e-2 against the dense matrices; exact against the rank-n Nystrom built directly.
    dM = [2.0 * K / f, dKl, f * f * np.eye(n)]
    tr = pre.trace()
    want = [np.trace(Mi @ g) for g in dM]
    np.testing.assert_allclose(tr, want, rtol=1e-2)
    assert tr[2] == pytest.approx(want[2], rel=1e-8)
    y = pre.dvp(r)
    for g, tol in ((0, 1e-2), (1, 1e-2), (2, 1e-8)):
        assert rel(y[g * n:(g + 1) * n], Mi @ (dM[g] @ r)) < tol
    from test_gpu_nys_grad import AmdNys
    direct = AmdNys(X, np.arange(d, dtype=np.int32), d, 1, 0, f, l, mu, n, np.arange(n), grad=True, k11_mode=1)
    np.testing.assert_array_equal(tr, direct.trace())
    assert pre.logdet() == direct.logdet()
    np.testing.assert_array_equal(y, direct.dvp(r))
    direct.free()
    pre.free()
    op.free()


def test_gradients_at_k_zero_use_the_whole_kernel_fsai(torch_cuda):
    """the k = 0 branch with require_grad (afn.c:274-284: the Schur FSAI of the whole kernel) is
    the FSAI preconditioner with gradients (kind 3), equal to Nfft4GPAmdPrecondFsai* built directly."""
    from preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd import _lib
    torch = torch_cuda
    n, d, lfil = 2000, 4, 12
    X, op = additive_problem(n=n, d=d, l=0.2, mu=0.05)
    pre = amd.PrecondAFN(X, 0, op=op, schur_lfil=lfil, require_grad=True)
    assert pre.kind == "fsai" and pre.k == 0
    L = _lib.lib()
    h = L.Nfft4GPAmdPrecondFsaiCreate()
    L.Nfft4GPAmdPrecondFsaiSetLfil(h, lfil)
    Xf = np.asfortranarray(X)
    assert L.Nfft4GPAmdPrecondFsaiSetupWithKernel(Xf.ctypes.data, n, n, d,
                                                  _lib.fnptr("Nfft4GPNFFTAdditiveKernelGaussianKernel"), op.h, 1,
                                                  h) == 0
    r = np.random.default_rng(33).random(n)
    z1 = pre.solve(torch.zeros(n, dtype=torch.float64, device="cuda"), torch.tensor(r, device="cuda")).cpu().numpy()
    z2 = np.zeros(n)
    assert L.Nfft4GPAmdPrecondFsaiSolve(h, n, z2.ctypes.data, np.ascontiguousarray(r).ctypes.data) == 0
    np.testing.assert_array_equal(z1, z2)
    assert pre.logdet() == L.Nfft4GPAmdPrecondFsaiLogdet(h)
    t = np.zeros(3)
    tp = ctypes.c_void_p(t.ctypes.data)
    assert L.Nfft4GPAmdPrecondFsaiTrace(h, ctypes.byref(tp)) == 0
    np.testing.assert_array_equal(pre.trace(), t)
    L.Nfft4GPAmdPrecondFsaiFree(h)
    pre.free()
    op.free()
