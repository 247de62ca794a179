"""The AFN's gradients against the reference's own specification of them: the MATLAB prototype
(afn_setup.m with require_grad, chol_setup.m, schurCombinedKernelMat.m, fsai_setup.m, afn_dvp.m, afn_trace.m,
afn_logdet.m), restated in numpy in oracle/afn_spec.py (CPU-checked in tests/test_afn_spec.py).  The
reference's C afn.c has no gradient, so this restatement is the parity anchor; tests/test_gpu_afn_grad.py
checks the same quantities against finite differences of this library's own apply.

Same points, order (predefined rank: the first k points are the landmarks) and Schur-FSAI pattern (this
library's, which is checked to be the KNN pattern of fsai_setup.m's knnpattern):
* the Schur FSAI's values G equal the restatement's (1e-9 of each row's norm);
* Logdet equals afn_logdet.m (1e-10), Trace equals afn_trace.m (1e-8);
* Dvp equals M^{-1} afn_dvp.m(x) (1e-8; afn_dvp.m returns dM/dtheta x, the C interface M^{-1} dM/dtheta x).
"""
import ctypes as C

import numpy as np
import pytest

import afn_spec as S
from test_gpu_afn_grad import AmdAFN

from preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd import _lib

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / np.linalg.norm(np.asarray(b)))


@pytest.mark.parametrize("n,d,k,lfil,theta", [(300, 3, 30, 12, (1.1, 0.3, 0.05)), (240, 2, 40, 8, (0.8, 0.15, 0.02))])
def test_afn_gradients_match_matlab_spec(torch_cuda, n, d, k, lfil, theta):
    rng = np.random.default_rng(n + d)
    X = rng.random((n, d))
    P = AmdAFN(k, lfil=lfil)
    P.setup(X, *theta)
    L = _lib.lib()
    afn = C.c_void_p()
    kind = C.c_int()
    L.Nfft4GPAmdPrecondAFNInfo(P.h, C.byref(kind), None, C.byref(afn), None)
    assert kind.value == 0 and afn.value
    n2 = n - k
    kk = C.c_int()
    perm = np.zeros(n, np.int32)
    nnz = L.Nfft4GPAmdAfnInfo(afn.value, C.byref(kk), perm.ctypes.data, None, None, None)
    assert kk.value == k and nnz > 0
    np.testing.assert_array_equal(perm, np.arange(n))  # predefined rank: natural order (afn.c:245-256)
    ia = np.zeros(n2 + 1, np.int32)
    ja = np.zeros(nnz, np.int32)
    aa = np.zeros(nnz)
    L.Nfft4GPAmdAfnInfo(afn.value, None, None, ia.ctypes.data, ja.ctypes.data, aa.ctypes.data)
    pattern = []
    for i in range(n2):
        cols = ja[ia[i]:ia[i + 1]]
        assert cols[-1] == i  # the diagonal last (fsai.c:689-696)
        pattern.append(sorted(cols[:-1].tolist()))
    # the pattern is fsai_setup.m's knnpattern with lfil - 1 neighbours (the C lfil counts the diagonal)
    want = S.knn_pattern(X[k:], lfil - 1)
    assert sum(set(a) != set(b) for a, b in zip(pattern, want)) == 0
    R = S.afn_setup(X, k, *theta, pattern)
    for i in range(n2):
        cols = ja[ia[i]:ia[i + 1]]
        row = R["G"][i, cols]
        assert np.linalg.norm(aa[ia[i]:ia[i + 1]] - row) <= 1e-9 * np.linalg.norm(row), i
    assert P.logdet() == pytest.approx(S.afn_logdet(R), rel=1e-10)
    np.testing.assert_allclose(P.trace(), S.afn_trace(R), rtol=1e-8)
    x = rng.random(n) - 0.5
    y = P.dvp(x)
    spec = S.afn_dvp(R, x)
    for g in range(3):
        assert rel(y[g * n:(g + 1) * n], S.afn_solve(R, spec[g])) < 1e-8, g
    P.free()


@pytest.mark.parametrize("n,d,k,theta", [(400, 6, 24, (1.2, 0.15, 0.04)), (300, 4, 40, (0.9, 0.1, 0.01))])
def test_nystrom_gradients_match_matlab_ran_spec(torch_cuda, n, d, k, theta):
    """The Nystrom with gradients on landmarks perm[:k] (Nfft4GPAmdPrecondNys*, k11 mode 1; the AFN flow's
    Nystrom branches) against MATLAB's ran_setup.m / ran_solve.m / ran_logdet.m / ran_trace.m / ran_dvp.m
    (oracle/ran_spec.py) on the additive kernel of 1-D windows: apply 1e-9, Logdet 1e-10, Trace and
    M^{-1} ran_dvp 1e-7 (MATLAB shifts K11 by sqrt(n) eps(||K1||_2) and S by -nu, nys.c by sqrt(k) ulp(||K11||_F):
    rounding-level differences in the factors, amplified by K11's conditioning)."""
    import ran_spec as R
    from test_gpu_nys_grad import AmdNys
    rng = np.random.default_rng(n + k)
    X = rng.random((n, d))
    win = np.arange(d, dtype=np.int32)
    perm = rng.permutation(n).astype(np.int32)
    P = AmdNys(X, win, d, 1, 0, *theta, k, perm, grad=True, k11_mode=1)
    Rs = R.ran_setup(X, [[c] for c in range(d)], *theta, perm, k)
    r = rng.random(n) - 0.5
    assert rel(P.solve(r), R.ran_solve(Rs, r)) < 1e-9
    assert P.logdet() == pytest.approx(R.ran_logdet(Rs), rel=1e-10)
    np.testing.assert_allclose(P.trace(), R.ran_trace(Rs), rtol=1e-7)
    y = P.dvp(r)
    spec = R.ran_dvp(Rs, r)
    for g in range(3):
        assert rel(y[g * n:(g + 1) * n], R.ran_solve(Rs, spec[g])) < 1e-7, g
    P.free()
