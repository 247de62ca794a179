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
