"""CPU check of oracle/afn_spec.py, the numpy restatement of the reference's MATLAB AFN with gradients
(afn_setup.m, chol_setup.m, schurCombinedKernelMat.m, fsai_setup.m, afn_dvp.m / afn_trace.m / afn_logdet.m):
its Logdet is log det of its own M, its Trace and Dvp are the derivatives of its own M(theta) (central
differences with the FSAI pattern held fixed).  The GPU test tests/test_gpu_afn_matlab.py then compares this
library's AFN gradients with it."""
import numpy as np
import pytest

import afn_spec as S


def _M(P):
    n = P["n"]
    return np.linalg.inv(np.column_stack([S.afn_solve(P, e) for e in np.eye(n)]))


def test_restatement_is_self_consistent():
    rng = np.random.default_rng(3)
    n, d, k, lfil = 70, 2, 9, 6
    X = rng.random((n, d))
    theta = np.array([1.2, 0.3, 0.05])
    pattern = S.knn_pattern(X[k:], lfil)
    P = S.afn_setup(X, k, *theta, pattern)
    M = _M(P)
    assert np.allclose(M, M.T, atol=1e-10 * np.abs(M).max())
    assert S.afn_logdet(P) == pytest.approx(np.linalg.slogdet(M)[1], rel=1e-10)
    x = rng.random(n) - 0.5
    y = S.afn_dvp(P, x)
    tr = S.afn_trace(P)
    for g in range(3):
        h = 1e-5 * theta[g]
        Ms = []
        for s in (1.0, -1.0):
            t = theta.copy()
            t[g] += s * h
            Ms.append(_M(S.afn_setup(X, k, *t, pattern)))
        dM = (Ms[0] - Ms[1]) / (2 * h)
        np.testing.assert_allclose(y[g], dM @ x, rtol=1e-6, atol=1e-8 * np.abs(dM @ x).max())
        assert tr[g] == pytest.approx(np.trace(np.linalg.solve(M, dM)), rel=1e-6)


def test_ran_restatement_is_self_consistent():
    """oracle/ran_spec.py (MATLAB ran_*.m): Logdet is log det of its own M, Trace is tr(M^{-1} dM) with dM
    from its own ran_dvp, and ran_dvp's dK_f / dK_l blocks are the central differences of the noise-free
    Nystrom K1' K11^{-1} K1 (plus the f^2 I of mu)."""
    import ran_spec as R
    rng = np.random.default_rng(5)
    n, d, k = 60, 3, 12
    X = rng.random((n, d))
    win = [[0], [1], [2]]
    perm = rng.permutation(n)
    theta = np.array([1.1, 0.2, 0.03])
    P = R.ran_setup(X, win, *theta, perm, k)
    Minv = np.column_stack([R.ran_solve(P, e) for e in np.eye(n)])
    M = np.linalg.inv(Minv)
    assert R.ran_logdet(P) == pytest.approx(np.linalg.slogdet(M)[1], rel=1e-9)
    dM = [np.column_stack([R.ran_dvp(P, e)[g] for e in np.eye(n)]) for g in range(3)]
    np.testing.assert_allclose(R.ran_trace(P), [np.trace(Minv @ g) for g in dM], rtol=1e-7)

    def nys(t):
        K1, _ = R.additive_noise_free(X, win, t[0], t[1], perm[:k], np.arange(n))
        K11, _ = R.additive_noise_free(X, win, t[0], t[1], perm[:k], perm[:k])
        return K1.T @ np.linalg.solve(K11, K1)

    for g in range(2):
        h = 1e-5 * theta[g]
        tp, tm = theta.copy(), theta.copy()
        tp[g] += h
        tm[g] -= h
        fd = (nys(tp) - nys(tm)) / (2 * h)
        np.testing.assert_allclose(dM[g], fd, rtol=1e-5, atol=1e-7 * np.abs(fd).max())
