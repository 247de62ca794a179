"""GPU Nystrom preconditioner with gradients (csrc/nys_grad.hip) against the reference's own nys.c with
require_grad (oracle/_ref: Nfft4GPPrecondNysSetupWithKernel / Dvp / Trace / Logdet, nys.c:175-660) on its
dense additive kernel, and inside Nfft4GPGpLoss against the reference's loss with its own preconditioner
(tests/golden/krylov_synth.npz, loss_nys8).

Tolerances: Dvp 1e-8 relative (GEMVs with a different association; the preconditioner solves amplify the
1e-16 rounding by cond(M) on these small kernels), traces 1e-8 relative plus 1e-10 of the largest trace
(the f and l traces are differences of terms of that size; k-space restatement of the reference's n x k
sums), logdet 1e-11 (from s, which matches to ~1e-12)."""
import ctypes as C
import os

import numpy as np
import pytest

import oracle as O

import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
from preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd import _lib

pytestmark = pytest.mark.gpu
needs_ref = pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built")
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / np.linalg.norm(np.asarray(b)))


class AmdNys:
    """This library's Nfft4GPAmdPrecondNys* over an additive NFFT handle (the reference's call sequence:
    Create, SetRank, SetPerm, SetupWithKernel, then Solve / Dvp / Trace / Logdet)."""

    def __init__(self, X, win, nw, dw, kernel, f, l, mu, k, perm, grad=True, k11_mode=0):
        self.L = _lib.lib()
        self.op = amd.NFFTAdditiveKernel(X, win, nw, dw)
        assert self.op.setup(kernel, f, l, mu) == 0
        self.perm = np.ascontiguousarray(np.asarray(perm, dtype=np.int32))
        self.n = self.op.n
        self.h = self.L.Nfft4GPAmdPrecondNysCreate()
        self.L.Nfft4GPAmdPrecondNysSetRank(self.h, k)
        self.L.Nfft4GPAmdPrecondNysSetPerm(self.h, self.perm.ctypes.data, 0)
        self.L.Nfft4GPAmdPrecondNysSetK11Mode(self.h, k11_mode)
        fk = _lib.fnptr("Nfft4GPNFFTAdditiveKernelGaussianKernel" if kernel == 0 else
                        "Nfft4GPNFFTAdditiveKernelMatern12Kernel")
        Xf = np.asfortranarray(X)
        rc = self.L.Nfft4GPAmdPrecondNysSetupWithKernel(Xf.ctypes.data, self.n, self.n, X.shape[1], fk, self.op.h,
                                                        1 if grad else 0, self.h)
        assert rc == 0

    def solve(self, r):
        x = np.zeros(self.n)
        assert self.L.Nfft4GPAmdPrecondNysSolve(self.h, self.n, x.ctypes.data, np.ascontiguousarray(r).ctypes.data) == 0
        return x

    def dvp(self, x, mask=None):
        y = np.zeros(3 * self.n)
        yp = C.c_void_p(y.ctypes.data)
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.int32)
        assert self.L.Nfft4GPAmdPrecondNysDvp(self.h, self.n, m.ctypes.data if m is not None else None,
                                              np.ascontiguousarray(x).ctypes.data, C.byref(yp)) == 0
        return y

    def trace(self):
        t = np.zeros(3)
        tp = C.c_void_p(t.ctypes.data)
        assert self.L.Nfft4GPAmdPrecondNysTrace(self.h, C.byref(tp)) == 0
        return t

    def logdet(self):
        return float(self.L.Nfft4GPAmdPrecondNysLogdet(self.h))

    def free(self):
        self.L.Nfft4GPAmdPrecondNysFree(self.h)


@needs_ref
@pytest.mark.parametrize("kernel,l,k", [(0, 0.1, 24), (0, 0.05, 48), (1, 1.0, 32)])
def test_nys_grad_matches_reference(torch_cuda, kernel, l, k):
    n, d = 1500, 4
    rng = np.random.default_rng(41)
    X = rng.random((n, d))
    win = np.arange(d, dtype=np.int32)
    f, mu = 1.2, 0.02
    perm = rng.permutation(n).astype(np.int32)
    dense = O.RefDenseAdditive(X, win, d, 1, kernel=kernel)
    ref = O.RefNystrom(dense, f, l, mu, k, perm, grad=True)
    ours = AmdNys(X, win, d, 1, kernel, f, l, mu, k, perm)
    x = rng.random(n) - 0.5
    assert rel(ours.solve(x), ref.solve(np.zeros(n), x.copy())) < 1e-9
    y_ref = ref.dvp(x)
    y = ours.dvp(x)
    for g in range(3):
        assert rel(y[g * n:(g + 1) * n], y_ref[g * n:(g + 1) * n]) < 1e-8, g
    # masked call: only the l gradient is written
    ym = ours.dvp(x, mask=[0, 1, 0])
    assert np.all(ym[:n] == 0.0) and np.all(ym[2 * n:] == 0.0)
    assert rel(ym[n:2 * n], y_ref[n:2 * n]) < 1e-8
    t_ref = ref.trace()
    t = ours.trace()
    # traces 0 and 1 are differences of terms of the size of trace 2 (n f^2 / eta): absolute error held to
    # 1e-10 of that scale (measured 1.2e-11), relative 1e-8 otherwise
    np.testing.assert_allclose(t, t_ref, rtol=1e-8, atol=1e-10 * np.abs(t_ref).max())
    assert ours.logdet() == pytest.approx(ref.logdet(), rel=1e-11)
    ours.free()


def test_nys_grad_landmarks_matches_numpy(torch_cuda):
    """k11 mode 1 (K11 = K(perm[:k], perm[:k]), gradient panels over every window) with a padded last
    window (skip_last = 1: windows {0,1}, {2,-1}) against a numpy restatement of nys.c:175-516."""
    n, k, f, l, mu = 900, 20, 1.1, 0.15, 0.03
    rng = np.random.default_rng(42)
    X = rng.random((n, 3))
    win = np.array([0, 1, 2, -1], dtype=np.int32)
    perm = rng.permutation(n).astype(np.int32)
    ours = AmdNys(X, win, 2, 2, 0, f, l, mu, k, perm, k11_mode=1)
    groups = [[0, 1], [2]]

    def kern(A, B):
        K = np.zeros((len(A), len(B)))
        Kl = np.zeros_like(K)
        for cols in groups:
            r2 = sum((A[:, c][:, None] - B[:, c][None, :]) ** 2 for c in cols)
            e = np.exp(-r2 / (2 * l * l))
            K += e
            Kl += r2 / l ** 3 * e
        return f * f * K / 2, 2 / f * f * f * K / 2, f * f * Kl / 2

    K, dKf, dKl = kern(X, X[perm[:k]])
    K11, dK11f, dK11l = kern(X[perm[:k]], X[perm[:k]])
    fro = np.linalg.norm(K11)
    G = np.linalg.inv(np.linalg.cholesky(K11 + np.sqrt(k) * (np.nextafter(fro, fro + 1) - fro) * np.eye(k)))
    GdKG = [G @ dK11f @ G.T, G @ dK11l @ G.T]
    dU = K @ G.T
    w1, V = np.linalg.eigh(dU.T @ dU)
    U = (dU @ V[:, ::-1]) / np.sqrt(w1[::-1])
    eta, f2 = mu * f * f, f * f
    s = 1.0 / (w1[::-1] + eta)
    Minv = lambda r: U @ (s * (U.T @ r)) + (r - U @ (U.T @ r)) / eta
    x = rng.random(n) - 0.5
    y = ours.dvp(x)
    for g, dK in enumerate([dKf, dKl]):
        a = G.T @ (G @ (K.T @ x))
        b = G.T @ (G @ (dK.T @ x))
        c = G.T @ (GdKG[g] @ (G @ (K.T @ x)))
        assert rel(y[g * n:(g + 1) * n], Minv(dK @ a - K @ c + K @ b)) < 1e-8, g
    assert rel(y[2 * n:], f2 * Minv(x)) < 1e-9
    UUU = dU @ np.linalg.inv(dU.T @ dU + eta * np.eye(k))
    tr = np.array([np.sum((2 * dK @ G.T - dU @ GdKG[g]) * dU) for g, dK in enumerate([dKf, dKl])] + [n * f2])
    for il in range(k):
        xc = dU[:, il]
        for g, dK in enumerate([dKf, dKl]):
            a = G.T @ (G @ (K.T @ xc))
            b = G.T @ (G @ (dK.T @ xc))
            c = G.T @ (GdKG[g] @ (G @ (K.T @ xc)))
            tr[g] -= (dK @ a - K @ c + K @ b) @ UUU[:, il]
        tr[2] -= f2 * xc @ UUU[:, il]
    np.testing.assert_allclose(ours.trace(), tr / eta, rtol=1e-8, atol=1e-10 * np.abs(tr / eta).max())
    ld = np.log(eta) * (n - k) + np.sum(np.log(1.0 / s))
    assert ours.logdet() == pytest.approx(ld, rel=1e-10)
    ours.free()


@needs_ref
def test_gp_loss_with_gpu_nystrom(torch_cuda):
    """Nfft4GPGpLoss with the reference's dense operator callbacks and THIS library's Nystrom with gradients
    (setup / solve / trace / logdet / dvp all on the GPU) against the reference's loss with its own Nystrom
    (krylov_synth loss_nys8 / grad_nys8: k = 8, pcg_synth's permutation)."""
    z = np.load(os.path.join(GOLD, "pcg_synth.npz"), allow_pickle=False)
    kz = np.load(os.path.join(GOLD, "krylov_synth.npz"), allow_pickle=False)
    X = np.asfortranarray(np.asarray(z["X"]))
    win, nw, dw = np.asarray(z["windows"], dtype=np.int32), int(z["nw"]), int(z["dw"])
    n, d = X.shape
    g = O.RefGpLoss(X, win, nw, dw)  # the reference's dense kernel / SYMV / grad SYMV, no preconditioner
    args = list(g.args(np.asarray(kz["hyper"]), np.asarray(z["b"]), int(kz["maxits"]), int(kz["nvecs"]),
                       np.asarray(kz["rademacher"], dtype=np.float64)))
    L = _lib.lib()
    pop = amd.NFFTAdditiveKernel(X, win, nw, dw)  # the preconditioner's kernel data (gp_loss.c:146-150)
    perm = np.ascontiguousarray(np.asarray(z["nys_perm"], dtype=np.int32))
    h = L.Nfft4GPAmdPrecondNysCreate()
    L.Nfft4GPAmdPrecondNysSetRank(h, 8)
    L.Nfft4GPAmdPrecondNysSetPerm(h, perm.ctypes.data, 0)
    args[11] = _lib.fnptr("Nfft4GPNFFTAdditiveKernelGaussianKernel")
    args[12] = pop.h
    args[14:20] = [_lib.fnptr(name) for name in (
        "Nfft4GPAmdPrecondNysSetupWithKernel", "Nfft4GPAmdPrecondNysSolve", "Nfft4GPAmdPrecondNysTrace",
        "Nfft4GPAmdPrecondNysLogdet", "Nfft4GPAmdPrecondNysDvp", "Nfft4GPAmdPrecondNysReset")]
    args[20] = h
    fn = L.Nfft4GPGpLoss
    fn.argtypes = O.RefGpLoss.ARGTYPES
    fn.restype = C.c_int
    loss = np.zeros(1)
    grad = np.zeros(3)
    assert fn(*args, loss.ctypes.data_as(_lib.dp), grad.ctypes.data_as(_lib.dp)) == 0
    L.Nfft4GPAmdPrecondNysFree(h)
    assert loss[0] == pytest.approx(float(kz["loss_nys8"]), rel=1e-8)
    np.testing.assert_allclose(grad, kz["grad_nys8"], rtol=1e-6, atol=1e-9)
