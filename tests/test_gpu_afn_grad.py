"""AFN preconditioner with gradients (csrc/afn_setup.hip + csrc/afn_grad.hip; MATLAB afn_dvp.m, afn_trace.m,
afn_logdet.m -- the reference's C afn.c has no gradient, so there is no reference output to pin against).

The checks are properties of the preconditioner itself, with M^{-1} assembled column by column from this
library's own apply (Nfft4GPAmdPrecondAFNSolve) at the hyperparameters theta and theta +- h e_g:
* Logdet equals log det M of the assembled matrix (1e-9 relative);
* Trace_g equals tr(M^{-1} dM/dtheta_g) and Dvp_g(x) equals M^{-1} (dM/dtheta_g) x with dM/dtheta_g the
  central difference of the assembled M (1e-5 relative: the O(h^2) truncation and cond(M) eps / h rounding
  at h = 1e-5 theta are both below 1e-7 here);
* the masked call writes only the selected gradient, device vectors give the host result;
* the AFN callbacks (SetupWithKernel / Solve / Trace / Logdet / Dvp / Reset) inside the reference's own
  Nfft4GPGpLoss and inside this library's, on the reference's dense Gaussian operator: same loss and
  gradient.  (The preconditioned Lanczos estimate is not the exact loss: lanczos.c starts its M-inner-
  product Lanczos from plain Rademacher vectors, so the estimate carries a bias that depends on M.)
The rank is predefined (max_k = -k: natural order, afn.c:245-256) so that the ordering and the Schur FSAI's
pattern (geometric) do not move with theta."""
import ctypes as C

import numpy as np
import pytest

import oracle as O

from preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd import _lib

pytestmark = pytest.mark.gpu
needs_ref = pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built")


class AmdAFN:
    """Nfft4GPAmdPrecondAFN* in the loss's call sequence: Create, SetupWithKernel (require_grad), then
    Solve / Dvp / Trace / Logdet."""

    def __init__(self, k, lfil=20):
        self.L = _lib.lib()
        self.h = self.L.Nfft4GPAmdPrecondAFNCreate(-k, 0, 3, lfil, 500)
        assert self.h

    def setup(self, X, f, l, mu, grad=True, kernel=0):
        X = np.asfortranarray(X)
        self.n, d = X.shape
        params = _lib.kernel_params(f, l, mu, self.n)
        fk = _lib.fnptr("Nfft4GPNFFTAdditiveKernelMatern12Kernel") if kernel == 1 else None
        rc = self.L.Nfft4GPAmdPrecondAFNSetupWithKernel(X.ctypes.data, self.n, self.n, d, fk, params,
                                                        1 if grad else 0, self.h)
        self.L.Nfft4GPKernelParamFree(params)
        assert rc == 0
        kind = C.c_int()
        self.L.Nfft4GPAmdPrecondAFNInfo(self.h, C.byref(kind), None, None, None)
        assert kind.value == 0  # the AFN itself

    def minv(self):
        M = np.zeros((self.n, self.n))
        e = np.zeros(self.n)
        x = np.zeros(self.n)
        for j in range(self.n):
            e[:] = 0.0
            e[j] = 1.0
            assert self.L.Nfft4GPAmdPrecondAFNSolve(self.h, self.n, x.ctypes.data, e.ctypes.data) == 0
            M[:, j] = x
        return M

    def dvp(self, x, mask=None):
        y = np.full(3 * self.n, np.nan)
        yp = C.c_void_p(y.ctypes.data)
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.int32)
        assert self.L.Nfft4GPAmdPrecondAFNDvp(self.h, self.n, None if m is None else m.ctypes.data,
                                              np.ascontiguousarray(x).ctypes.data, C.byref(yp)) == 0
        return y

    def trace(self):
        t = np.zeros(3)
        tp = C.c_void_p(t.ctypes.data)
        assert self.L.Nfft4GPAmdPrecondAFNTrace(self.h, C.byref(tp)) == 0
        return t

    def logdet(self):
        return float(self.L.Nfft4GPAmdPrecondAFNLogdet(self.h))

    def free(self):
        self.L.Nfft4GPAmdPrecondAFNFree(self.h)


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / np.linalg.norm(np.asarray(b)))


@pytest.mark.parametrize("kernel,n,d,k,l", [(0, 360, 3, 40, 0.3), (0, 300, 2, 60, 0.15), (1, 320, 3, 32, 0.5)],
                         ids=["gauss3d", "gauss2d", "matern3d"])
def test_afn_grad_against_finite_differences(torch_cuda, kernel, n, d, k, l):
    rng = np.random.default_rng(n + k)
    X = rng.random((n, d))
    theta = np.array([1.1, l, 0.05])
    P = AmdAFN(k)
    P.setup(X, *theta, kernel=kernel)
    Minv0 = P.minv()
    x = rng.random(n) - 0.5
    y = P.dvp(x)
    tr = P.trace()
    ld = P.logdet()
    sign, ld_dense = np.linalg.slogdet(Minv0)
    assert sign > 0
    assert ld == pytest.approx(-ld_dense, rel=1e-9)
    for g in range(3):
        h = 1e-5 * theta[g]
        Ms = []
        for s in (1.0, -1.0):
            t = theta.copy()
            t[g] += s * h
            P.setup(X, *t, grad=False, kernel=kernel)
            Ms.append(np.linalg.inv(P.minv()))
        dM = (Ms[0] - Ms[1]) / (2 * h)
        assert tr[g] == pytest.approx(np.trace(Minv0 @ dM), rel=1e-5, abs=1e-7 * n), g
        assert rel(y[g * n:(g + 1) * n], Minv0 @ (dM @ x)) < 1e-5, g
    P.free()


def test_afn_grad_mask_and_device_vectors(torch_cuda):
    import torch

    n, d, k = 400, 3, 48
    rng = np.random.default_rng(5)
    X = rng.random((n, d))
    P = AmdAFN(k)
    P.setup(X, 1.3, 0.25, 0.02)
    x = rng.random(n) - 0.5
    y = P.dvp(x)
    assert np.all(np.isfinite(y))
    ym = P.dvp(x, mask=[0, 1, 0])
    assert np.all(ym[:n] == 0.0) and np.all(ym[2 * n:] == 0.0)
    assert np.array_equal(ym[n:2 * n], y[n:2 * n])
    xd = torch.tensor(x, device="cuda")
    yd = torch.zeros(3 * n, dtype=torch.float64, device="cuda")
    yp = C.c_void_p(yd.data_ptr())
    assert P.L.Nfft4GPAmdPrecondAFNDvp(P.h, n, None, C.c_void_p(xd.data_ptr()), C.byref(yp)) == 0
    torch.cuda.synchronize()
    assert np.array_equal(yd.cpu().numpy(), y)
    # dvp / trace without gradients fail loudly instead of returning zeros
    P.setup(X, 1.3, 0.25, 0.02, grad=False)
    yy = np.zeros(3 * n)
    yp = C.c_void_p(yy.ctypes.data)
    assert P.L.Nfft4GPAmdPrecondAFNDvp(P.h, n, None, x.ctypes.data, C.byref(yp)) != 0
    P.free()


def test_afn_grad_python_front_end(torch_cuda):
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd

    n, d = 300, 3
    rng = np.random.default_rng(8)
    X = rng.random((n, d))
    pre = amd.PrecondAFN(X, -30, 1.2, 0.3, 0.04, require_grad=True)
    assert pre.kind == "afn" and pre.k == 30
    x = rng.random(n) - 0.5
    ref = AmdAFN(30)
    ref.setup(X, 1.2, 0.3, 0.04)
    assert np.array_equal(pre.dvp(x), ref.dvp(x))
    np.testing.assert_array_equal(pre.trace(), ref.trace())
    assert pre.logdet() == ref.logdet()
    ref.free()
    pre.free()


@needs_ref
def test_gp_loss_with_afn_gradients(torch_cuda):
    """The reference's own Nfft4GPGpLoss (oracle/_ref, gp_loss.c:96-307 with lanczos.c:421-610) and this
    library's, both with the reference's dense Gaussian operator and THIS library's AFN with gradients as the
    precond_* callbacks (host vectors through the C ABI): the same loss and gradient to 1e-8 -- the AFN
    plugs into the reference's loss as its Nystrom and FSAI do."""
    lib = O.ref_lib()
    rng = np.random.default_rng(11)
    n, d, k, nvecs, maxits = 500, 3, 64, 8, 40
    X = np.asfortranarray(rng.random((n, d)))
    y = rng.random(n) - 0.5
    theta = np.array([1.1, 0.3, 0.02])
    hyper = np.log(np.expm1(theta))  # transform 0 is the softplus (transform.h:16): the loss sees theta
    R = np.asfortranarray(np.sign(rng.random((n, nvecs)) - 0.5))
    kh = O.ref_gaussian_params(1.0, 1.0, 0.01, n)
    pkh = O.ref_gaussian_params(1.0, 1.0, 0.01, n)
    P = AmdAFN(k)
    f = lambda name: C.cast(getattr(lib, name), C.c_void_p).value  # noqa: E731
    dwork = np.zeros(4 * n * n + 4 * n)

    def run(fn):
        cb = [_lib.fnptr("Nfft4GPAmdPrecondAFN" + s) for s in ("SetupWithKernel", "Solve", "Trace", "Logdet", "Dvp",
                                                               "Reset")]
        args = (hyper.ctypes.data, X.ctypes.data, y.ctypes.data, n, n, d, f("Nfft4GPKernelGaussianKernel"), kh, None,
                f("Nfft4GPDenseMatSymv"), f("Nfft4GPDenseGradMatSymv"), f("Nfft4GPKernelGaussianKernel"), pkh, None,
                *cb, P.h, 0, 1e-10, maxits, maxits, nvecs, R.ctypes.data, 0, None, 0, dwork.ctypes.data)
        fn.argtypes = O.RefGpLoss.ARGTYPES
        fn.restype = C.c_int
        loss = np.zeros(1)
        grad = np.zeros(3)
        assert fn(*args, loss.ctypes.data_as(_lib.dp), grad.ctypes.data_as(_lib.dp)) == 0
        return loss[0], grad

    loss_ref, grad_ref = run(lib.Nfft4GPGpLoss)
    loss, grad = run(_lib.lib().Nfft4GPGpLoss)
    P.free()
    print("loss", loss_ref, loss, "grad", grad_ref, grad)
    assert np.isfinite(loss) and np.all(np.isfinite(grad))
    assert loss == pytest.approx(loss_ref, rel=1e-8)
    np.testing.assert_allclose(grad, grad_ref, rtol=1e-6, atol=1e-9)
