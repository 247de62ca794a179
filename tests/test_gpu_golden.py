"""GPU parity against the committed golden fixtures (tests/golden/*.npz), through the C ABI:
the HIP additive matvec / grad matvec vs the oracle's NFFT outputs, the HIP Nystrom apply vs the
reference's nys.c output, and the device-controlled PCG vs the reference's pcg.c runs (dense operator
of the fixture supplied as a C callback, so both solvers see the same operator)."""
import ctypes as C
import os

import numpy as np
import pytest

import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
from preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd import _lib

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

ONE_D = [("foo1d", "gauss_l0.1", 0, 0.1), ("foo1d", "gauss_l1.0", 0, 1.0), ("foo1d", "matern_l0.1", 1, 0.1),
         ("foo1d", "matern_l1.0", 1, 1.0), ("synth1d", "gauss_l0.3", 0, 0.3), ("synth1d", "matern_l1.0", 1, 1.0)]


def load(name):
    return np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / np.linalg.norm(np.asarray(b)))


@pytest.mark.parametrize("name,pre,kernel,l", ONE_D)
def test_matvec_matches_golden(torch_cuda, name, pre, kernel, l):
    torch = torch_cuda
    z = load(name)
    X = np.asarray(z["X"])
    op = amd.NFFTAdditiveKernel(X, np.asarray(z["windows"], np.int32), int(z["nw"]), int(z["dw"]))
    assert op.setup(kernel, float(z["f"]), l, float(z["mu"])) == 0
    x = np.asarray(z["x"])
    n = x.size
    xd = torch.tensor(x, device="cuda")
    yd = torch.zeros(n, dtype=torch.float64, device="cuda")
    op.matsymv(xd, 1.0, 0.0, yd)
    # the product's design error (tap polynomials, fixed-point coordinates): <= 1e-9 at l = 0.1
    assert rel(yd.cpu().numpy(), z[pre + "_nfft_y"]) < 1e-8
    y0 = torch.tensor(np.cos(np.arange(n)), device="cuda")
    op.matsymv(xd, 0.7, -1.5, y0)
    assert rel(y0.cpu().numpy(), z[pre + "_nfft_y_ab"]) < 1e-8
    g = torch.zeros(3 * n, dtype=torch.float64, device="cuda")
    op.gradmatsymv(xd, 1.0, 0.0, g)
    g = g.cpu().numpy()
    gz = z[pre + "_nfft_grad"]
    for i in range(3):
        assert rel(g[i * n:(i + 1) * n], gz[i * n:(i + 1) * n]) < 1e-8, i


# ---- dense operator of a fixture as a plain host C callback -------------------------------------
class DenseHostOp:
    """func_symmatvec on HOST vectors (how the reference calls every operator): y = alpha*K x + beta*y
    with K the reference's dense additive Gaussian f^2 ((1/nw) sum_c exp(-|x_c - x_c'|^2 / 2 l^2) + mu I)
    (kernels.c:680-1289, 3099-3494).  Nfft4GPSolverPcg stages vectors for it (callback mode -1)."""

    def __init__(self, z):
        X, f, l, mu = np.asarray(z["X"]), float(z["f"]), float(z["l"]), float(z["mu"])
        n, nw = X.shape
        K = np.zeros((n, n))
        for c in range(nw):
            d = X[:, c][:, None] - X[:, c][None, :]
            K += np.exp(-d * d / (2 * l * l))
        self.K = f * f * (K / nw + mu * np.eye(n))
        self.n = n
        self.h = None

        def mv(_m, nn, alpha, xp, beta, yp):
            xv = np.ctypeslib.as_array(C.cast(xp, _lib.dp), shape=(nn,))
            yv = np.ctypeslib.as_array(C.cast(yp, _lib.dp), shape=(nn,))
            yv[:] = alpha * (self.K @ xv) + (beta * yv if beta != 0.0 else 0.0)
            return 0

        self._cb = _lib.SYMMATVEC(mv)
        self.matvec_fnptr = C.cast(self._cb, C.c_void_p).value


class RefDenseOp:
    """The reference's own Nfft4GPDenseMatSymv (matops.c:3-13, compiled in oracle/_ref) on the dense
    additive matrix built by its Nfft4GPKernelAdditiveKernel: the drop-in scenario of a reference
    caller handing its host operator to this library's PCG."""

    def __init__(self, z):
        import oracle as O
        self.dense = O.RefDenseAdditive(np.asarray(z["X"]), np.asarray(z["windows"], np.int32), int(z["nw"]),
                                        int(z["dw"]), kernel=0)
        self.dense.matrices(float(z["f"]), float(z["l"]), float(z["mu"]), grad=False)
        self.n = self.dense.n
        self.h = C.cast(self.dense._K, C.c_void_p).value
        self.matvec_fnptr = C.cast(self.dense.lib.Nfft4GPDenseMatSymv, C.c_void_p).value


def test_nystrom_apply_matches_golden(torch_cuda):
    torch = torch_cuda
    z = load("pcg_synth")
    pre = amd.NystromPrecond(z["nys_U"], z["nys_s"], float(z["nys_eta"]), z["nys_perm"])
    r = np.asarray(z["nys_rhs"])
    xd = torch.zeros(r.size, dtype=torch.float64, device="cuda")
    pre.solve(xd, torch.tensor(r, device="cuda"))
    assert rel(xd.cpu().numpy(), z["nys_out"]) <= 1e-12


@pytest.mark.parametrize("opkind", ["numpy", "reference"])
@pytest.mark.parametrize("with_nys", [False, True])
def test_pcg_matches_golden(torch_cuda, with_nys, opkind):
    torch = torch_cuda
    import oracle as O
    if opkind == "reference" and not O.ref_available():
        pytest.skip("oracle/_ref not built")
    z = load("pcg_synth")
    op = DenseHostOp(z) if opkind == "numpy" else RefDenseOp(z)
    pre = amd.NystromPrecond(z["nys_U"], z["nys_s"], float(z["nys_eta"]), z["nys_perm"]) if with_nys else None
    key = "pcgnys" if with_nys else "pcg"
    b = torch.tensor(np.asarray(z["b"]), device="cuda")
    x = torch.zeros(op.n, dtype=torch.float64, device="cuda")
    x, rr, hist, it = amd.pcg(op, b, x, maxits=1000, tol=1e-6, precond=pre)
    it_ref = int(z[key + "_iters"])
    assert it > 0 and abs(it - it_ref) <= max(2, it_ref // 20), (it, it_ref)
    assert rr <= 1e-6
    assert rel(x.cpu().numpy(), z[key + "_x"]) < 1e-5
    h_ref = np.asarray(z[key + "_hist"])
    k = min(10, it, it_ref)
    np.testing.assert_allclose(hist[:k], h_ref[:k], rtol=1e-6)
    # pcg.c:188: the converged entry holds the ABSOLUTE true-residual norm
    assert hist[it] == pytest.approx(rr * np.linalg.norm(np.asarray(z["b"])), rel=1e-12)


def test_pcg_host_vectors_with_reference_operator(torch_cuda):
    """Host b / x (the reference's convention end to end) with the reference's dense operator."""
    import oracle as O
    if not O.ref_available():
        pytest.skip("oracle/_ref not built")
    z = load("pcg_synth")
    op = RefDenseOp(z)
    x = np.zeros(op.n)
    x, rr, hist, it = amd.pcg(op, np.asarray(z["b"]).copy(), x, maxits=1000, tol=1e-6)
    assert it > 0 and abs(it - int(z["pcg_iters"])) <= max(2, int(z["pcg_iters"]) // 20)
    assert rel(x, z["pcg_x"]) < 1e-5


def test_reference_nys_struct_through_the_reference_name(torch_cuda):
    """Nfft4GPPrecondNysSolve (the reference's name, nys.c:115-173) on the precond_nys the reference's own
    setup built (oracle/_ref, nys.c:518-660): device and host vectors equal the reference's Solve to 1e-12;
    PCG with it matches pcg_synth's Nystrom run; a re-setup of the same struct at another l is seen (the
    HBM mirror is rebuilt, not reused) and k = 0 gives rhs / eta."""
    torch = torch_cuda
    import oracle as O
    if not O.ref_available():
        pytest.skip("oracle/_ref not built")
    z = load("pcg_synth")
    dense = O.RefDenseAdditive(np.asarray(z["X"]), np.asarray(z["windows"], np.int32), int(z["nw"]), int(z["dw"]))
    nys = O.RefNystrom(dense, float(z["f"]), float(z["l"]), float(z["mu"]), int(z["nys_k"]), z["nys_perm"])
    pre = amd.ReferenceNystrom(nys.h, nys.n)
    r = np.asarray(z["nys_rhs"])
    want = nys.solve(np.zeros(nys.n), r.copy())
    assert rel(want, z["nys_out"]) <= 1e-12
    xd = torch.zeros(r.size, dtype=torch.float64, device="cuda")
    pre.solve(xd, torch.tensor(r, device="cuda"))
    assert rel(xd.cpu().numpy(), want) <= 1e-12
    xh = np.zeros(r.size)
    pre.solve(xh, r.copy())
    assert rel(xh, want) <= 1e-12
    tits = nys.st._tits
    op = RefDenseOp(z)
    b = torch.tensor(np.asarray(z["b"]), device="cuda")
    x = torch.zeros(op.n, dtype=torch.float64, device="cuda")
    x, rr, hist, it = amd.pcg(op, b, x, maxits=1000, tol=1e-6, precond=pre)
    it_ref = int(z["pcgnys_iters"])
    assert it > 0 and abs(it - it_ref) <= max(2, it_ref // 20), (it, it_ref)
    assert rr <= 1e-6 and rel(x.cpu().numpy(), z["pcgnys_x"]) < 1e-5
    assert nys.st._tits - tits >= it  # _tits counts the applies (nys.c:170)
    # Reset + re-setup of the same struct (the loss's cycle, gp_loss.c:161 / :300; nys.c:76-100, :518-660) at
    # l = 0.2: new factors, possibly at the same addresses
    nys.lib.Nfft4GPPrecondNysReset.argtypes = [C.c_void_p]
    nys.lib.Nfft4GPPrecondNysReset(C.c_void_p(nys.h))
    dense.st._params[1] = 0.2
    fk = C.cast(nys.lib.Nfft4GPKernelAdditiveKernel, C.c_void_p)
    assert nys.lib.Nfft4GPPrecondNysSetupWithKernel(O._d(dense._data), dense.n, dense.n, dense.d, fk, dense.h, 0,
                                                    nys.h) == 0
    want2 = nys.solve(np.zeros(nys.n), r.copy())
    assert rel(want2, want) > 1e-6
    pre.solve(xd, torch.tensor(r, device="cuda"))
    assert rel(xd.cpu().numpy(), want2) <= 1e-12
    # k = 0: x = rhs / eta
    k_saved = nys.st._k
    nys.st._k = 0
    pre.solve(xd, torch.tensor(r, device="cuda"))
    assert rel(xd.cpu().numpy(), r / nys.st._eta) <= 1e-15
    nys.st._k = k_saved
    pre.free()


# ---- FSAI (fsai.c:106-123) and AFN (afn.c:82-143) applies ----------------------------------------
class DenseGaussHostOp(DenseHostOp):
    """func_symmatvec on host vectors for the precond_synth fixture: the reference's dense Gaussian
    kernel f^2 (exp(-|xi - xj|^2 / 2 l^2) + mu I) (kernels.c:680-1289) over its 3-D points."""

    def __init__(self, z):
        from oracle import gaussian_block
        X, f, l, mu = np.asarray(z["X"]), float(z["f"]), float(z["l"]), float(z["mu"])
        n = X.shape[0]
        idx = np.arange(n)
        self.K = gaussian_block(X, f, l, idx, idx) + f * f * mu * np.eye(n)
        self.n = n
        self.h = None

        def mv(_m, nn, alpha, xp, beta, yp):
            xv = np.ctypeslib.as_array(C.cast(xp, _lib.dp), shape=(nn,))
            yv = np.ctypeslib.as_array(C.cast(yp, _lib.dp), shape=(nn,))
            yv[:] = alpha * (self.K @ xv) + (beta * yv if beta != 0.0 else 0.0)
            return 0

        self._cb = _lib.SYMMATVEC(mv)
        self.matvec_fnptr = C.cast(self._cb, C.c_void_p).value


def _fsai(z, pre="fsai"):
    return amd.FsaiPrecond(z[pre + "_i"], z[pre + "_j"], z[pre + "_a"])


def _afn(z):
    from oracle import gaussian_block
    X, f, l = np.asarray(z["X"]), float(z["f"]), float(z["l"])
    k, perm = int(z["afn_k"]), np.asarray(z["afn_perm"])
    S = _fsai(z, "schur")
    return amd.AfnPrecond(perm, z["afn_L11"], gaussian_block(X, f, l, perm[:k], perm[k:]), S)


def test_fsai_apply_is_bitwise_reference(torch_cuda):
    """Each CSR row is summed in Nfft4GPCsrMv's order with unfused multiply and add (matops.c:231-262):
    the result equals the reference's Nfft4GPPrecondFsaiSolve bit for bit, device and host vectors."""
    torch = torch_cuda
    z = load("precond_synth")
    pre = _fsai(z)
    r = np.asarray(z["fsai_rhs"])
    xd = torch.zeros(r.size, dtype=torch.float64, device="cuda")
    pre.solve(xd, torch.tensor(r, device="cuda"))
    np.testing.assert_array_equal(xd.cpu().numpy(), z["fsai_out"])
    xh = np.zeros(r.size)
    pre.solve(xh, r.copy())
    np.testing.assert_array_equal(xh, z["fsai_out"])


def test_afn_apply_matches_golden(torch_cuda):
    torch = torch_cuda
    z = load("precond_synth")
    pre = _afn(z)
    r = np.asarray(z["afn_rhs"])
    xd = torch.zeros(r.size, dtype=torch.float64, device="cuda")
    pre.solve(xd, torch.tensor(r, device="cuda"))
    assert rel(xd.cpu().numpy(), z["afn_out"]) <= 1e-12
    xh = np.zeros(r.size)
    pre.solve(xh, r.copy())
    assert rel(xh, z["afn_out"]) <= 1e-12


@pytest.mark.parametrize("k", [0, "n"])
def test_afn_apply_edge_ranks(torch_cuda, k):
    """afn.c:101-110: k = n solves with A11 on the UNPERMUTED rhs, k = 0 is the Schur FSAI alone."""
    import scipy.linalg as sl
    from oracle import afn_apply, fsai_apply, gaussian_block
    torch = torch_cuda
    rng = np.random.default_rng(5)
    n = 300
    X = rng.random((n, 2))
    perm = rng.permutation(n).astype(np.int32)
    r = rng.random(n) - 0.5
    if k == 0:
        z = load("precond_synth")
        ia, ja, aa = (np.asarray(z[c]) for c in ("fsai_i", "fsai_j", "fsai_a"))
        n = ia.size - 1
        r = rng.random(n) - 0.5
        S = amd.FsaiPrecond(ia, ja, aa)
        pre = amd.AfnPrecond(np.arange(n), np.zeros((0, 0)), np.zeros((0, n)), S)
        ref = afn_apply(np.arange(n), np.zeros((0, 0)), None, lambda v: fsai_apply(ia, ja, aa, v), r)
    else:
        A = gaussian_block(X, 1.0, 0.3, perm, perm) + 0.05 * np.eye(n)
        L = sl.cholesky(A, lower=True)
        pre = amd.AfnPrecond(perm, L, np.zeros((n, 0)), None)
        ref = afn_apply(perm, L, None, None, r)
    xd = torch.zeros(n, dtype=torch.float64, device="cuda")
    pre.solve(xd, torch.tensor(r, device="cuda"))
    assert rel(xd.cpu().numpy(), ref) <= 1e-11


@pytest.mark.parametrize("kind", ["fsai", "afn"])
def test_pcg_with_fsai_afn_matches_golden(torch_cuda, kind):
    """This library's PCG (device vectors, the preconditioner called with device pointers) against the
    reference's pcg.c with the reference's FSAI / the restated AFN on the same dense operator."""
    torch = torch_cuda
    z = load("precond_synth")
    op = DenseGaussHostOp(z)
    pre = _fsai(z) if kind == "fsai" else _afn(z)
    key = "pcg" + kind
    b = torch.tensor(np.asarray(z["b"]), device="cuda")
    x = torch.zeros(op.n, dtype=torch.float64, device="cuda")
    x, rr, hist, it = amd.pcg(op, b, x, maxits=1000, tol=1e-6, precond=pre)
    it_ref = int(z[key + "_iters"])
    assert it > 0 and abs(it - it_ref) <= max(2, it_ref // 20), (it, it_ref)
    assert rr <= 1e-6
    assert rel(x.cpu().numpy(), z[key + "_x"]) < 1e-5
    k = min(10, it, it_ref)
    np.testing.assert_allclose(hist[:k], np.asarray(z[key + "_hist"])[:k], rtol=1e-6)
