"""GPU tests of the device-resident PCG, vector ops and the Nystrom apply against the reference's own
compiled code (oracle/_ref: pcg.c, vecops.c, nys.c) driven with the oracle's NFFT matvec."""
import numpy as np
import pytest

import oracle as O
from oracle import OracleAdditiveNFFT

import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd

pytestmark = pytest.mark.gpu
needs_ref = pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built")


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / np.linalg.norm(np.asarray(b)))


def problem(n=4000, d=4, seed=906, l=0.1, mu=0.01):
    rng = np.random.default_rng(seed)
    X = rng.random((n, d))
    b = rng.random(n) - 0.5
    win = np.arange(d, dtype=np.int32)
    op = amd.NFFTAdditiveKernel(X, win, d, 1)
    assert op.setup(amd.GAUSSIAN, 1.0, l, mu) == 0
    orc = OracleAdditiveNFFT(X, win, d, 1)
    orc.setup(0, 1.0, l, mu)
    return X, b, win, op, orc


def test_vecops_host_and_device(torch_cuda):
    torch = torch_cuda
    L = amd.lib()
    rng = np.random.default_rng(0)
    n = 100_003
    x = rng.random(n)
    y = rng.random(n)
    assert abs(L.Nfft4GPVecDdot(x.ctypes.data, n, y.ctypes.data) - x @ y) <= 1e-12 * abs(x @ y)
    assert abs(L.Nfft4GPVecNorm2(x.ctypes.data, n) - np.linalg.norm(x)) <= 1e-12 * np.linalg.norm(x)
    xd = torch.tensor(x, device="cuda")
    yd = torch.tensor(y, device="cuda")
    assert abs(L.Nfft4GPVecDdot(xd.data_ptr(), n, yd.data_ptr()) - x @ y) <= 1e-12 * abs(x @ y)
    L.Nfft4GPVecAxpy(0.5, xd.data_ptr(), n, yd.data_ptr())
    np.testing.assert_allclose(yd.cpu().numpy(), y + 0.5 * x, rtol=1e-14, atol=1e-15)
    L.Nfft4GPVecScale(yd.data_ptr(), n, 2.0)
    np.testing.assert_allclose(yd.cpu().numpy(), 2 * (y + 0.5 * x), rtol=1e-14, atol=1e-15)
    yd.fill_(float("nan"))
    L.Nfft4GPVecScale(yd.data_ptr(), n, 0.0)  # scale 0 fills zeros (vecops.c:74-77)
    assert float(yd.abs().sum()) == 0.0
    h = x.copy()
    L.Nfft4GPVecFill(h.ctypes.data, n, 3.0)
    assert np.all(h == 3.0)
    h2 = y.copy()
    L.Nfft4GPVecAxpy(-1.5, x.ctypes.data, n, h2.ctypes.data)
    np.testing.assert_allclose(h2, y - 1.5 * x, rtol=1e-14, atol=1e-15)


@needs_ref
@pytest.mark.parametrize("ptrs", ["host", "device"])
def test_pcg_matches_reference_pcg(torch_cuda, ptrs):
    torch = torch_cuda
    n = 4000
    X, b, win, op, orc = problem(n)

    def mv(alpha, xv, beta, yv):
        yv[:] = orc.matsymv(np.array(xv), alpha, beta, np.array(yv))

    x_ref, rr_ref, hist_ref, it_ref = O.ref_pcg(mv, n, b, maxits=2000, tol=1e-6)
    assert it_ref > 0
    if ptrs == "host":
        x, rr, hist, it = amd.pcg(op, b.copy(), np.zeros(n), maxits=2000, tol=1e-6)
    else:
        xd = torch.zeros(n, dtype=torch.float64, device="cuda")
        x, rr, hist, it = amd.pcg(op, torch.tensor(b, device="cuda"), xd, maxits=2000, tol=1e-6)
        x = x.cpu().numpy()
    assert it > 0 and rr <= 1e-6
    assert abs(it - it_ref) <= max(2, int(0.05 * it_ref)), (it, it_ref)
    # CG residual histories are chaotic in finite precision (1e-10 matvec differences grow with
    # the iteration); compare the early, well-conditioned part and the outcome
    k = min(8, it, it_ref)
    np.testing.assert_allclose(hist[:k], hist_ref[:k], rtol=1e-4)
    assert rel(x, x_ref) <= 1e-4


def test_pcg_early_exits(torch_cuda):
    n = 2000
    X, b, win, op, orc = problem(n)
    x, rr, hist, it = amd.pcg(op, np.zeros(n), np.ones(n), maxits=100, tol=1e-6)
    assert it == 0 and rr == 0.0 and len(hist) == 1 and np.all(x == 0)   # pcg.c:32-41
    xs, _, _, it1 = amd.pcg(op, b.copy(), np.zeros(n), maxits=2000, tol=1e-8)
    assert it1 > 0
    x2, rr2, hist2, it2 = amd.pcg(op, b.copy(), xs.copy(), maxits=100, tol=1e-6)
    assert it2 == 0 and len(hist2) == 1 and rr2 < 1e-6                   # pcg.c:70-84
    # not converged within maxits -> iter stays 0 (pcg.c:19,197)
    _, rr3, hist3, it3 = amd.pcg(op, b.copy(), np.zeros(n), maxits=3, tol=1e-12)
    assert it3 == 0 and len(hist3) == 4 and rr3 > 1e-12


@needs_ref
def test_nystrom_apply_matches_reference(torch_cuda):
    torch = torch_cuda
    n, d, k = 3000, 4, 64
    rng = np.random.default_rng(5)
    X = rng.random((n, d))
    win = np.arange(d, dtype=np.int32)
    dense = O.RefDenseAdditive(X, win, d, 1, kernel=0)
    perm = rng.permutation(n).astype(np.int32)
    nys = O.RefNystrom(dense, 1.0, 0.1, 0.01, k, perm)
    U, s, eta, p = nys.factors()
    pre = amd.NystromPrecond(U, s, eta, p)
    r = rng.random(n) - 0.5
    x_ref = nys.solve(np.zeros(n), r.copy())
    x = pre.solve(np.zeros(n), r.copy())
    assert rel(x, x_ref) <= 1e-12
    xd = torch.zeros(n, dtype=torch.float64, device="cuda")
    pre.solve(xd, torch.tensor(r, device="cuda"))
    assert rel(xd.cpu().numpy(), x_ref) <= 1e-12


@needs_ref
def test_preconditioned_pcg_matches_reference(torch_cuda):
    # rank 32: at k >= 128 the reference's Nystrom setup on this 4-window problem hits its tiny
    # singular value branch (matops.c:124-127) and returns NaN factors
    n, d, k = 4000, 4, 32
    X, b, win, op, orc = problem(n)
    rng = np.random.default_rng(6)
    dense = O.RefDenseAdditive(X, win, d, 1, kernel=0)
    nys = O.RefNystrom(dense, 1.0, 0.1, 0.01, k, rng.permutation(n).astype(np.int32))
    U, s, eta, p = nys.factors()
    pre = amd.NystromPrecond(U, s, eta, p)

    def mv(alpha, xv, beta, yv):
        yv[:] = orc.matsymv(np.array(xv), alpha, beta, np.array(yv))

    def pc(xv, rv):
        xv[:] = nys.solve(np.zeros(n), np.array(rv))

    x_ref, rr_ref, hist_ref, it_ref = O.ref_pcg(mv, n, b, maxits=2000, tol=1e-6, precond_py=pc)
    x, rr, hist, it = amd.pcg(op, b.copy(), np.zeros(n), maxits=2000, tol=1e-6, precond=pre)
    assert it_ref > 0 and it > 0
    assert abs(it - it_ref) <= max(2, int(0.05 * it_ref)), (it, it_ref)
    assert rel(x, x_ref) <= 1e-4


# ---- GPU Nystrom setup (Nfft4GPAmdNysSetupAdditive) vs the reference's nys.c setup -------------------
@needs_ref
# cases where the reference's own factors are finite and moderately conditioned (its K11 quirk makes
# e.g. a Gaussian at l = 0.3 with k = 64 produce s ~ 1e-16 and NaN columns)
@pytest.mark.parametrize("kernel,l,k", [(0, 0.1, 32), (0, 0.05, 64), (0, 0.03, 128), (1, 1.0, 48), (1, 0.3, 96)])
def test_gpu_nystrom_setup_matches_reference(torch_cuda, kernel, l, k):
    torch = torch_cuda
    n, d = 3000, 4
    rng = np.random.default_rng(21)
    X = rng.random((n, d))
    win = np.arange(d, dtype=np.int32)
    f, mu = 1.2, 0.02
    perm = rng.permutation(n).astype(np.int32)
    dense = O.RefDenseAdditive(X, win, d, 1, kernel=kernel)
    ref = O.RefNystrom(dense, f, l, mu, k, perm)
    U_ref, s_ref, eta_ref, _ = ref.factors()
    op = amd.NFFTAdditiveKernel(X, win, d, 1)
    assert op.setup(kernel, f, l, mu) == 0
    pre = amd.NystromPrecond.from_additive(op, perm, k, k11="reference")
    U, s, eta = pre.factors(perm)
    assert eta == pytest.approx(eta_ref, rel=1e-15)
    np.testing.assert_allclose(s, s_ref, rtol=1e-7)
    # eigenvector signs are arbitrary: compare columns up to sign, and the sign-free apply
    sign = np.sign(np.sum(U * U_ref, axis=0))
    np.testing.assert_allclose(U * sign, U_ref, rtol=0, atol=1e-7 * np.abs(U_ref).max())
    r = rng.random(n) - 0.5
    x_ref = ref.solve(np.zeros(n), r.copy())
    xd = torch.zeros(n, dtype=torch.float64, device="cuda")
    pre.solve(xd, torch.tensor(r, device="cuda"))
    assert rel(xd.cpu().numpy(), x_ref) < 1e-7


def test_gpu_nystrom_setup_orthonormal_large(torch_cuda):
    """Full-size property: U = U1 V w^{-1/2} has orthonormal columns (n = 2e5, k = 256, 16 windows; the
    additive kernel's numerical rank, ~30 per 1-D window at l = 0.1, stays above k)."""
    n, d, k = 200_000, 16, 256
    rng = np.random.default_rng(22)
    X = rng.random((n, d))
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    assert op.setup(amd.GAUSSIAN, 1.0, 0.1, 0.01) == 0
    pre = amd.NystromPrecond.from_additive(op, rng.permutation(n).astype(np.int32), k, k11="landmarks")
    U, s, eta = pre.factors()
    assert np.all(np.isfinite(U)) and np.all(s > 0) and np.all(np.diff(s) >= -1e-12 * s.max())
    G = U.T @ U
    assert np.abs(G - np.eye(k)).max() < 1e-6


@pytest.mark.parametrize("kernel,l", [(0, 0.1), (1, 1.0)])
def test_gpu_nystrom_landmarks_matches_numpy(torch_cuda, kernel, l):
    """k11 = "landmarks": the same pipeline with K11 = K(perm[:k], perm[:k]), restated in numpy."""
    n, d, k, f, mu = 2500, 3, 40, 1.1, 0.05
    rng = np.random.default_rng(23)
    X = rng.random((n, d))
    perm = rng.permutation(n).astype(np.int32)
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    assert op.setup(kernel, f, l, mu) == 0
    pre = amd.NystromPrecond.from_additive(op, perm, k, k11="landmarks")
    U, s, eta = pre.factors(perm)

    def kern(r2):
        return np.exp(-r2 / (2 * l * l)) if kernel == 0 else np.exp(-np.sqrt(r2) / l)

    Kp = sum(kern((X[perm, w][:, None] - X[perm[:k], w][None, :]) ** 2) for w in range(d)) * f * f / d
    K11 = Kp[:k].copy()
    fro = np.linalg.norm(K11)
    Lc = np.linalg.cholesky(K11 + np.sqrt(k) * (np.nextafter(fro, fro + 1) - fro) * np.eye(k))
    U1 = Kp @ np.linalg.inv(Lc).T
    w1, V = np.linalg.eigh(U1.T @ U1)
    Ur = (U1 @ V[:, ::-1]) / np.sqrt(w1[::-1])
    s_r = 1.0 / (w1[::-1] + mu * f * f)
    np.testing.assert_allclose(s, s_r, rtol=1e-7)
    sign = np.sign(np.sum(U * Ur, axis=0))
    np.testing.assert_allclose(U * sign, Ur, rtol=0, atol=1e-7 * np.abs(Ur).max())


@pytest.mark.parametrize("tA,M,N,K", [(0, 128, 128, 16), (0, 300, 200, 37), (0, 1000, 512, 512),
                                      (1, 128, 128, 16), (1, 130, 70, 300), (1, 256, 256, 4099)])
def test_mfma_gemm_f64_ragged(torch_cuda, tA, M, N, K):
    """The MFMA f64 GEMM behind the Nystrom setup (128 x 128 tiles, K steps of 16, swapped operands)
    on ragged shapes in both A layouts, against numpy."""
    import ctypes as C
    torch = torch_cuda
    f = amd.lib().Nfft4GPAmdDebugGemm
    f.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_longlong, C.c_void_p, C.c_longlong,
                  C.c_void_p, C.c_longlong]
    rng = np.random.default_rng(M + N + K)
    A = rng.standard_normal((K, M) if tA else (M, K))
    Bm = rng.standard_normal((K, N))
    ref = (A.T if tA else A) @ Bm
    Ad = torch.tensor(A.ravel(order="F"), device="cuda")
    Bd = torch.tensor(Bm.ravel(order="F"), device="cuda")
    Cd = torch.full((M * N,), np.nan, dtype=torch.float64, device="cuda")
    assert f(tA, M, N, K, Ad.data_ptr(), A.shape[0], Bd.data_ptr(), K, Cd.data_ptr(), M) == 0
    Cm = Cd.cpu().numpy().reshape(N, M).T
    assert np.abs(Cm - ref).max() <= 1e-12 * np.sqrt(K) * np.abs(ref).max()


def test_nystrom_fp32_storage_pcg(torch_cuda):
    """Nfft4GPAmdNysSetStorage(32): the apply reads an fp32 copy of U (fp64 accumulation).  The apply moves
    by ~1e-7 relative; PCG still stops on its fp64 true residual (pcg.c:181-193), so it reaches the same
    tolerance, in about as many iterations."""
    torch = torch_cuda
    n, d, k = 20000, 8, 64
    rng = np.random.default_rng(51)
    X = rng.random((n, d))
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    assert op.setup(amd.GAUSSIAN, 1.0, 0.1, 0.01) == 0
    pre = amd.NystromPrecond.from_additive(op, rng.permutation(n).astype(np.int32), k, k11="landmarks")
    r = torch.tensor(rng.random(n) - 0.5, device="cuda")
    z64 = torch.zeros(n, dtype=torch.float64, device="cuda")
    pre.solve(z64, r)
    b = torch.tensor(rng.random(n) - 0.5, device="cuda")
    x64 = torch.zeros(n, dtype=torch.float64, device="cuda")
    _, rel64, _, it64 = amd.pcg(op, b, x64, maxits=2000, tol=1e-6, precond=pre)
    pre.set_storage(32)
    z32 = torch.zeros(n, dtype=torch.float64, device="cuda")
    pre.solve(z32, r)
    assert rel(z32.cpu().numpy(), z64.cpu().numpy()) < 1e-6
    x32 = torch.zeros(n, dtype=torch.float64, device="cuda")
    _, rel32, _, it32 = amd.pcg(op, b, x32, maxits=2000, tol=1e-6, precond=pre)
    assert it64 > 0 and it32 > 0 and rel32 <= 1e-6
    assert abs(it32 - it64) <= max(2, it64 // 10), (it32, it64)
    pre.set_storage(64)
    z = torch.zeros(n, dtype=torch.float64, device="cuda")
    pre.solve(z, r)
    assert torch.equal(z, z64)
    pre.free()


def test_nystrom_landmarks_rank_above_numerical_rank(torch_cuda):
    """k11 = "landmarks" with k above the kernel's numerical rank: eigenvalues of U1'U1 at rounding level
    (negative ones would give NaN factors through sqrt, as in the reference's Nfft4GPTrilNystromSvd) drop
    their columns; the factors stay finite and PCG converges in a few iterations."""
    torch = torch_cuda
    rng = np.random.default_rng(8)
    n, d, k = 20000, 2, 300
    X = rng.random((n, d))
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    assert op.setup(amd.GAUSSIAN, 1.0, 0.1, 0.01) == 0  # l = 0.1: the NFFT operator is SPD
    pre = amd.NystromPrecond.from_additive(op, rng.permutation(n).astype(np.int32), k, k11="landmarks")
    b = torch.tensor(rng.random(n) - 0.5, device="cuda")
    x = torch.zeros(n, dtype=torch.float64, device="cuda")
    z = torch.zeros(n, dtype=torch.float64, device="cuda")
    pre.solve(z, b)
    assert torch.isfinite(z).all()
    _, rr, _, it = amd.pcg(op, b, x, maxits=500, tol=1e-8, precond=pre)
    assert 0 < it <= 20 and rr <= 1e-8, (it, rr)
