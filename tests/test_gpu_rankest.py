"""GPU rank estimation (Nfft4GPAmdRankestNysScaled / Default / AfnRankEstimate, afn_setup.hip) against
the reference's rankest.c compiled in oracle/_ref, after the same srand(): both draw the subsamples
with libc rand() in the same sequence (Nfft4GPRandPerm, utils.c:72-105), so the estimated ranks and the
selected points must agree exactly."""
import ctypes as C

import numpy as np
import pytest

import oracle as O

from preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd import _lib

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built")]
LIBC = C.CDLL(None)
CASES = [(5000, 2, 0.5, 0.01, 300), (5000, 3, 0.1, 0.01, 300), (20000, 2, 1.0, 0.001, 500), (3000, 4, 0.3, 0.05, 200)]


@pytest.mark.parametrize("n,d,l,mu,max_rank", CASES)
def test_rankest_nys_scaled_matches_reference(torch_cuda, n, d, l, mu, max_rank):
    X = np.asfortranarray(np.random.default_rng(n + d).random((n, d)))
    P = O.ref_gaussian_params(1.0, l, mu, n)
    r_ref = O.ref_rankest(X, P, max_rank, seed=11)
    LIBC.srand(11)
    r = _lib.lib().Nfft4GPAmdRankestNysScaled(X.ctypes.data, n, n, d, 0, P, max_rank, 500, 5)
    assert r == r_ref


@pytest.mark.parametrize("n,d,l,mu,max_rank", CASES)
def test_rankest_default_matches_reference(torch_cuda, n, d, l, mu, max_rank):
    X = np.asfortranarray(np.random.default_rng(n + d).random((n, d)))
    P = O.ref_gaussian_params(1.0, l, mu, n)
    r_ref, p_ref = O.ref_rankest(X, P, max_rank, which="default", seed=12)
    LIBC.srand(12)
    perm = np.zeros(max_rank, np.int32)
    r = _lib.lib().Nfft4GPAmdRankestDefault(X.ctypes.data, n, n, d, 0, P, max_rank, 500, 5, 0.9, perm.ctypes.data)
    assert r == r_ref
    np.testing.assert_array_equal(perm[:r], p_ref)


def ref_afn_rank(X, P, max_k, perm_opt, nsamples, seed):
    """afn.c:165-256 restated over the reference's compiled rankest / ordering / Nfft4GPRandPerm."""
    lib = O.ref_lib()
    lib.Nfft4GPRandPerm.restype = O._ip
    lib.Nfft4GPRandPerm.argtypes = [C.c_int, C.c_int]
    n = X.shape[0]
    max_k = min(max_k, n)
    LIBC.srand(seed)

    def rand_perm(k):
        p = lib.Nfft4GPRandPerm(n, k)
        out = np.ctypeslib.as_array(p, shape=(k,)).copy()
        LIBC.free(p)
        return out

    rank = O.ref_rankest(X, P, max_k, nsample=nsamples)
    if rank >= max_k:
        k = max_k
        sel = O.ref_sort_fps(X, k)[0] if perm_opt == 1 else rand_perm(k)
    else:
        k, sel = O.ref_rankest(X, P, max_k, nsample=nsamples, which="default")
        if k == max_k and perm_opt == 0:
            sel = rand_perm(k)
    return k, sel


@pytest.mark.parametrize("n,d,l,mu,max_k,perm_opt", [(5000, 3, 0.1, 0.01, 300, 1), (5000, 3, 0.1, 0.01, 300, 0),
                                                     (5000, 2, 0.5, 0.01, 300, 1), (4000, 2, 0.05, 0.01, 100, 1)])
def test_afn_rank_estimate_matches_reference_flow(torch_cuda, n, d, l, mu, max_k, perm_opt):
    X = np.asfortranarray(np.random.default_rng(n + d + max_k).random((n, d)))
    P = O.ref_gaussian_params(1.0, l, mu, n)
    k_ref, sel_ref = ref_afn_rank(X, P, max_k, perm_opt, 500, seed=13)
    LIBC.srand(13)
    perm = np.zeros(n, np.int32)
    k = _lib.lib().Nfft4GPAmdAfnRankEstimate(X.ctypes.data, n, n, d, max_k, perm_opt, 500, 0, P, perm.ctypes.data)
    assert k == k_ref
    if perm_opt == 1 or k < max_k:
        np.testing.assert_array_equal(perm[:len(sel_ref)], sel_ref)
    else:  # the random sample as a set (Nfft4GPRandPerm's quick-split order is not reproduced)
        np.testing.assert_array_equal(np.sort(perm[:k]), np.sort(sel_ref))
    np.testing.assert_array_equal(np.sort(perm), np.arange(n))


def test_afn_rank_estimate_front_end_then_setup(torch_cuda):
    """amd.afn_rank_estimate then AfnPrecond.setup with its k and order: PCG on the dense kernel
    converges faster than without a preconditioner."""
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    from test_gpu_golden import DenseGaussHostOp
    torch = torch_cuda
    rng = np.random.default_rng(2)
    n, d, f, l, mu = 3000, 3, 1.0, 0.1, 0.01
    X = rng.random((n, d))
    k, perm = amd.afn_rank_estimate(X, 300, f, l, mu, perm_opt="fps")
    assert 0 < k <= 300
    pre = amd.AfnPrecond.setup(X, k, f, l, mu, perm_opt="perm", perm=perm, schur_lfil=20)
    op = DenseGaussHostOp({"X": X, "f": f, "l": l, "mu": mu})
    b = torch.tensor(rng.random(n) - 0.5, device="cuda")
    x0 = torch.zeros(n, dtype=torch.float64, device="cuda")
    _, rr, _, it = amd.pcg(op, b, x0.clone(), maxits=2000, tol=1e-8, precond=pre)
    _, rr0, _, it0 = amd.pcg(op, b, x0.clone(), maxits=2000, tol=1e-8)
    assert rr <= 1e-8 and it > 0 and (it0 == 0 or it < it0), (it, it0)


def test_afn_rank_estimate_additive_kernel(torch_cuda):
    """With this library's additive NFFT handle as the kernel, the subsamples' kernel matrices are the dense
    additive kernel of their window coordinates: a 1-D-window additive kernel in 6 features has a much
    smaller numerical rank than the 6-D Gaussian of the same length scale, so the estimate is smaller."""
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    rng = np.random.default_rng(6)
    n, d, f, l, mu = 20000, 6, 1.0, 0.3, 0.001
    X = np.asfortranarray(rng.random((n, d)))
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    op.setup(amd.GAUSSIAN, f, l, mu)
    L = _lib.lib()
    P = _lib.kernel_params(f, l, mu, n)
    LIBC.srand(3)
    r_plain = L.Nfft4GPAmdRankestNysScaled(X.ctypes.data, n, n, d, 0, P, 2000, 500, 5)
    LIBC.srand(3)
    r_add = L.Nfft4GPAmdRankestNysScaled(X.ctypes.data, n, n, d, 0, op.h, 2000, 500, 5)
    L.Nfft4GPKernelParamFree(P)
    assert r_plain >= 0 and r_add >= 0
    assert r_add < r_plain, (r_add, r_plain)
