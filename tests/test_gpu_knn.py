"""The FSAI pattern's KNN (Nfft4GPDistanceEuclidKnn, kernels.c:121-278: row i >= lfil holds the lfil-1
nearest earlier points by (squared distance, index), then i) on the GPU: the fp32-screened scans
(k_knn_screen, the default) must give exactly the rows of the fp64 two-pass scan (k_knn_bounded) and of the
radix select over every point (k_knn), on random, clustered, tied and badly centred data; rows the screen
cannot settle fall back to k_knn (counted)."""
import ctypes as C
import time

import numpy as np
import pytest

import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd

pytestmark = pytest.mark.gpu


def knn(X, lfil, variant):
    X = np.asfortranarray(X, dtype=np.float64)
    n, d = X.shape
    f = amd.lib().Nfft4GPAmdDebugKnn
    f.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    f.restype = C.c_int
    ja = np.full((n - lfil) * lfil, -1, np.int32)
    nfail = C.c_int(-1)
    assert f(X.ctypes.data, n, n, d, lfil, variant, ja.ctypes.data, C.byref(nfail)) == 0
    return ja.reshape(n - lfil, lfil), nfail.value


def brute(X, lfil, rows):
    out = {}
    for i in rows:
        t = X[:i] - X[i]
        d2 = np.zeros(i)
        for c in range(X.shape[1]):  # the fma chain's order; ties by index
            d2 = d2 + t[:, c] * t[:, c]
        out[i] = np.lexsort((np.arange(i), d2))[: lfil - 1]
    return out


def check_same(X, lfil, expect_few_fallbacks=True):
    a, nf = knn(X, lfil, 1)
    b, _ = knn(X, lfil, 0)
    c, _ = knn(X, lfil, 2)
    e, nf3 = knn(X, lfil, 3)  # the one-launch 32-row screen
    f, nf4 = knn(X, lfil, 4)  # the one-launch 256-row bf16-split screen
    n = X.shape[0]
    assert np.array_equal(a, c) and np.array_equal(b, c) and np.array_equal(e, c) and np.array_equal(f, c)
    if expect_few_fallbacks:
        assert nf3 <= max(2, (n - lfil) // 100), nf3
        assert nf4 <= max(2, (n - lfil) // 100), nf4
    assert np.array_equal(a[:, -1], np.arange(lfil, n))
    if expect_few_fallbacks:
        assert nf <= max(2, (n - lfil) // 100), nf
    return a, nf


@pytest.mark.parametrize("n,d,lfil", [(20000, 32, 20), (6000, 3, 20), (5000, 64, 32), (3000, 8, 2), (300, 5, 64)])
def test_knn_screen_matches_exact_random(torch_cuda, n, d, lfil):
    X = np.random.default_rng(n + d).random((n, d))
    a, _ = check_same(X, lfil)
    rows = [lfil, lfil + 1, n // 2, n - 1]
    ref = brute(X, lfil, rows)
    for i in rows:
        assert np.array_equal(a[i - lfil, :-1], ref[i]), i


def test_knn_screen_clustered_and_ties(torch_cuda):
    rng = np.random.default_rng(3)
    centres = rng.random((20, 16)) * 10
    X = centres[rng.integers(0, 20, 15000)] + 0.01 * rng.standard_normal((15000, 16))
    # clusters 1e-2 wide at |x| ~ 20: the fp32 margin exceeds the neighbour distances, so most rows go on to
    # the fp64 scan (and what that leaves to the radix select) -- still the exact rows
    _, nf = check_same(X, 20, expect_few_fallbacks=False)
    assert nf > 64
    # coordinates on a coarse grid: many exactly equal distances, ties broken by index
    G = np.round(rng.random((8000, 6)) * 4) / 4
    check_same(G, 20, expect_few_fallbacks=False)


def test_knn_screen_far_from_origin_falls_back_exactly(torch_cuda):
    """Coordinates far from the origin against their spread: the fp32 margin swamps the bins, every row
    goes to the exact radix select, and the rows are still exact."""
    X = 1e4 + np.random.default_rng(5).random((4000, 8))
    a, nf = check_same(X, 20, expect_few_fallbacks=False)
    assert nf > 0


def test_knn_screen_speed_config_c_slice(torch_cuda):
    """Timing at n = 2e5, d = 32 (config C's features): the screened scans against the fp64 scans."""
    X = np.random.default_rng(906).random((200000, 32))
    t, r, nf = {}, {}, {}
    for v in (4, 3, 1, 0):
        knn(X[:30000], 20, v)
        t0 = time.time()
        r[v], nf[v] = knn(X, 20, v)
        t[v] = time.time() - t0
    assert np.array_equal(r[1], r[0]) and np.array_equal(r[3], r[0]) and np.array_equal(r[4], r[0])
    print(f"KNN n=2e5 d=32: tiled screen {t[4]:.3f} s (fallback rows {nf[4]}), one-launch screen {t[3]:.3f} s "
          f"(fallback rows {nf[3]}), two-launch screen {t[1]:.3f} s (fallback rows {nf[1]}), fp64 {t[0]:.3f} s")
    assert nf[1] <= 2000 and nf[3] <= 2000 and nf[4] <= 2000


@pytest.mark.parametrize("kind", ["random", "clustered"])
def test_knn_screen_subsampled_count(torch_cuda, kind):
    """Row groups with >= 65536 earlier points count on a systematic half of them (the subset's
    (lfil-1)-th smallest key bounds the row's, so the collect limit still holds every neighbour): the rows
    equal the fp64 scan's on random and clustered data at n = 9e4."""
    rng = np.random.default_rng(11)
    n, d = 90000, 8
    if kind == "random":
        X = rng.random((n, d))
    else:
        centres = rng.random((50, d))
        X = centres[rng.integers(0, 50, n)] + 0.02 * rng.standard_normal((n, d))
    a, nf = knn(X, 20, 1)
    b, _ = knn(X, 20, 0)
    e, nf3 = knn(X, 20, 3)
    f, nf4 = knn(X, 20, 4)
    assert np.array_equal(a, b) and np.array_equal(e, b) and np.array_equal(f, b)
    if kind == "random":
        assert nf <= (n - 20) // 100, nf
        assert nf3 <= (n - 20) // 100, nf3
        assert nf4 <= (n - 20) // 100, nf4
