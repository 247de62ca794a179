"""CPU tests of the product's host logic (no GPU): C-ABI library, setup math, chunk layout, and a
numpy replay of the kernels' arithmetic against the oracle."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
from emulate import EmulatedPlan, circulant, layout, prepare, tap_poly
from oracle import OracleAdditiveNFFT, oracle_lib


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / np.linalg.norm(np.asarray(b)))


def test_library_exports_every_header_symbol():
    syms = amd.header_symbols()
    assert len(syms) >= 40
    out = subprocess.run(["nm", "-D", "--defined-only", amd._lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    L = amd.lib()
    for s in syms:
        assert getattr(L, s) is not None
    assert b"gfx950" in L.Nfft4GPAmdVersion()


def test_library_is_gfx950_code_object():
    """Every device code object in the library targets gfx950 (bundle target ids); rocPRIM's host code carries
    other architectures' names only as strings of its run-time config lookup."""
    import re
    blob = open(amd._lib.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_struct_layout_matches_reference():
    # SRC/linearalg/kernels.h:65-95 on LP64
    st = amd._lib.NfftKernelStruct
    assert st._params.offset == 0 and st._iparams.offset == 40
    assert st._noise_level.offset == 72 and st._buffer.offset == 88
    assert st._external.offset == 168 and C.sizeof(st) == 176


@pytest.mark.skipif(os.environ.get("HIP_VISIBLE_DEVICES") is None and amd.lib().Nfft4GPAmdDeviceAvailable(),
                    reason="a GPU is visible")
def test_no_device_fails_loudly():
    L = amd.lib()
    assert L.Nfft4GPAmdDeviceAvailable() == 0
    rng = np.random.default_rng(0)
    X = rng.random((100, 2))
    op = amd.NFFTAdditiveKernel(X, np.array([0, 1], np.int32), 2, 1)
    assert op.setup(amd.GAUSSIAN, 1.0, 1.0, 0.01) == -1
    with pytest.raises(RuntimeError):
        op.matsymv(np.zeros(100))


def test_tap_polynomials_match_window():
    Cm = tap_poly()
    lib = oracle_lib()
    u = np.linspace(-0.5, 0.5, 2001)
    peak = lib.orc_window_phi(0.0)
    err = 0.0
    for t in range(10):
        exact = np.array([lib.orc_window_phi(uu + 0.5 + 4 - t) for uu in u])
        approx = np.polynomial.polynomial.polyval(u, Cm[t])
        err = max(err, np.max(np.abs(exact - approx)) / peak)
    # Chebyshev-node interpolation error of the degree-(NC-1) tap polynomials (window.cpp)
    bound = {12: 1e-12, 10: 5e-10, 8: 5e-8}[Cm.shape[1]]
    assert err < bound, err


def test_bhat_and_circulant_match_oracle():
    rng = np.random.default_rng(1)
    X = rng.random((500, 1))
    orc = OracleAdditiveNFFT(X, np.array([0], np.int32), 1, 1)
    for kernel in (0, 1):
        orc.setup(kernel, 1.0, 0.7, 0.01)
        info = orc.comp_info(0)
        bh, _ = circulant(0 if kernel == 0 else 2, info["sigma0"], 1.0)
        np.testing.assert_allclose(bh, info["bhat"], rtol=1e-12, atol=1e-15)
        bhd, _ = circulant(1 if kernel == 0 else 3, info["sigma0"], 1.0)
        np.testing.assert_allclose(bhd, info["bhat_d"], rtol=1e-12, atol=1e-15)


def test_prepare_matches_reference_scaling():
    rng = np.random.default_rng(2)
    X = rng.random((3000, 1)) * 7.0 - 2.0
    orc = OracleAdditiveNFFT(X, np.array([0], np.int32), 1, 1)
    orc.setup(0, 1.0, 1.0, 0.01)
    sc, q = prepare(X[:, 0])
    assert sc == orc.comp_info(0)["scale"]
    xs = orc.comp_points(0)[:, 0]
    # 32-bit fixed point of x mod 1: error <= 2^-33
    back = (q.astype(np.int64) - (q >= 2 ** 31) * 2 ** 32) / 2.0 ** 32
    assert np.max(np.abs(back - xs)) <= 2.0 ** -33
    # radius already in [0.125, 0.25] -> scale 1 (nfft_interface.c:188-196)
    sc2, _ = prepare(np.linspace(-0.2, 0.2, 101) + 5.0)
    assert sc2 == 1.0
    assert prepare(np.full(10, 3.0))[0] == -1.0


@pytest.mark.parametrize("n,B,CG,rec", [(10000, 4064, 8, 5), (5000, 1000, 3, 5), (777, 4064, 2, 5), (9000, 256, 3, 5),
                                        (10000, 4064, 4, 4), (5000, 1024, 3, 4)])
def test_layout_invariants(n, B, CG, rec):
    """The chunk layout of both records (rec 4: the 32-bit precision mode's one word per slot, whose offset may move
    by up to 2^-21 of a cell to carry the 12-bit local index in its low bits)."""
    nw = 5
    rng = np.random.default_rng(n)
    qc = np.zeros((nw, n), np.uint32)
    for c in range(nw):
        x = rng.beta(0.5, 2.0, n) if c == 0 else rng.random(n)
        _, qc[c] = prepare(x)
    L = layout(qc.ravel(), n, nw, B, CG, rec)
    meta, loc, q = L["meta"], L["loc"], L["q"]
    comp, cell = meta >> 6, meta & 63
    seen = np.zeros((nw, n), np.int64)
    ng = L["ngroups"]
    assert ng == (nw + CG - 1) // CG and L["nblocks"] == (n + B - 1) // B
    assert np.all(np.diff(L["tile_off"]) >= 0) and L["tile_off"][-1] == L["ntiles"]
    for b in range(L["nblocks"]):
        for g in range(ng):
            t0, t1 = L["tile_off"][b * ng + g], L["tile_off"][b * ng + g + 1]
            cc = comp[t0:t1]
            assert np.all((cc >= g * CG) & (cc < min(nw, (g + 1) * CG)))
            real = loc[t0:t1] < B
            # every real slot: its coordinate is the point's and lies in the chunk's cell
            tt, ll, rr = np.nonzero(real)
            j = b * B + loc[t0:t1][tt, ll, rr]
            c = cc[tt, ll]
            if rec == 5:
                assert np.all(q[t0:t1][tt, ll, rr] == (qc[c, j] & 0x3FFFFFF))   # offset in the cell
            else:  # the offset in 2^-32 of a cell, moved by at most 2048 units to carry the index (4095 within
                # 2048 units of the cell's ends, where the nearest congruent value would leave the cell)
                ueff = L["u"][t0:t1][tt, ll, rr]
                utrue = (qc[c, j] & 0x3FFFFFF) * 2.0 ** -26 - 0.5
                dv = np.abs(ueff - utrue) * 2.0 ** 32
                edge = np.minimum(utrue + 0.5, 0.5 - utrue) * 2.0 ** 32 < 4096
                assert np.all(dv[~edge] <= 2048) and np.all(dv <= 4095)
            assert np.all((qc[c, j] >> 26) == cell[t0:t1][tt, ll])          # the chunk's cell
            lanes = np.broadcast_to(np.arange(64)[None, :, None], loc[t0:t1].shape)
            assert np.all(loc[t0:t1][~real] == B + lanes[~real] % 32)         # dummies -> pad slots
            # bank balance: at each point slot the 32 lanes of a half mostly use distinct (loc mod 32);
            # random order repeats 36 % of residues, the unavoidable floor (residue counts != 16) is ~10 %
            conflicts = 0
            for t in range(t0, t1):
                for r in range(16):
                    for h in range(2):
                        res = loc[t, 32 * h:32 * h + 32, r] % 32
                        conflicts += 32 - len(np.unique(res))
            assert conflicts <= 0.22 * (t1 - t0) * 16 * 64
            np.add.at(seen, (c, j), 1)
    assert np.all(seen == 1)  # every (window, point) exactly once


@pytest.mark.parametrize("l,bound", [(1.0, 1e-8), (0.1, 1e-7), (0.01, 1e-6)])
def test_emulated_32bit_records_match_oracle(l, bound):
    """The 32-bit precision mode (Nfft4GPAmdSetPrecision 32: one word per (point, window), offsets to 2^-21 of a
    cell) replayed on the CPU against the oracle: within the north star's 1e-6 at TEST1's shortest length scale
    (the fp64 default's 5-byte records: ~4e-9 there)."""
    rng = np.random.default_rng(11)
    n, d = 8000, 4
    X = rng.random((n, d))
    x = rng.random(n) - 0.5
    orc = OracleAdditiveNFFT(X, np.arange(d, dtype=np.int32), d, 1)
    orc.setup(0, 1.0, l, 0.01)
    em = EmulatedPlan(X, [[c] for c in range(d)], B=4064, CG=4, rec=4)
    em.setup(0, 1.0, l, 0.01)
    e = rel(em.matsymv(x), orc.matsymv(x))
    assert e < bound, e


@pytest.mark.parametrize("kernel", [0, 1])
def test_emulated_kernels_match_oracle(kernel):
    rng = np.random.default_rng(3)
    n, d = 6000, 4
    X = rng.random((n, d))
    x = rng.random(n) - 0.5
    y0 = rng.random(3 * n)
    win = np.arange(d, dtype=np.int32)
    orc = OracleAdditiveNFFT(X, win, d, 1)
    orc.setup(kernel, 1.2, 0.8, 0.02)
    em = EmulatedPlan(X, [[c] for c in range(d)], B=1024, CG=3)
    em.setup(kernel, 1.2, 0.8, 0.02)
    assert rel(em.matsymv(x), orc.matsymv(x)) < 1e-8
    assert rel(em.matsymv(x, -1.0, 0.5, y0[:n]), orc.matsymv(x, -1.0, 0.5, y0[:n])) < 1e-8
    g = em.matsymv(x, 0.3, 2.0, y0, grad=True)
    gr = orc.gradmatsymv(x, 0.3, 2.0, y0)
    for k in range(3):
        s = slice(k * n, (k + 1) * n)
        assert rel(g[s], gr[s]) < 1e-8


def test_host_eigensolver_and_cholesky_inverse():
    """The Nystrom setup's host k x k steps (nystrom.hip) against numpy/LAPACK."""
    L = amd.lib()
    rng = np.random.default_rng(8)
    for n in (1, 7, 96, 300):
        B = rng.standard_normal((n, n))
        A = np.asfortranarray(B @ B.T + 0.5 * np.eye(n))
        w = np.zeros(n)
        V = np.zeros((n, n), order="F")
        assert L.Nfft4GPAmdHostSymEig(A.ctypes.data, n, w.ctypes.data, V.ctypes.data) == 0
        wr = np.linalg.eigvalsh(A)
        assert np.all(np.diff(w) >= 0)                                  # ascending, as dsyev
        assert np.abs(w - wr).max() <= 1e-13 * wr.max()
        assert np.abs(A @ V - V * w).max() <= 1e-12 * wr.max()
        assert np.abs(V.T @ V - np.eye(n)).max() <= 1e-13
        G = np.zeros((n, n), order="F")
        assert L.Nfft4GPAmdHostCholInverse(A.ctypes.data, n, 0.25, G.ctypes.data) == 0
        Lc = np.linalg.cholesky(A + 0.25 * np.eye(n))
        np.testing.assert_allclose(G, np.linalg.inv(Lc), rtol=0, atol=1e-12 * np.abs(np.linalg.inv(Lc)).max())
    # not positive definite: the failing column is reported
    A = np.asfortranarray(np.diag([1.0, -1.0, 2.0]))
    assert L.Nfft4GPAmdHostCholInverse(A.ctypes.data, 3, 0.0, np.zeros(9).ctypes.data) == 2


def test_transform_matches_reference_formulas():
    """Nfft4GPTransform (transform.c:4-89): softplus (with the +-20 thresholds), sigmoid, exp, identity,
    forward with derivative and inverse (host code, no device needed)."""
    L = amd.lib()
    t, dt = C.c_double(), C.c_double()
    for v in (-25.0, -3.0, 0.0, 0.7, 19.0, 25.0):
        assert L.Nfft4GPTransform(0, v, 0, C.byref(t), C.byref(dt)) == 0
        if v > 20:
            exp_t, exp_dt = v, 1.0
        elif v < -20:
            exp_t, exp_dt = np.exp(v), np.exp(v)
        else:
            exp_t, exp_dt = np.log1p(np.exp(v)), np.exp(v) / (1 + np.exp(v))
        assert t.value == pytest.approx(exp_t, rel=1e-15) and dt.value == pytest.approx(exp_dt, rel=1e-15)
        assert L.Nfft4GPTransform(0, t.value, 1, C.byref(t), None) == 0
        if -20 <= v <= 20:
            assert t.value == pytest.approx(v, rel=1e-9, abs=1e-9)
    assert L.Nfft4GPTransform(1, 0.3, 0, C.byref(t), C.byref(dt)) == 0
    s = 1 / (1 + np.exp(-0.3))
    assert t.value == pytest.approx(s) and dt.value == pytest.approx(s * (1 - s))
    assert L.Nfft4GPTransform(2, 0.3, 0, C.byref(t), C.byref(dt)) == 0
    assert t.value == pytest.approx(np.exp(0.3)) and dt.value == pytest.approx(np.exp(0.3))
    assert L.Nfft4GPTransform(3, 0.3, 0, C.byref(t), C.byref(dt)) == 0
    assert t.value == 0.3 and dt.value == 1.0
    assert L.Nfft4GPTransform(7, 0.3, 0, C.byref(t), C.byref(dt)) == -1


def test_random_vectors_follow_libc_rand():
    """Nfft4GPVecRand / Nfft4GPVecRadamacher (vecops.c:15-46): libc rand() / RAND_MAX in order, so a
    srand seed reproduces the reference's probes."""
    libc = C.CDLL(None)
    L = amd.lib()
    libc.srand(807)
    expect = np.array([libc.rand() for _ in range(1000)], dtype=np.float64) / 2147483647.0
    libc.srand(807)
    x = np.zeros(1000)
    L.Nfft4GPVecRand(x.ctypes.data, 1000)
    np.testing.assert_array_equal(x, expect)
    libc.srand(807)
    L.Nfft4GPVecRadamacher(x.ctypes.data, 1000)
    np.testing.assert_array_equal(x, np.where(expect < 0.5, -1.0, 1.0))


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                    "oracle", "_ref", "libnfft4gp_ref.so")),
                    reason="oracle/_ref not built")
def test_compiled_reference_reproduces_krylov_fixture():
    """Re-run the reference's FGMRES and logdet quadrature (oracle/_ref) from the krylov_synth inputs."""
    import oracle as O
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    z = np.load(os.path.join(gold, "pcg_synth.npz"))
    k = np.load(os.path.join(gold, "krylov_synth.npz"))
    r = O.RefDenseAdditive(z["X"], z["windows"], int(z["nw"]), int(z["dw"]), kernel=0)
    r.matrices(float(k["f"]), float(k["l"]), float(k["mu"]), grad=True)

    def mv(a, xv, b, yv):
        yv[:] = r.matsymv(xv, a, b, yv.copy())

    def dmv(a, xv, b, yv):
        yv[:] = r.gradmatsymv(xv, a, b, yv.copy())

    n = z["X"].shape[0]
    x, rr, hist, it = O.ref_fgmres(mv, n, z["b"], 100, 400, 1e-8)
    assert it == int(k["fg_iters"])
    np.testing.assert_allclose(x, k["fg_x"], rtol=1e-9, atol=1e-12)
    val, g = O.ref_logdet_quadrature(mv, dmv, n, int(k["maxits"]), int(k["nvecs"]), k["rademacher"].astype(float))
    assert val == pytest.approx(float(k["ld_val"]), rel=1e-12)
    np.testing.assert_allclose(g, k["ld_grad"], rtol=1e-10)
