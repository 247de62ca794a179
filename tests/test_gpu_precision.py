"""The 32-bit precision mode (Nfft4GPAmdSetPrecision(h, 32), the analogue of the reference's
NFFT4GP_USING_FLOAT32, SRC/utils/utils.h:28-31, granted by BASELINE configs[4]: "fp32 matvec / fp64 accumulate"):
one 32-bit record per (point, window), the offset in the cell to 2^-21 of a cell (2^-27 of the period) with the
12-bit local index in its low bits; fp64 arithmetic.  Against the oracle it is held to the north star's 1e-6
(measured ~1e-7 at TEST1's shortest length scale); switching back to 64 gives the fp64 default bit for bit."""
import os
import sys

import numpy as np
import pytest

import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
TOL_CONTRACT = 1e-6


def rel(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def load(name):
    return np.load(os.path.join(HERE, "golden", name + ".npz"), allow_pickle=False)


@pytest.mark.parametrize("l", [1.0, 0.1])
def test_32bit_config_c_against_oracle(torch_cuda, l):
    """BASELINE configs[2] at full size (n = 1e6, 32 windows) in the 32-bit mode: matvec and the 3 gradient blocks
    within 1e-6 of the oracle."""
    from oracle import OracleAdditiveNFFT
    torch = torch_cuda
    rng = np.random.default_rng(906)
    n, d = 1_000_000, 32
    X = rng.random((n, d))
    x = rng.random(n) - 0.5
    win = np.arange(d, dtype=np.int32)
    op = amd.NFFTAdditiveKernel(X, win, d, 1)
    op.set_precision(32)
    assert op.setup(amd.GAUSSIAN, 1.0, l, 0.01) == 0
    assert op.layout_info()["layout_bytes"] < 4.6 * n * d  # one word per slot (+ padding, meta), no lo bytes
    xd = torch.tensor(x, device="cuda")
    y = op.matsymv(xd).cpu().numpy()
    g = op.gradmatsymv(xd).cpu().numpy()
    orc = OracleAdditiveNFFT(X, win, d, 1)
    orc.setup(0, 1.0, l, 0.01)
    e = rel(y, orc.matsymv(x))
    gr = orc.gradmatsymv(x)
    eg = [rel(g[i * n:(i + 1) * n], gr[i * n:(i + 1) * n]) for i in range(3)]
    print(f"32-bit mode, config C l={l}: matvec {e:.2e}, grad {', '.join(f'{v:.2e}' for v in eg)}")
    assert e <= TOL_CONTRACT and max(eg) <= TOL_CONTRACT, (e, eg)
    op.free()


@pytest.mark.parametrize("name", ["foo1d", "synth1d"])
@pytest.mark.parametrize("l", [0.01, 0.03])
def test_32bit_short_length_scales(torch_cuda, name, l):
    """TEST1's shortest length scales (TESTS/TEST1/foo.ipynb: logspace(-2, 2, 20)), where a point's position error
    is amplified most: within the north star's 1e-6."""
    from oracle import OracleAdditiveNFFT
    z = load(name)
    X = np.asarray(z["X"])
    win = np.asarray(z["windows"], np.int32)
    nw, dw = int(z["nw"]), int(z["dw"])
    x = np.asarray(z["x"])
    f, mu = float(z["f"]), float(z["mu"])
    op = amd.NFFTAdditiveKernel(X, win, nw, dw)
    op.set_precision(32)
    assert op.setup(amd.GAUSSIAN, f, l, mu) == 0
    orc = OracleAdditiveNFFT(X, win, nw, dw)
    orc.setup(0, f, l, mu)
    e = rel(op.matsymv(x), orc.matsymv(x))
    print(f"32-bit mode, {name} l={l}: matvec rel err {e:.2e}")
    assert e <= TOL_CONTRACT, e


def test_precision_switch_rebuilds_the_layout(torch_cuda):
    """SetPrecision after the first setup rebuilds the layout and re-sets the kernel; back at 64 the handle computes
    the fp64 default bit for bit (the same layout as a fresh handle)."""
    torch = torch_cuda
    rng = np.random.default_rng(4)
    n, d = 50_000, 6
    X = rng.random((n, d))
    x = torch.tensor(rng.random(n) - 0.5, device="cuda")
    win = np.arange(d, dtype=np.int32)
    a = amd.NFFTAdditiveKernel(X, win, d, 1)
    b = amd.NFFTAdditiveKernel(X, win, d, 1)
    for h in (a, b):
        assert h.setup(amd.GAUSSIAN, 1.0, 0.3, 0.01) == 0
    y64 = a.matsymv(x)
    a.set_precision(32)
    y32 = a.matsymv(x)
    bytes32 = a.layout_info()["layout_bytes"]
    a.set_precision(64)
    assert a.layout_info()["layout_bytes"] > bytes32
    e = float(torch.linalg.norm(y32 - y64) / torch.linalg.norm(y64))
    print(f"32-bit against fp64 default: {e:.2e}")
    assert 0.0 < e <= 1e-6
    # LDS atomics: equal to rounding, not bitwise (unless deterministic)
    assert float(torch.linalg.norm(a.matsymv(x) - b.matsymv(x)) / torch.linalg.norm(y64)) <= 1e-14
    a.free()
    b.free()


def test_32bit_config_e_reduced_loss(torch_cuda):
    """BASELINE configs[4] reduced (64 windows, n = 2e4): the loss and its gradient in the 32-bit mode against the
    reference's gp_loss.c on the oracle's operator.  Bound: the 32-bit records move each point by
    <= 2^-27 of the period, which perturbs the operator by eps ~ 3e-7 relative (the matvec tests above); the loss's
    quadratic term y^T K^-1 y / n and log det / n then move by at most eps kappa, kappa ~ (1 + mu) / mu = 101 here,
    so ~3e-5 relative; the tests allow 1e-4 (loss) and 3e-4 (gradient, one more operator application)."""
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_golden import config_e_inputs
    z = load("config_e_reduced")
    n, d, nvecs, maxits, seed = (int(z[k]) for k in ("n", "d", "nvecs", "maxits", "seed"))
    X, y, R = config_e_inputs(n, d, nvecs, seed)
    win = np.arange(d, dtype=np.int32)
    op = amd.NFFTAdditiveKernel(X, win, d, 1)
    op.set_precision(32)
    hyper = np.asarray(z["hyper"])
    loss, grad = amd.gp_loss(X, win, d, 1, y, hyper, maxits=maxits, nvecs=nvecs, rademacher=R, tol=1e-8,
                             transform=0, op=op)
    lerr = abs(loss - float(z["loss"])) / abs(float(z["loss"]))
    gerr = float(np.max(np.abs(np.asarray(grad) - z["grad"]) / np.maximum(np.abs(z["grad"]), 1e-9)))
    print(f"32-bit config E reduced: loss rel {lerr:.2e}, grad rel {gerr:.2e}")
    assert lerr <= 1e-4 and gerr <= 3e-4, (lerr, gerr)
    op.free()
