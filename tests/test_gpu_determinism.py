"""The deterministic 1-D matvec (opt-in Nfft4GPAmdSetDeterministic, nfft_kernels.hip DET): at
BASELINE configs[2] (config C: n = 1e6, 32 additive 1-D windows) two matvecs, two gradient matvecs and two PCG
solves of the same input are bitwise equal, so the PCG iteration count is one number, not a range.  The reference
adds its components in a fixed order (SRC/external/nfft_interface.c:807-811); here the spread's moment-table
flushes and the interpolation's y adds are rounded to a grid on which every partial sum is exact, so the LDS
atomics' order cannot show.  That rounding costs ~2^-45 relative: the deterministic matvec stays within 1e-12 of
the plain fp64-atomic one (SetDeterministic(0)), and both within the oracle bound of test_gpu_configs.py."""
import numpy as np
import pytest

import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def config_c_op(torch_cuda):
    rng = np.random.default_rng(906)
    n, d = 1_000_000, 32
    X = rng.random((n, d))
    x = rng.random(n) - 0.5
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    assert op.setup(amd.GAUSSIAN, f=1.0, l=0.1, mu=0.01) == 0
    op.set_deterministic(True)
    yield op, torch_cuda.tensor(x, device="cuda")
    op.free()


def test_matvec_and_grad_bitwise_reproducible(torch_cuda, config_c_op):
    torch = torch_cuda
    op, xd = config_c_op
    y1 = op.matsymv(xd)
    y2 = op.matsymv(xd)
    g1 = op.gradmatsymv(xd)
    g2 = op.gradmatsymv(xd)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    assert torch.equal(g1, g2)
    # the plain fp64 atomics: within the deterministic rounding of the same operator
    op.set_deterministic(False)
    y3 = op.matsymv(xd)
    g3 = op.gradmatsymv(xd)
    op.set_deterministic(True)
    torch.cuda.synchronize()
    e = ((y1 - y3).norm() / y3.norm()).item()
    eg = ((g1 - g3).norm() / g3.norm()).item()
    print(f"deterministic vs fp64 atomics: matvec {e:.2e}, gradient {eg:.2e}")
    assert e < 1e-12 and eg < 1e-12, (e, eg)


@pytest.mark.parametrize("fusep", ["1", "0"], ids=["fused_update", "separate_update"])
def test_pcg_bitwise_reproducible(torch_cuda, config_c_op, monkeypatch, fusep):
    """Two PCG solves to 1e-6 at config C, l = 0.1 (the bench's PCG leg): the same iterations, history and x.
    The second solve of the fused_update case runs with the direction update as its own launch
    (NFFT4GP_AMD_PCG_FUSEP=0, k_pcg_pupdate): the fused k_pcg_xr does the same arithmetic, so the same bits."""
    torch = torch_cuda
    op, _ = config_c_op
    n = op.n
    b = torch.tensor(np.random.default_rng(907).random(n) - 0.5, device="cuda")
    runs = []
    for k in range(2):
        monkeypatch.setenv("NFFT4GP_AMD_PCG_FUSEP", "0" if (fusep == "0" or k == 1) else "1")
        x = torch.zeros(n, dtype=torch.float64, device="cuda")
        _, relres, hist, it = amd.pcg(op, b, x, maxits=3000, tol=1e-6)
        torch.cuda.synchronize()
        runs.append((x, relres, np.asarray(hist), it))
    (x1, r1, h1, i1), (x2, r2, h2, i2) = runs
    print(f"PCG at config C: {i1} and {i2} iterations, rel res {r1:.6e} / {r2:.6e}")
    assert i1 > 0 and i1 == i2
    assert r1 == r2
    np.testing.assert_array_equal(h1, h2)
    assert torch.equal(x1, x2)


def test_fgmres_mgs_sweep_in_one_launch_is_bitwise(torch_cuda, config_c_op, monkeypatch):
    """FGMRES with the reference's MGS (fgmres.c, matops.c:274-346): the sweep of each step in one launch
    (k_mgs_chain, the default where the grid fits) against one k_gs_step launch per projection
    (NFFT4GP_AMD_MGS_CHAIN=0): the same per-element and per-reduction arithmetic, so the same bits."""
    torch = torch_cuda
    op, _ = config_c_op
    n = op.n
    amd.lib().Nfft4GPAmdSetFgmresOrtho(0)
    b = torch.tensor(np.random.default_rng(908).random(n) - 0.5, device="cuda")
    runs = []
    for chain in ("1", "0"):
        monkeypatch.setenv("NFFT4GP_AMD_MGS_CHAIN", chain)
        x = torch.zeros(n, dtype=torch.float64, device="cuda")
        _, relres, hist, it = amd.fgmres(op, b, x, kdim=60, maxits=100, tol=1e-12)
        torch.cuda.synchronize()
        runs.append((x, relres, np.asarray(hist), it))
    (x1, r1, h1, i1), (x2, r2, h2, i2) = runs
    print(f"FGMRES(60) 100 steps: rel res {r1:.6e} / {r2:.6e}")
    assert i1 == i2 == 100
    assert r1 == r2
    np.testing.assert_array_equal(h1, h2)
    assert torch.equal(x1, x2)


@pytest.mark.parametrize("n", [1_500_000, 10_000_000], ids=["n1.5e6_S2", "n1e7_S10"])
def test_fgmres_mgs_sweep_wide_is_bitwise(torch_cuda, monkeypatch, n):
    """Past k_mgs_chain's one-pass grid (n > ~1e6) the MGS sweep runs as k_mgs_wide: w in registers over S strided
    passes, v_{j-1} re-read for each update.  Against one k_gs_step launch per projection on the same grid
    (NFFT4GP_AMD_MGS_CHAIN=0) the same per-element and per-reduction arithmetic: the same bits.  BASELINE
    configs[4]'s n = 1e7 takes S = 10 passes; 4 windows keep the operator cheap, deterministic mode keeps the two
    runs' matvecs equal."""
    torch = torch_cuda
    rng = np.random.default_rng(909)
    d = 4
    X = rng.random((n, d))
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    assert op.setup(amd.GAUSSIAN, f=1.0, l=0.1, mu=0.01) == 0
    op.set_deterministic(True)
    amd.lib().Nfft4GPAmdSetFgmresOrtho(0)
    b = torch.tensor(rng.random(n) - 0.5, device="cuda")
    runs = []
    try:
        for chain in ("1", "0"):
            monkeypatch.setenv("NFFT4GP_AMD_MGS_CHAIN", chain)
            x = torch.zeros(n, dtype=torch.float64, device="cuda")
            _, relres, hist, it = amd.fgmres(op, b, x, kdim=30, maxits=30, tol=1e-14)
            torch.cuda.synchronize()
            runs.append((x, relres, np.asarray(hist), it))
    finally:
        op.free()
    (x1, r1, h1, i1), (x2, r2, h2, i2) = runs
    print(f"n {n}: FGMRES(30) rel res {r1:.6e} / {r2:.6e}")
    assert i1 == i2 and i1 > 0
    assert r1 == r2
    np.testing.assert_array_equal(h1, h2)
    assert torch.equal(x1, x2)
