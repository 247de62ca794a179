"""How much the REFERENCE's restarted FGMRES history moves under one-ulp operator noise on the distributed
Krylov test's problem (tests/test_gpu_dist_krylov.py: config_e_reduced, n = 2e4, 64 windows, kdim 25,
maxits 120, tol 1e-10 -- it stagnates at 0.24, so the reference's restart, scaled by the Givens estimate
(fgmres.c:236-243), amplifies rounding).  The oracle's NFFT operator, its output multiplied by
(1 + 1.1e-16 N(0, 1)), seeds 1-5 against the unperturbed run.  CPU, ~3 minutes on 8 threads.

    OMP_NUM_THREADS=8 python tools/fgmres_restart_sensitivity.py
"""
import os, sys, time, numpy as np
sys.path.insert(0, '/root/repo/tests/golden'); sys.path.insert(0, '/root/repo/oracle'); sys.path.insert(0,'/root/repo/tests')
from make_golden import config_e_inputs
from oracle import ref_fgmres, OracleAdditiveNFFT
z = dict(np.load('/root/repo/tests/golden/config_e_reduced.npz'))
n, d, nvecs, maxits, seed = (int(z[k]) for k in ("n", "d", "nvecs", "maxits", "seed"))
X, y, R = config_e_inputs(n, d, nvecs, seed)
o = OracleAdditiveNFFT(X, np.arange(d, dtype=np.int32), d, 1)
o.setup(0, 1.0, 0.1, 0.01)
hs = []
for s in range(6):
    rng = np.random.default_rng(s)
    def mv(alpha, xv, beta, yv, s=s, rng=rng):
        out = o.matsymv(xv, alpha, beta, yv.copy())
        if s: out = out * (1 + 1.1e-16 * rng.standard_normal(out.shape))
        yv[:] = out
    t = time.time()
    x, rr, hist, it = ref_fgmres(mv, n, y, 25, 120, 1e-10)
    hs.append(hist[:it + 1]); print(s, it, rr, time.time() - t, flush=True)
h0 = hs[0]
for h in hs[1:]:
    m = min(len(h), len(h0))
    print("first cycle", np.max(np.abs(h[:26] - h0[:26]) / h0[:26]), "all", np.max(np.abs(h[:m] - h0[:m]) / h0[:m]))
