import ctypes, numpy as np, sys
sys.path.insert(0, '.')
import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
import torch
libc = ctypes.CDLL(None)
X = np.random.default_rng(3).random((20000, 8))
op = amd.NFFTAdditiveKernel(X, np.arange(8, dtype=np.int32), 8, 1)
assert op.setup(0, f=1.0, l=0.5, mu=0.1) == 0
for rep in range(3):
    libc.srand(807)
    k, perm = amd.afn_rank_estimate(X, 256, perm_opt="random", op=op)
    print("est", k, perm[:5], libc.rand(), flush=True)
for rep in range(2):
    libc.srand(807)
    pre = amd.PrecondAFN(X, 256, perm_opt="random", op=op)
    print("flow", pre.kind, pre.k, libc.rand(), flush=True)
    pre.free()
L = amd.lib()
for rep in range(2):
    libc.srand(807)
    r1 = L.Nfft4GPAmdRankestNysScaled(X.ctypes.data, 20000, 20000, 8, 0, op.h, 256, 500, 5)
    print("scaled", r1, libc.rand(), flush=True)
