"""AFN apply kernels in isolation (for rocprofv3 --kernel-trace --stats): n points, rank k, FPS order, the Schur
solve ("fsai": kernel FSAI, lfil 20; "noise": I / mu) and the K12 storage (64 / 32).

    python tools/afn_apply_probe.py [n] [k] [fsai|noise] [64|32]
"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 512
schur = sys.argv[3] if len(sys.argv) > 3 else "fsai"
storage = int(sys.argv[4]) if len(sys.argv) > 4 else 64
X = np.asfortranarray(np.random.default_rng(1).random((n, 3)))
pre = amd.AfnPrecond.setup(X, k, 1.0, 0.05, 0.01, perm_opt="fps", schur_lfil=20, schur=schur)
if storage == 32:
    pre.set_storage(32)
x = torch.zeros(n, dtype=torch.float64, device="cuda")
r = torch.rand(n, dtype=torch.float64, device="cuda")
for _ in range(3):
    pre.solve(x, r)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    pre.solve(x, r)
torch.cuda.synchronize()
print(f"AFN apply n={n} k={k} schur={schur} storage={storage}: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms")
