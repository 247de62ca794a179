"""Config C: GPU Nystrom setup (rank k, landmarks K11) + preconditioned PCG vs plain PCG."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd  # noqa: E402

n = int(os.environ.get("N", 1000000))
d = int(os.environ.get("D", 32))
ks = [int(v) for v in os.environ.get("KS", "128,512").split(",")]
l = float(os.environ.get("L", 0.1))
rng = np.random.default_rng(906)
X = rng.random((n, d))
op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
assert op.setup(amd.GAUSSIAN, 1.0, l, 0.01) == 0
b = torch.tensor(np.random.default_rng(907).random(n) - 0.5, device="cuda")
x = torch.zeros(n, dtype=torch.float64, device="cuda")
torch.cuda.synchronize()
t0 = time.time()
_, rr, hist, it = amd.pcg(op, b, x, maxits=3000, tol=1e-6)
torch.cuda.synchronize()
print(f"plain: {time.time() - t0:.4f}s iters={it} relres={rr:.2e}", flush=True)
perm = np.random.default_rng(5).permutation(n).astype(np.int32)
for k in ks:
    torch.cuda.synchronize()
    t0 = time.time()
    pre = amd.NystromPrecond.from_additive(op, perm, k, k11="landmarks")
    torch.cuda.synchronize()
    ts = time.time() - t0
    x = torch.zeros(n, dtype=torch.float64, device="cuda")
    t0 = time.time()
    _, rr, hist, it = amd.pcg(op, b, x, maxits=3000, tol=1e-6, precond=pre)
    torch.cuda.synchronize()
    print(f"nys k={k}: setup {ts:.3f}s pcg {time.time() - t0:.4f}s iters={it} relres={rr:.2e}", flush=True)
    pre.free()
