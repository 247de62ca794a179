"""Driver for rocprofv3: config-C PCG at l = 0.1 (the bench's PCG leg), optionally Nystrom-free.
Prints wall time and iterations; analyse the kernel trace with tools/trace_gaps.py."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd  # noqa: E402

n = int(os.environ.get("N", 1000000))
d = int(os.environ.get("D", 32))
maxits = int(os.environ.get("MAXITS", 3000))
rng = np.random.default_rng(906)
X = rng.random((n, d))
op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
assert op.setup(amd.GAUSSIAN, 1.0, 0.1, 0.01) == 0
b = torch.tensor(np.random.default_rng(907).random(n) - 0.5, device="cuda")
for rep in range(2):
    x = torch.zeros(n, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    t0 = time.time()
    _, rr, hist, it = amd.pcg(op, b, x, maxits=maxits, tol=1e-6)
    torch.cuda.synchronize()
    t = time.time() - t0
    print(f"rep {rep}: {t:.4f}s iters={it} relres={rr:.3e} ms/iter={1e3 * t / max(it, 1):.4f}", flush=True)
