"""Minimal driver for rocprofv3: config-C setup + a few additive matvecs (and grad matvecs)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd  # noqa: E402

n = int(os.environ.get("N", 1000000))
d = int(os.environ.get("D", 32))
reps = int(os.environ.get("REPS", 20))
rng = np.random.default_rng(906)
X = rng.random((n, d))
x = rng.random(n) - 0.5
op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
assert op.setup(amd.GAUSSIAN, 1.0, 1.0, 0.01) == 0
xd = torch.tensor(x, device="cuda")
yd = torch.zeros(n, dtype=torch.float64, device="cuda")
for _ in range(reps):
    op.matsymv(xd, 1.0, 0.0, yd)
torch.cuda.synchronize()
print("done", float(yd.norm()))
