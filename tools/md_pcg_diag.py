"""test_gpu_md.py::test_pcg_tiled_3d's PCG, repeated, with its iteration counts and residual history tails."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd  # noqa: E402

torch.cuda.set_device(0)
rng = np.random.default_rng(61)
n = 60000
X = rng.random((n, 6))
op = amd.NFFTAdditiveKernel(X, np.arange(6, dtype=np.int32), 2, 3)
assert op.setup(0, 1.0, 0.3, 0.01) == 0
b = rng.random(n) - 0.5
for rep in range(4):
    x = torch.zeros(n, dtype=torch.float64, device="cuda")
    x, rr, hist, it = amd.pcg(op, torch.tensor(b, device="cuda"), x, maxits=6000, tol=1e-8)
    h = np.asarray(hist)
    nz = np.nonzero(h)[0]
    print(f"rep {rep}: it {it} rr {rr:.3e} hist entries {len(nz)} last {h[nz[-1]] if len(nz) else None:.3e} "
          f"first {h[:3]}", flush=True)
