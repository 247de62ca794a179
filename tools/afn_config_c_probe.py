"""AFN setup at BASELINE config C on the additive kernel (rank 512, kernel FSAI of the Schur complement,
lfil 20), for rocprofv3 --kernel-trace --stats."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd  # noqa: E402

n, d, k = 1000000, 32, 512
X = np.asfortranarray(np.random.default_rng(906).random((n, d)))
op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
op.setup(amd.GAUSSIAN, 1.0, 0.1, 0.01)
perm = np.random.default_rng(908).permutation(n).astype(np.int32)
t0 = time.perf_counter()
pre = amd.AfnPrecond.setup(X, k, 1.0, 0.1, 0.01, perm_opt="perm", perm=perm, schur_lfil=20, op=op)
torch.cuda.synchronize()
print(f"AFN setup n={n} d={d} k={k}: {time.perf_counter() - t0:.3f} s")
