"""Writes the deterministic-mode matvec y of a config (C: n 1e6, 32 windows; E: n 1e7, 64 windows, --precision 32 / 64)
to an .npy, so two processes with different NFFT4GP_AMD_* knobs (read once per process) can be compared bit for bit.

    python tools/interp_check.py --out gpurun_out/y_a.npy [--n 1000000 --d 32 --precision 64]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=32)
    ap.add_argument("--precision", type=int, default=64)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    rng = np.random.default_rng(906)
    X = rng.random((a.n, a.d))
    x = rng.random(a.n) - 0.5
    op = amd.NFFTAdditiveKernel(X, np.arange(a.d, dtype=np.int32), a.d, 1)
    if a.precision == 32:
        op.set_precision(32)
    assert op.setup(amd.GAUSSIAN, f=1.0, l=1.0, mu=0.01) == 0
    op.set_deterministic(True)
    xd = torch.tensor(x, device="cuda")
    y = op.matsymv(xd, 0.7, 0.0)
    y2 = torch.tensor(np.cos(np.arange(a.n)), device="cuda")
    op.matsymv(xd, 1.3, -0.4, y2)  # beta != 0
    torch.cuda.synchronize()
    np.save(a.out, np.concatenate([y.cpu().numpy(), y2.cpu().numpy()]))
    print(a.out, float(np.linalg.norm(y.cpu().numpy())))


if __name__ == "__main__":
    main()
