"""Config-C loss + gradient (bench.py's run_loss leg: Nfft4GPGpLoss, 10 probes x 50 Lanczos steps, FGMRES 50) timed
several times on one operator, to split its wall time from its kernel time under rocprofv3.

    python tools/loss_probe.py [--reps 3] [--ortho 0]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ortho", type=int, default=0)
    args = ap.parse_args()
    import torch
    import bench
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    torch.cuda.set_device(0)
    rng = np.random.default_rng(906)
    n, d = 1_000_000, 32
    X = rng.random((n, d))
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    assert op.setup(amd.GAUSSIAN, f=1.0, l=1.0, mu=0.01) == 0
    for rep in range(args.reps):
        t0 = time.perf_counter()
        r = bench.run_loss(op, torch, n, d, X, ortho=args.ortho)
        print(json.dumps({"rep": rep, "wall_s": time.perf_counter() - t0, **r}), flush=True)


if __name__ == "__main__":
    main()
