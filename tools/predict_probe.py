"""Predictive std wall time (Nfft4GPAdditiveNFFTGpPredict with std) against the batch size of its solves
(NFFT4GP_AMD_PREDICT_BATCH): one point per batch is the reference's loop (nfft_interface.c:1015-1057), one
FGMRES at a time.  Synthetic data; TEST2's call shape (tol 1e-8, maxits 50 for the mean, no preconditioner).

    python tools/predict_probe.py [--n 20000] [--npred 64] [--d 8] [--batches 1,16,32]
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
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--npred", type=int, default=64)
    ap.add_argument("--d", type=int, default=8)
    ap.add_argument("--batches", default="1,16,32")
    args = ap.parse_args()
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    torch.cuda.set_device(0)
    rng = np.random.default_rng(5)
    X = rng.random((args.n, args.d))
    Xp = rng.random((args.npred, args.d))
    y = np.sin(3 * X[:, 0]) + X[:, 1] ** 2 + 0.05 * rng.standard_normal(args.n)
    win = np.arange(args.d, dtype=np.int32)
    hyper = np.array([0.3, -0.5, -2.0])
    ref = None
    for bm in args.batches.split(","):
        os.environ["NFFT4GP_AMD_PREDICT_BATCH"] = bm
        amd.gp_predict(X, Xp[:2], win, args.d, 1, y, hyper, maxits=50, tol=1e-8, with_std=True)  # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mean, std = amd.gp_predict(X, Xp, win, args.d, 1, y, hyper, maxits=50, tol=1e-8, with_std=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if ref is None:
            ref = std
        print(json.dumps({"n": args.n, "npred": args.npred, "windows": args.d, "batch": int(bm), "predict_s": dt,
                          "ms_per_point": dt / args.npred * 1e3,
                          "std_maxrel_vs_first": float(np.max(np.abs(std - ref) / np.abs(ref)))}), flush=True)


if __name__ == "__main__":
    main()
