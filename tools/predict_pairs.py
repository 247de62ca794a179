"""Predictive standard deviations with paired FGMRES solves (print_level -1) against one solve at a time
(print_level 0, which prints per cycle and so disables the pairing): values and time.

    python tools/predict_pairs.py [--n 4000] [--npred 16]
"""
import argparse
import contextlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@contextlib.contextmanager
def quiet_stdout():
    fd = os.dup(1)
    null = os.open(os.devnull, os.O_WRONLY)
    os.dup2(null, 1)
    try:
        yield
    finally:
        os.dup2(fd, 1)
        os.close(null)
        os.close(fd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4000)
    ap.add_argument("--d", type=int, default=8)
    ap.add_argument("--npred", type=int, default=16)
    args = ap.parse_args()
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    torch.cuda.set_device(0)
    rng = np.random.default_rng(5)
    X = rng.random((args.n, args.d))
    Xp = rng.random((args.npred, args.d))
    y = rng.random(args.n) - 0.5
    win = np.arange(args.d, dtype=np.int32)
    out = {"n": args.n, "d": args.d, "npred": args.npred}
    res = {}
    for name, pl in (("paired", -1), ("single", 0)):
        amd.gp_predict(X, Xp, win, args.d, 1, y, (1.0, 0.3, 0.05), maxits=50, tol=1e-8, with_std=True,
                       transform=3, print_level=-1)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with quiet_stdout():
            res[name] = amd.gp_predict(X, Xp, win, args.d, 1, y, (1.0, 0.3, 0.05), maxits=50, tol=1e-8,
                                       with_std=True, transform=3, print_level=pl)
        torch.cuda.synchronize()
        out[name + "_s"] = time.perf_counter() - t0
    m1, s1 = res["paired"]
    m2, s2 = res["single"]
    out["std_max_rel_diff"] = float(np.max(np.abs(s1 - s2) / np.abs(s2)))
    out["mean_max_abs_diff"] = float(np.max(np.abs(m1 - m2)))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
