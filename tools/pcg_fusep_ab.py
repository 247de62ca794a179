"""PCG to 1e-6 at config C, l = 0.1 (the bench's PCG leg) with the direction update fused into k_pcg_xr
(NFFT4GP_AMD_PCG_FUSEP=1, the default) and as its own launch (=0), alternated on one box.

    python tools/pcg_fusep_ab.py [--reps 3]
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
    args = ap.parse_args()
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    torch.cuda.set_device(0)
    rng = np.random.default_rng(906)
    n, d = 1_000_000, 32
    X = rng.random((n, d))
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    assert op.setup(amd.GAUSSIAN, f=1.0, l=0.1, mu=0.01) == 0
    b = torch.tensor(np.random.default_rng(907).random(n) - 0.5, device="cuda")
    for rep in range(args.reps):
        for f in ("1", "0"):
            os.environ["NFFT4GP_AMD_PCG_FUSEP"] = f
            x = torch.zeros(n, dtype=torch.float64, device="cuda")
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _, relres, _, it = amd.pcg(op, b, x, maxits=3000, tol=1e-6)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"fusep": int(f), "rep": rep, "pcg_s": dt, "iters": it, "ms_per_iter": dt / it * 1e3,
                              "relres": relres}), flush=True)


if __name__ == "__main__":
    main()
