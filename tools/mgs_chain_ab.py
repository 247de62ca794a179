"""FGMRES with the reference's MGS at config C, l = 1 (the bench's fgmres leg: kdim = maxits = 1000, tol 1e-6):
the sweep of each step in one launch (k_mgs_chain, NFFT4GP_AMD_MGS_CHAIN=1, the default) against one k_gs_step
launch per projection (=0), alternated on one box; also the config-C loss (its FGMRES solve uses MGS).

    python tools/mgs_chain_ab.py [--reps 2]
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
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import torch
    import bench
    torch.cuda.set_device(0)
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    n, d = 1_000_000, 32
    X = np.random.default_rng(906).random((n, d))
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    assert op.setup(amd.GAUSSIAN, f=1.0, l=1.0, mu=0.01) == 0
    for rep in range(args.reps):
        for chain in ("1", "0"):
            os.environ["NFFT4GP_AMD_MGS_CHAIN"] = chain
            r = bench.run_fgmres(op, torch, n)
            lo = bench.run_loss(op, torch, n, d, X)
            print(json.dumps({"chain": int(chain), "rep": rep, "fgmres_time_s": r["fgmres_time_s"],
                              "fgmres_iters": r["fgmres_iters"], "fgmres_rel_res": r["fgmres_rel_res"],
                              "fgmres_ms_per_iter": r.get("fgmres_ms_per_iter"), "loss_time_s": lo["loss_time_s"],
                              "loss_value": lo["loss_value"]}), flush=True)


if __name__ == "__main__":
    main()
