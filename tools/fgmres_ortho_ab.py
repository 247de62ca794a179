"""The bench's FGMRES legs (config C, l = 1, kdim = maxits = 1000) for ortho 1 (block CGS2) and 2 (delayed CGS2),
with the block dots' reduction folded into their launch (default) and as its own launch (NFFT4GP_AMD_BD_FOLD=0),
alternated on one box.

    python tools/fgmres_ortho_ab.py [--reps 2]
"""
import argparse
import json
import os
import sys

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
        for fold in ("1", "0"):
            os.environ["NFFT4GP_AMD_BD_FOLD"] = fold
            row = {"fold": int(fold), "rep": rep}
            for ortho in (1, 2):
                r = bench.run_fgmres(op, torch, n, ortho=ortho)
                p = ["fgmres_", "fgmres_cgs2_", "fgmres_dcgs2_"][ortho]
                row[p + "time_s"] = r[p + "time_s"]
                row[p + "iters"] = r[p + "iters"]
                row[p + "rel_res"] = r[p + "rel_res"]
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
