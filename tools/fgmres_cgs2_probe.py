"""FGMRES with the block CGS2 (Nfft4GPAmdSetFgmresOrtho(1)) and delayed CGS2 (2) orthogonalisations at the bench's FGMRES
configuration (config C, l = 1, kdim = maxits = 1000, tol 1e-6): time, iterations, second passes.
    python tools/fgmres_cgs2_probe.py [reps]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    L = amd.lib()
    L.Nfft4GPAmdSetStream(s.cuda_stream)
    n, d = 1_000_000, 32
    rng = np.random.default_rng(906)
    X = rng.random((n, d))
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    assert op.setup(amd.GAUSSIAN, f=1.0, l=1.0, mu=0.01) == 0
    b = torch.tensor(np.random.default_rng(907).random(n) - 0.5, device="cuda")
    for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
        for ortho in (1, 2):
            L.Nfft4GPAmdSetFgmresOrtho(ortho)
            xs = torch.zeros_like(b)
            L.Nfft4GPAmdFgmresSecondPasses()
            torch.cuda.synchronize()
            t0 = time.time()
            _, rr, hist, it = amd.fgmres(op, b, xs, kdim=1000, maxits=1000, tol=1e-6)
            torch.cuda.synchronize()
            dt = time.time() - t0
            print(json.dumps({"ortho": ortho, "rep": rep, "iters": it, "rel_res": rr, "time_s": round(dt, 4),
                              "second_passes": int(L.Nfft4GPAmdFgmresSecondPasses()),
                              "hist_10": float(hist[10]), "hist_100": float(hist[100])}), flush=True)


if __name__ == "__main__":
    main()
