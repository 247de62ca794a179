"""Restarted FGMRES(50): block CGS2 (ortho 1) against delayed CGS2 (ortho 2), and the intrinsic sensitivity of
CGS2 itself to a one-ulp perturbation of b -- separates an algorithmic difference from rounding amplification.
    python tools/diag_dcgs2.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    n, d = 30000, 8
    rng = np.random.default_rng(17)
    X = rng.random((n, d))
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    assert op.setup(amd.GAUSSIAN, f=1.0, l=1.0, mu=0.01) == 0
    bh = rng.random(n) - 0.5
    runs = {}
    for name, o, pert in [("cgs2", 1, 0), ("cgs2_ulp", 1, 1), ("dcgs2", 2, 0), ("dcgs2_ulp", 2, 1), ("mgs", 0, 0)]:
        bb = bh.copy()
        if pert:
            bb[::7] = np.nextafter(bb[::7], 2.0)
        b = torch.tensor(bb, device="cuda")
        amd.lib().Nfft4GPAmdSetFgmresOrtho(o)
        x = torch.zeros_like(b)
        _, rr, hist, it = amd.fgmres(op, b, x, kdim=50, maxits=400, tol=1e-8)
        runs[name] = (hist[:it + 1].copy(), x.cpu().numpy())
    amd.lib().Nfft4GPAmdSetFgmresOrtho(0)
    h0 = runs["cgs2"][0]
    for name, (h, x) in runs.items():
        r = np.abs(h - h0) / h0
        first = int(np.argmax(r > 1e-8)) if np.any(r > 1e-8) else -1
        print(f"{name:10s} first idx >1e-8 rel: {first:4d}  max rel hist diff {r.max():.3e}  "
              f"x rel diff {np.linalg.norm(x - runs['cgs2'][1]) / np.linalg.norm(runs['cgs2'][1]):.3e}  "
              f"hist[49:53] {h[49:53]}", flush=True)


if __name__ == "__main__":
    main()
