"""One GP loss + gradient (Nfft4GPGpLoss) at config C (n = 1e6, 32 windows) as bench.py's loss leg runs it,
for a kernel-trace profile:  rocprofv3 --kernel-trace --stats -- python3 tools/loss_probe.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    n, d = int(os.environ.get("LOSS_N", "1000000")), 32
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    amd.lib().Nfft4GPAmdSetStream(s.cuda_stream)
    X = np.asfortranarray(np.random.default_rng(906).random((n, d)))
    win = np.arange(d, dtype=np.int32)
    op = amd.NFFTAdditiveKernel(X, win, d, 1)
    assert op.setup(amd.GAUSSIAN, f=1.0, l=1.0, mu=0.01) == 0
    rng = np.random.default_rng(909)
    y = rng.random(n) - 0.5
    R = np.where(rng.random((n, 10)) < 0.5, -1.0, 1.0)
    Rl = torch.tensor(np.asfortranarray(R).T.copy(), device="cuda")
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.time()
        lval = float(os.environ.get("LOSS_L", "0.1"))
        loss, grad = amd.gp_loss(X, win, d, 1, y, (1.0, lval, 0.01), maxits=50, nvecs=10, rademacher=Rl, tol=1e-6,
                                 transform=3, op=op)
        torch.cuda.synchronize()
        print(f"loss {loss:.12e} grad {list(grad)} time {time.time() - t0:.3f} s", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
