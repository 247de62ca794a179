"""Two-vector matvec (Nfft4GPAmdAdditiveMatSymvMulti) against single matvecs: agreement and time.

    python tools/multi_probe.py [--n 1000000] [--d 32] [--nv 10]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=32)
    ap.add_argument("--nv", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    torch.cuda.set_device(0)
    L = amd.lib()
    L.Nfft4GPAmdSetStream(torch.cuda.current_stream().cuda_stream)
    n, d, nv = args.n, args.d, args.nv
    rng = np.random.default_rng(3)
    X = np.asfortranarray(rng.random((n, d)))
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    assert op.setup(amd.GAUSSIAN, f=1.0, l=0.1, mu=0.01) == 0
    V = torch.tensor(rng.random((nv, n)) - 0.5, device="cuda")
    Y1 = torch.zeros_like(V)
    Y2 = torch.zeros_like(V)

    def single():
        for v in range(nv):
            op.matsymv(V[v], 1.0, 0.0, Y1[v])

    def multi():
        assert L.Nfft4GPAmdAdditiveMatSymvMulti(op.h, n, nv, 1.0, V.data_ptr(), n, 0.0, Y2.data_ptr(), n) == 0

    out = {"n": n, "d": d, "nv": nv}
    for name, fn in (("single", single), ("multi", multi)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fn()
        torch.cuda.synchronize()
        out[name + "_ms_per_vec"] = (time.perf_counter() - t0) / args.reps / nv * 1e3
    out["max_rel_diff"] = float(((Y1 - Y2).norm(dim=1) / Y1.norm(dim=1)).max())
    out["speedup"] = out["single_ms_per_vec"] / out["multi_ms_per_vec"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
