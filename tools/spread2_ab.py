"""A/B of the two-vector matvec's spread (Nfft4GPAmdAdditiveMatSymvMulti, nrhs = 2 per pass): one handle per
setting of the layout / kernel knobs (read at handle creation), timed on the same vectors, each column checked
against the single-vector matvec.

    python tools/spread2_ab.py --n 10000000 --d 64 --settings "0:1:4064 1:1:4064 2:1:4064 1:4:4064 1:1:2032"

A setting is SPREAD2:GPW:BLOCK (NFFT4GP_AMD_SPREAD2 0 = two single-vector spreads, 1 / 2 = k_spread_multi on
512 / 1024 threads; NFFT4GP_AMD_SPREAD2_GPW; NFFT4GP_AMD_BLOCK).
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
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=32)
    ap.add_argument("--nv", type=int, default=10)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--settings", default="0:1:0 1:1:0 2:1:0")
    args = ap.parse_args()
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    L = amd.lib()
    L.Nfft4GPAmdSetStream(s.cuda_stream)
    n, d, nv = args.n, args.d, args.nv
    rng = np.random.default_rng(3)
    X = np.asfortranarray(rng.random((n, d)))
    V = torch.tensor(rng.random((nv, n)) - 0.5, device="cuda")
    for setting in args.settings.split():
        sp, gpw, blk = (int(v) for v in setting.split(":"))
        os.environ["NFFT4GP_AMD_SPREAD2"] = str(sp)
        os.environ["NFFT4GP_AMD_SPREAD2_GPW"] = str(gpw)
        if blk > 0:
            os.environ["NFFT4GP_AMD_BLOCK"] = str(blk)
        else:
            os.environ.pop("NFFT4GP_AMD_BLOCK", None)
        op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
        assert op.setup(amd.GAUSSIAN, f=1.0, l=0.1, mu=0.01) == 0
        Y1 = torch.zeros_like(V)
        Y2 = torch.zeros_like(V)

        def single():
            for v in range(nv):
                op.matsymv(V[v], 1.0, 0.0, Y1[v])

        def multi():
            assert L.Nfft4GPAmdAdditiveMatSymvMulti(op.h, n, nv, 1.0, V.data_ptr(), n, 0.0, Y2.data_ptr(), n) == 0

        out = {"setting": setting, "n": n, "d": d, "nv": nv, "block": op.layout_info()["block"]}
        for name, fn in (("single", single), ("multi", multi)):
            t_end = time.perf_counter() + 0.3
            while time.perf_counter() < t_end:
                fn()
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                fn()
            torch.cuda.synchronize()
            out[name + "_ms_per_vec"] = round((time.perf_counter() - t0) / args.reps / nv * 1e3, 4)
        out["max_rel_diff"] = float(((Y1 - Y2).norm(dim=1) / Y1.norm(dim=1)).max())
        out["speedup"] = round(out["single_ms_per_vec"] / out["multi_ms_per_vec"], 3)
        print(json.dumps(out), flush=True)
        op.free()
        del Y1, Y2
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
