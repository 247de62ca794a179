"""Multi-feature windows (nfft_md.hip): matvec time per configuration, hipEvent-timed over repeated
matvecs on the library stream.
    python tools/md_probe.py [n,nw,dw ...]
Configurations (default below, or the ones given): n points, nw windows of dw features (2-D / 3-D windows; TEST1's bike is 3 x 3-D)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CONFIGS = [(17379, 3, 3), (100000, 3, 3), (1000000, 4, 2), (1000000, 16, 2), (1000000, 3, 3), (1000000, 10, 3)]


def main():
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    amd.lib().Nfft4GPAmdSetStream(s.cuda_stream)
    configs = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or CONFIGS
    for n, nw, dw in configs:
        rng = np.random.default_rng(n + nw)
        X = np.asfortranarray(rng.random((n, nw * dw)))
        win = np.arange(nw * dw, dtype=np.int32)
        op = amd.NFFTAdditiveKernel(X, win, nw, dw)
        t0 = time.time()
        assert op.setup(amd.GAUSSIAN, 1.0, 1.0, 0.01) == 0
        setup = time.time() - t0
        x = torch.tensor(rng.random(n) - 0.5, device="cuda")
        y = torch.zeros(n, dtype=torch.float64, device="cuda")
        for _ in range(3):
            op.matsymv(x, 1.0, 0.0, y)
        torch.cuda.synchronize()
        reps = 20 if n * nw * dw ** 3 < 1e8 else 5
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            op.matsymv(x, 1.0, 0.0, y)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(json.dumps({"n": n, "nwindows": nw, "features_per_window": dw, "setup_s": round(setup, 3),
                          "ms_per_matvec": ms, "taps_per_point_window": 10 ** dw}), flush=True)
        del op


if __name__ == "__main__":
    main()
