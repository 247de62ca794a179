"""The Nystrom setup's three MFMA products at config C (n = 1e6, k = 512; nystrom.hip k_gemm_f64): per-product
hipEvent times over several setups, the same way bench.py's nys_setup_mfma reports them, plus a checksum of U
(the products' accumulation order does not depend on the GEMM variant, so U is bitwise the same).
    python tools/gemm_probe.py   (profiles/r04_gemm_ahead_ab.txt compared a removed two-step-lookahead variant)"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    n, d, k = 1_000_000, 32, 512
    X = np.asfortranarray(np.random.default_rng(906).random((n, d)))
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    assert op.setup(amd.GAUSSIAN, f=1.0, l=0.1, mu=0.01) == 0
    perm = np.random.default_rng(908).permutation(n).astype(np.int32)
    rows = []
    for rep in range(4):
        pre = amd.NystromPrecond.from_additive(op, perm, k, k11="landmarks")
        torch.cuda.synchronize()
        ms = pre.setup_times()
        if rep > 0:
            rows.append({key: ms[key] for key in ("gemm1", "gram", "gemm2")})
        pre.free()
    med = {key: float(np.median([r[key] for r in rows])) for key in rows[0]}
    flops = 2.0 * n * k * k
    print(json.dumps({"ms": med,
                      "tflops": {key: flops / (v * 1e-3) / 1e12 for key, v in med.items()},
                      "frac": {key: flops / (v * 1e-3) / 1e12 / 78.6 for key, v in med.items()}}), flush=True)


if __name__ == "__main__":
    main()
