"""Time the FSAI pattern's KNN variants (knn_pattern in fsai_setup.hip) on n points of d uniform features:
    python tools/knn_probe.py [--n 1000000] [--d 32] [--lfil 20] [--variants 1,0]
and check that they agree."""
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
    ap.add_argument("--lfil", type=int, default=20)
    ap.add_argument("--variants", default="1,0")
    args = ap.parse_args()
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    f = amd.lib().Nfft4GPAmdDebugKnn
    f.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    n, d, lfil = args.n, args.d, args.lfil
    X = np.asfortranarray(np.random.default_rng(906).random((n, d)))
    out, ref = {}, None
    for v in [int(x) for x in args.variants.split(",")]:
        ja = np.zeros((n - lfil) * lfil, np.int32)
        nf = C.c_int()
        t0 = time.time()
        assert f(X.ctypes.data, n, n, d, lfil, v, ja.ctypes.data, C.byref(nf)) == 0
        out[f"variant{v}_s"] = time.time() - t0
        out[f"variant{v}_fallback_rows"] = nf.value
        if ref is None:
            ref = ja
        else:
            out[f"variant{v}_same"] = bool(np.array_equal(ref, ja))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
