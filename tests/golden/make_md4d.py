"""Generate tests/golden/md4d.npz: a window of 4 features (n = 300, seeded points), the oracle's CPU
restatement of the reference's NFFT path (oracle/nfft4gp_oracle.c; 64^4 grids, ~80 s per matvec on the
host, too slow for a test) and, when oracle/_ref is built, the reference's dense operator
(kernels.c:3046-3494) for the truncation check.  TEST INFRASTRUCTURE.
    python tests/golden/make_md4d.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from oracle import OracleAdditiveNFFT, RefDenseAdditive, ref_available  # noqa: E402


def main():
    rng = np.random.default_rng(404)
    n, d = 300, 4
    X = rng.random((n, d))
    x = rng.random(n) - 0.5
    win = np.arange(d, dtype=np.int32)
    f, l, mu = 1.0, 1.0, 0.01
    o = OracleAdditiveNFFT(X, win, 1, d)
    o.setup(0, f, l, mu)
    y = o.matsymv(x)
    g = o.gradmatsymv(x)
    out = {"X": X, "x": x, "f": f, "l": l, "mu": mu, "y_nfft": y, "g_nfft": g}
    if ref_available():
        R = RefDenseAdditive(X, win, 1, d)
        R.matrices(f, l, mu, grad=False)
        out["y_dense"] = R.matsymv(x)
    np.savez(os.path.join(HERE, "md4d.npz"), **out)
    print({k: np.asarray(v).shape for k, v in out.items()})


if __name__ == "__main__":
    main()
