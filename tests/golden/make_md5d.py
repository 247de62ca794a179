"""Generate tests/golden/md5d.npz: a window of 5 features (n = 300, seeded points) and the reference's dense
operator on it (oracle/_ref: kernels.c:3046-3494, matops.c:3-29) -- matvec and the three gradient outputs --
for the N = 32 truncation check of the 64^5-grid path.  The oracle's host NFFT of a 64^5 grid (17 GB of complex
cells, ~1.7e11 products per matvec) is out of reach here, so the 5-feature NFFT values are pinned through the
slice property in tests/test_gpu_md.py instead.  TEST INFRASTRUCTURE.
    python tests/golden/make_md5d.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from oracle import RefDenseAdditive, ref_available  # noqa: E402


def main():
    assert ref_available(), "build oracle/_ref first (make -C oracle ref)"
    rng = np.random.default_rng(505)
    n, d = 300, 5
    X = rng.random((n, d))
    x = rng.random(n) - 0.5
    win = np.arange(d, dtype=np.int32)
    f, l, mu = 1.0, 1.0, 0.01
    R = RefDenseAdditive(X, win, 1, d)
    R.matrices(f, l, mu, grad=True)
    out = {"X": X, "x": x, "f": f, "l": l, "mu": mu, "y_dense": R.matsymv(x), "g_dense": R.gradmatsymv(x)}
    np.savez(os.path.join(HERE, "md5d.npz"), **out)
    print({k: np.asarray(v).shape for k, v in out.items()})


if __name__ == "__main__":
    main()
