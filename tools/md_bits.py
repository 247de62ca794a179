"""One multi-feature matvec and gradient matvec per configuration written to an .npy (compare two settings' files
bit for bit: python tools/md_bits.py out.npy [n,nw,dw ...], then numpy.array_equal on the two files)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    out = []
    for a in sys.argv[2:] or ["17379,3,3", "20000,3,2", "2000,1,4", "1000,1,5"]:
        n, nw, dw = (int(v) for v in a.split(","))
        rng = np.random.default_rng(n + nw)
        X = np.asfortranarray(rng.random((n, nw * dw)))
        op = amd.NFFTAdditiveKernel(X, np.arange(nw * dw, dtype=np.int32), nw, dw)
        assert op.setup(amd.GAUSSIAN, 1.0, 0.5, 0.01) == 0
        x = torch.tensor(rng.random(n) - 0.5, device="cuda")
        out.append(op.matsymv(x).cpu().numpy())
        out.append(op.gradmatsymv(x).cpu().numpy())
        op.free()
    np.save(sys.argv[1], np.concatenate(out))


if __name__ == "__main__":
    main()
