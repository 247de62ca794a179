"""FSAI setup kernels in isolation (for rocprofv3 --kernel-trace --stats): n points in d dims, lfil."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd import _lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 3
lfil = int(sys.argv[3]) if len(sys.argv) > 3 else 30
grad = int(sys.argv[4]) if len(sys.argv) > 4 else 1
L = _lib.lib()
X = np.asfortranarray(np.random.default_rng(1).random((n, d)))
P = _lib.kernel_params(1.0, 0.05, 0.01, n)
h = L.Nfft4GPAmdPrecondFsaiCreate()
L.Nfft4GPAmdPrecondFsaiSetLfil(h, lfil)
t0 = time.perf_counter()
assert L.Nfft4GPAmdPrecondFsaiSetupWithKernel(X.ctypes.data, n, n, d, None, P, grad, h) == 0
print(f"FSAI setup n={n} d={d} lfil={lfil} grad={grad}: {time.perf_counter() - t0:.3f} s")
if len(sys.argv) > 5:  # dump the pattern and values (A/B of kernel variants: they must agree bitwise)
    nnz = L.Nfft4GPAmdPrecondFsaiCsr(h, None, None, None, None)
    ia = np.zeros(n + 1, np.int32)
    ja = np.zeros(nnz, np.int32)
    aa = np.zeros(nnz)
    da = np.zeros(3 * nnz)
    assert L.Nfft4GPAmdPrecondFsaiCsr(h, ia.ctypes.data, ja.ctypes.data, aa.ctypes.data, da.ctypes.data) == nnz
    np.savez(sys.argv[5], ia=ia, ja=ja, aa=aa)
