"""GP loss and prediction on the NFFT additive operator, over the C ABI.

``gp_loss``     Nfft4GPGpLoss (SRC/optimizer/gp_loss.c:96-307) with Nfft4GPNFFTAdditiveKernelGaussianKernel /
                Nfft4GPAdditiveNFFTMatSymv / Nfft4GPAdditiveNFFTGradMatSymv as kernel, matvec and grad matvec,
                no preconditioner (TEST1-style call of the north-star operator inside the loss); or, over
                one process per GPU, a dist.DistributedAdditiveKernel with Nfft4GPAmdDistGaussianKernel /
                Nfft4GPAmdDistMatSymv / Nfft4GPAmdDistGradMatSymv (BASELINE configs[4]).
``gp_predict``  Nfft4GPAdditiveNFFTGpPredict (SRC/external/nfft_interface.c:873-1068): posterior mean and,
                optionally, standard deviation at new points (a second handle over [X; Xp], as TEST4 does).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .nfft import NFFTAdditiveKernel

_vp = C.c_void_p
_GPLOSS_ARGS = [_vp, _vp, _vp, C.c_int, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                _vp, _vp, _vp, _vp, C.c_int, C.c_double, C.c_int, C.c_int, C.c_int, _vp, C.c_int, _vp, C.c_int, _vp,
                _lib.dp, _lib.dp]
_PREDICT_ARGS = [_vp, _vp, _vp, C.c_int, C.c_int, C.c_int, _vp, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                 _vp, _vp, _vp, _vp, _vp, C.c_int, C.c_double, C.c_int, C.c_int, C.c_int, _vp, C.POINTER(_lib.dp),
                 C.POINTER(_lib.dp)]


def gp_loss(X, windows, nwindows, dwindows, y, hyper, maxits=50, nvecs=10, rademacher=None, tol=1e-6,
            transform=0, mask=None, print_level=-1, op=None):
    """(loss, grad) of Nfft4GPGpLoss for the additive NFFT Gaussian kernel; ``hyper`` = (f, l, mu) before
    the transform (0 softplus, 1 sigmoid, 2 exp, 3 identity).  ``op``: an existing NFFTAdditiveKernel over
    the same X to reuse, as the reference's optimizer loop reuses its kernel handle across loss calls
    (its points, centring and scale stay those of its first setup, nfft_interface.c:150); or a
    dist.DistributedAdditiveKernel (every rank calls gp_loss collectively): with partition "rows", ``y``
    and ``rademacher`` hold this rank's rows [op.row_begin, op.row_end) only; with "components" they are
    whole.  Every rank returns the same loss and gradient."""
    from .dist import DistributedAdditiveKernel
    # the points only build a new handle: a given op holds its own (the kernel setup does not read `data`,
    # nfft_api.cpp), so no column-major copy of X is made then (256 MB at config C, ~0.1 s of host time)
    X = np.asarray(X, dtype=np.float64)
    if op is None:
        X = np.asfortranarray(X)
    n, d = X.shape
    setup_fn, mv, dmv = ("Nfft4GPNFFTAdditiveKernelGaussianKernel", "Nfft4GPAdditiveNFFTMatSymv",
                         "Nfft4GPAdditiveNFFTGradMatSymv")
    if op is None:
        op = NFFTAdditiveKernel(X, windows, nwindows, dwindows)
    elif isinstance(op, DistributedAdditiveKernel):
        if op.n_global != n:
            raise ValueError("op was created over a different number of points")
        n = op.n  # this rank's rows (the whole n for components)
        setup_fn, mv, dmv = "Nfft4GPAmdDistGaussianKernel", "Nfft4GPAmdDistMatSymv", "Nfft4GPAmdDistGradMatSymv"
    elif op.n != n:
        raise ValueError("op was created over a different number of points")
    if len(y) != n:
        raise ValueError(f"{len(y)} labels for {n} rows")
    L = _lib.lib()
    fn = L.Nfft4GPGpLoss
    fn.argtypes = _GPLOSS_ARGS
    fn.restype = C.c_int
    x = np.ascontiguousarray(np.asarray(hyper, dtype=np.float64))
    lab = np.ascontiguousarray(np.asarray(y, dtype=np.float64))
    if rademacher is None:
        R, r_ptr = None, None
    elif hasattr(rademacher, "data_ptr"):  # a torch tensor (n * nvecs, column-major probes); device OK
        R, r_ptr = rademacher, rademacher.data_ptr()
    else:
        R = np.asfortranarray(np.asarray(rademacher, dtype=np.float64))
        r_ptr = R.ctypes.data
    m = None if mask is None else np.ascontiguousarray(np.asarray(mask, dtype=np.int32))
    loss = np.zeros(1)
    grad = np.zeros(3)
    rc = fn(x.ctypes.data, X.ctypes.data, lab.ctypes.data, n, n, d,
            _lib.fnptr(setup_fn), op.h, None, _lib.fnptr(mv), _lib.fnptr(dmv),
            None, None, None, None, None, None, None, None, None, None, 0, float(tol), int(maxits), int(maxits),
            int(nvecs), r_ptr, int(transform),
            m.ctypes.data if m is not None else None, int(print_level), None, loss.ctypes.data_as(_lib.dp),
            grad.ctypes.data_as(_lib.dp))
    if rc:
        raise RuntimeError("Nfft4GPGpLoss failed")
    return float(loss[0]), grad


def gp_predict(X, Xp, windows, nwindows, dwindows, y, hyper, maxits=100, tol=1e-8, with_std=False,
               transform=0, print_level=-1):
    """(mean, std or None) of Nfft4GPAdditiveNFFTGpPredict at the rows of Xp."""
    X = np.asfortranarray(np.asarray(X, dtype=np.float64))
    Xp = np.asfortranarray(np.asarray(Xp, dtype=np.float64))
    n, d = X.shape
    npred = Xp.shape[0]
    Xa = np.asfortranarray(np.vstack([X, Xp]))
    op = NFFTAdditiveKernel(X, windows, nwindows, dwindows)
    opa = NFFTAdditiveKernel(Xa, windows, nwindows, dwindows)
    L = _lib.lib()
    fn = L.Nfft4GPAdditiveNFFTGpPredict
    fn.argtypes = _PREDICT_ARGS
    fn.restype = C.c_int
    x = np.ascontiguousarray(np.asarray(hyper, dtype=np.float64))
    lab = np.ascontiguousarray(np.asarray(y, dtype=np.float64))
    mean = np.zeros(npred)
    std = np.zeros(npred)
    mp = C.cast(mean.ctypes.data, _lib.dp)
    sp = C.cast(std.ctypes.data, _lib.dp)
    rc = fn(x.ctypes.data, X.ctypes.data, lab.ctypes.data, n, n, d, Xp.ctypes.data, npred, npred, Xa.ctypes.data,
            _lib.fnptr("Nfft4GPNFFTAdditiveKernelGaussianKernel"), op.h, opa.h, None, op.matvec_fnptr, None, None,
            None, None, None, None, 0, float(tol), int(maxits), int(transform), int(print_level), None,
            C.byref(mp), C.byref(sp) if with_std else None)
    if rc:
        raise RuntimeError("Nfft4GPAdditiveNFFTGpPredict failed")
    return mean, (std if with_std else None)
