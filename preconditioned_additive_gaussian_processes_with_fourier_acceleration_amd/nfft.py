"""Host-side mirror of the reference NFFT kernel interface (SRC/external/nfft_interface.c).

The reference is C; its "plugin" for this path is the pair

    func_kernel    setup  Nfft4GPNFFTAdditiveKernelGaussianKernel / ...Matern12Kernel   (:676-794)
    func_symmatvec apply  Nfft4GPAdditiveNFFTMatSymv / Nfft4GPAdditiveNFFTGradMatSymv   (:796-840)

on a handle made by Nfft4GPNFFTAdditiveKernelParamCreate (:622-674) whose _params[0] (f),
_params[1] (l) and _noise_level (mu) callers write directly.  ``NFFTAdditiveKernel`` wraps exactly
those C-ABI calls of ``libnfft4gp_amd.so`` (same names, same argument meaning, same -1 error
returns) so tests read like the reference's drivers (TESTS/TEST1/foo.cpp:203-254).

Vectors may be numpy arrays (host pointers: staged over PCIe by the library, synchronous) or torch
tensors on the GPU (device pointers: enqueued on the library stream, no host sync).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib

GAUSSIAN = 0
MATERN12 = 1


def _ptr(a):
    """(pointer, is_device) for a numpy array or a torch tensor."""
    if isinstance(a, np.ndarray):
        if not a.flags.c_contiguous or a.dtype != np.float64:
            raise ValueError("numpy vectors must be C-contiguous float64")
        return a.ctypes.data, False
    # torch tensor
    if not a.is_contiguous() or str(a.dtype) != "torch.float64":
        raise ValueError("torch vectors must be contiguous float64")
    return a.data_ptr(), a.is_cuda


def _numel(a) -> int:
    return int(a.size) if isinstance(a, np.ndarray) else int(a.numel())


def _check_len(name, a, need, exact=True):
    """The C entry points take raw pointers plus n: a short buffer would be read or written past its end
    (a host heap overflow through the staging copy, or an out-of-bounds device write)."""
    got = _numel(a)
    if (got != need) if exact else (got < need):
        raise ValueError(f"{name} has {got} entries; this call needs {'exactly' if exact else 'at least'} {need}")


def _empty_like(x, n):
    if isinstance(x, np.ndarray):
        return np.zeros(n)
    import torch
    return torch.zeros(n, dtype=torch.float64, device=x.device)


class NFFTAdditiveKernel:
    """Additive NFFT kernel handle (nfft4gp_kernel with the device plan in _external)."""

    def __init__(self, data, windows, nwindows: int, dwindows: int, shard: tuple[int, int] | None = None):
        data = np.asfortranarray(np.asarray(data, dtype=np.float64))
        if data.ndim != 2:
            raise ValueError("data must be n x d")
        self.n_global, self.d = data.shape
        self._data = data  # the library copies the window columns at creation
        self._win = np.ascontiguousarray(np.asarray(windows, dtype=np.int32).ravel())
        if self._win.size != nwindows * dwindows:
            raise ValueError("windows must hold nwindows*dwindows entries")
        self.nwindows, self.dwindows = nwindows, dwindows
        L = _lib.lib()
        if shard is None:
            self.row_begin, self.row_end = 0, self.n_global
            self.h = L.Nfft4GPNFFTAdditiveKernelParamCreate(self._data.ctypes.data, self.n_global, self.n_global,
                                                            self.d, self._win.ctypes.data, nwindows, dwindows)
        else:
            self.row_begin, self.row_end = shard
            self.h = L.Nfft4GPAmdAdditiveShardCreate(self._data.ctypes.data, self.n_global, self.n_global, self.d,
                                                     self._win.ctypes.data, nwindows, dwindows, self.row_begin,
                                                     self.row_end)
        if not self.h:
            raise RuntimeError("Nfft4GPNFFTAdditiveKernelParamCreate failed")
        self.n = self.row_end - self.row_begin
        self._st = _lib.NfftKernelStruct.from_address(self.h)
        self._kernel = None

    # hyperparameters live in the handle, exactly where the reference's callers write them
    @property
    def f(self):
        return self._st._params[0]

    @f.setter
    def f(self, v):
        self._st._params[0] = float(v)

    @property
    def l(self):
        return self._st._params[1]

    @l.setter
    def l(self, v):
        self._st._params[1] = float(v)

    @property
    def mu(self):
        return self._st._noise_level

    @mu.setter
    def mu(self, v):
        self._st._noise_level = float(v)

    @property
    def iparams(self):
        return tuple(self._st._iparams[:3])

    def setup(self, kernel: int = GAUSSIAN, f=None, l=None, mu=None) -> int:
        """The func_kernel call (nfft_interface.c:676-794); returns the C status (0 or -1)."""
        if f is not None:
            self.f = f
        if l is not None:
            self.l = l
        if mu is not None:
            self.mu = mu
        L = _lib.lib()
        fn = L.Nfft4GPNFFTAdditiveKernelGaussianKernel if kernel == GAUSSIAN else \
            L.Nfft4GPNFFTAdditiveKernelMatern12Kernel
        K = C.c_void_p()
        dK = C.c_void_p()
        rc = fn(self.h, self._data.ctypes.data, self.n_global, self.n_global, self.d, None, 0, None, 0,
                C.byref(K), C.byref(dK))
        if rc == 0:
            self._kernel = kernel
        return rc

    def _apply(self, fn, x, alpha, beta, y, mult):
        if self.row_begin != 0 or self.row_end != self.n_global:
            raise ValueError("a row-shard handle has no whole matvec: use shard_spread / shard_finish")
        _check_len("x", x, self.n)
        if y is None:
            y = _empty_like(x, mult * self.n)
        _check_len("y", y, mult * self.n)
        xp, xd = _ptr(x)
        yp, yd = _ptr(y)
        rc = fn(self.h, self.n, float(alpha), xp, float(beta), yp)
        if rc != 0:
            raise RuntimeError(f"matvec failed with status {rc}")
        return y

    def matsymv(self, x, alpha=1.0, beta=0.0, y=None):
        """y <- beta*y + alpha*f^2*((1/nw) sum_c K_c + mu I) x   (Nfft4GPAdditiveNFFTMatSymv)."""
        return self._apply(_lib.lib().Nfft4GPAdditiveNFFTMatSymv, x, alpha, beta, y, 1)

    def gradmatsymv(self, x, alpha=1.0, beta=0.0, y=None):
        """[dK/df x; dK/dl x; dK/dmu x] (3n), Nfft4GPAdditiveNFFTGradMatSymv."""
        return self._apply(_lib.lib().Nfft4GPAdditiveNFFTGradMatSymv, x, alpha, beta, y, 3)

    # ---- split phase for row-sharded multi-GPU use -------------------------------------------
    def shard_spread(self, x_local, grid):
        _check_len("x_local", x_local, self.n)
        size = self.shard_grid_size()
        if size < 0:
            raise RuntimeError("run the kernel setup before shard_spread")
        _check_len("grid", grid, size, exact=False)
        xp, _ = _ptr(x_local)
        gp, _ = _ptr(grid)
        if _lib.lib().Nfft4GPAmdShardSpread(self.h, xp, gp) != 0:
            raise RuntimeError("shard spread failed")
        return grid

    def shard_grid_size(self) -> int:
        """Doubles in the grid shard_spread writes (nw*64, or nw*64^dmax with multi-feature windows);
        -1 before the kernel setup."""
        return int(_lib.lib().Nfft4GPAmdShardGridSize(self.h))

    def shard_finish(self, grid, x_local, alpha=1.0, beta=0.0, y_local=None, grad=False):
        _check_len("x_local", x_local, self.n)
        if y_local is None:
            y_local = _empty_like(x_local, (3 if grad else 1) * self.n)
        _check_len("y_local", y_local, (3 if grad else 1) * self.n)
        size = self.shard_grid_size()
        if size < 0:
            raise RuntimeError("run the kernel setup before shard_finish")
        _check_len("grid", grid, size, exact=False)
        gp, _ = _ptr(grid)
        xp, _ = _ptr(x_local)
        yp, _ = _ptr(y_local)
        if _lib.lib().Nfft4GPAmdShardFinish(self.h, gp, int(grad), float(alpha), xp, float(beta), yp) != 0:
            raise RuntimeError("shard finish failed")
        return y_local

    # ---- introspection ---------------------------------------------------------------------------
    def layout_info(self) -> dict:
        out = (C.c_longlong * 10)()
        _lib.lib().Nfft4GPAmdAdditiveLayoutInfo(self.h, out, 10)
        keys = ["n", "nwindows", "block", "nblocks", "ntiles", "slots", "R", "comps_per_group", "ngroups",
                "layout_bytes"]
        return dict(zip(keys, [int(v) for v in out]))

    def set_deterministic(self, on: bool = True):
        """Nfft4GPAmdSetDeterministic: bitwise reproducible 1-D matvecs, or plain fp64 LDS atomics (the default)."""
        if _lib.lib().Nfft4GPAmdSetDeterministic(self.h, int(bool(on))) != 0:
            raise RuntimeError("Nfft4GPAmdSetDeterministic failed")

    def set_precision(self, bits: int):
        """Nfft4GPAmdSetPrecision: 32 (one 32-bit record per (point, window), BASELINE configs[4]'s fp32 matvec) or
        64 (the default 5-byte records); after the first setup the layout is rebuilt."""
        if _lib.lib().Nfft4GPAmdSetPrecision(self.h, int(bits)) != 0:
            raise RuntimeError("Nfft4GPAmdSetPrecision failed")

    def timing(self, enable: bool):
        _lib.lib().Nfft4GPAmdTimingEnable(self.h, int(enable))

    def timing_query(self):
        ms = (C.c_double * 3)()
        cnt = (C.c_longlong * 3)()
        _lib.lib().Nfft4GPAmdTimingQuery(self.h, ms, cnt)
        names = ["spread", "grid", "interp"]
        return {nm: (ms[i], int(cnt[i])) for i, nm in enumerate(names)}

    KERNELS = ("spread", "grid", "interp")

    def kernel_bench(self, kernel: str, x, y, reps: int = 50, grad: bool = False) -> float:
        """Mean ms of one launch of `kernel` ("spread" | "grid" | "interp"), timed with a single event
        pair around `reps` back-to-back launches on the library stream.  x, y: device vectors
        (y of length 3n when grad).  Call after a matvec (or gradmatsymv when grad) of the same setup."""
        px, dx = _ptr(x)
        py, dy = _ptr(y)
        if not (dx and dy):
            raise ValueError("kernel_bench needs device vectors")
        ms = C.c_double()
        rc = _lib.lib().Nfft4GPAmdKernelBench(self.h, self.KERNELS.index(kernel), int(grad), reps, px, py,
                                               C.byref(ms))
        if rc != 0:
            raise RuntimeError("Nfft4GPAmdKernelBench failed")
        return ms.value

    @property
    def matvec_fnptr(self) -> int:
        return _lib.fnptr("Nfft4GPAdditiveNFFTMatSymv")

    @property
    def gradmatvec_fnptr(self) -> int:
        return _lib.fnptr("Nfft4GPAdditiveNFFTGradMatSymv")

    def free(self):
        if getattr(self, "h", None):
            _lib.lib().Nfft4GPAdditiveNFFTKernelFree(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class NFFTKernel:
    """Single-component NFFT kernel (nfft_interface.c:3-620): ParamCreate(max_n, dim), setup, MatSymv."""

    def __init__(self, max_n: int, dim: int):
        L = _lib.lib()
        self.h = L.Nfft4GPNFFTKernelParamCreate(max_n, dim)
        self._st = _lib.NfftKernelStruct.from_address(self.h)
        self.dim = dim
        self.adj = None
        self.n = None

    def setup(self, data, kernel=GAUSSIAN, f=1.0, l=1.0, mu=0.0) -> int:
        data = np.asfortranarray(np.asarray(data, dtype=np.float64))
        n = data.shape[0]
        self._data = data
        self._st._params[0] = f
        self._st._params[1] = l
        self._st._noise_level = mu
        L = _lib.lib()
        fn = L.Nfft4GPNFFTKernelGaussianKernel if kernel == GAUSSIAN else L.Nfft4GPNFFTKernelMatern12Kernel
        K = C.c_void_p()
        dK = C.c_void_p()
        rc = fn(self.h, data.ctypes.data, n, n, self.dim, None, 0, None, 0, C.byref(K), C.byref(dK))
        if rc == 0:
            self.adj = K.value
            self.n = n
        return rc

    def matsymv(self, x, alpha=1.0, beta=0.0, y=None):
        _check_len("x", x, self.n)
        if y is None:
            y = _empty_like(x, self.n)
        _check_len("y", y, self.n)
        rc = _lib.lib().Nfft4GPNFFTMatSymv(self.adj, self.n, float(alpha), _ptr(x)[0], float(beta), _ptr(y)[0])
        if rc:
            raise RuntimeError("Nfft4GPNFFTMatSymv failed")
        return y

    def gradmatsymv(self, x, alpha=1.0, beta=0.0, y=None):
        _check_len("x", x, self.n)
        if y is None:
            y = _empty_like(x, 3 * self.n)
        _check_len("y", y, 3 * self.n)
        rc = _lib.lib().Nfft4GPNFFTGradMatSymv(self.adj, self.n, float(alpha), _ptr(x)[0], float(beta),
                                               _ptr(y)[0])
        if rc:
            raise RuntimeError("Nfft4GPNFFTGradMatSymv failed")
        return y

    def free(self):
        if getattr(self, "h", None):
            _lib.lib().Nfft4GPNFFTKernelParamFree(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
