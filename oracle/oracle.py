"""TEST INFRASTRUCTURE ONLY -- ctypes front-ends for the two CPU checkers.

* ``OracleAdditiveNFFT``: the C restatement of the reference's NFFT additive operator
  (``oracle/nfft4gp_oracle.c``; reference ``SRC/external/nfft_interface.c`` + NFFT3 fastsum).
* ``RefDense``: the reference's own dense path compiled from its sources into
  ``oracle/_ref/libnfft4gp_ref.so`` (``SRC/linearalg/kernels.c``, ``matops.c``, ``solvers/pcg.c``,
  ``preconds/nys.c`` ...).  Built here by ``make -C oracle ref``; it travels to the GPU box as a
  built file, the reference sources never do.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this
module.  The product package never does.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "libnfft4gp_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "libnfft4gp_ref.so")

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)


def _d(a):
    return a.ctypes.data_as(_dp)


def _i(a):
    return a.ctypes.data_as(_ip)


_olib = None


def oracle_lib(path: str | None = None):
    global _olib
    if _olib is None or path is not None:
        lib = C.CDLL(path or ORACLE_SO)
        lib.orc_additive_create.restype = C.c_void_p
        lib.orc_additive_create.argtypes = [_dp, C.c_int, C.c_int, C.c_int, _ip, C.c_int, C.c_int]
        lib.orc_additive_setup.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_double, C.c_double]
        lib.orc_additive_matsymv.argtypes = [C.c_void_p, C.c_int, C.c_double, _dp, C.c_double, _dp, C.c_int]
        lib.orc_additive_gradmatsymv.argtypes = [C.c_void_p, C.c_int, C.c_double, _dp, C.c_double, _dp, C.c_int]
        lib.orc_additive_comp_info.argtypes = [C.c_void_p, C.c_int, _ip, _dp, _dp, _dp, _dp]
        lib.orc_additive_comp_points.argtypes = [C.c_void_p, C.c_int, _dp]
        lib.orc_additive_free.argtypes = [C.c_void_p]
        lib.orc_window_phi.restype = C.c_double
        lib.orc_window_phi.argtypes = [C.c_double]
        lib.orc_window_phi_hut.restype = C.c_double
        lib.orc_window_phi_hut.argtypes = [C.c_int]
        lib.orc_num_threads.restype = C.c_int
        if path is not None:
            return lib
        _olib = lib
    return _olib


class OracleAdditiveNFFT:
    """Mirror of Nfft4GPNFFTAdditiveKernelParamCreate / ...GaussianKernel / AdditiveNFFTMatSymv."""

    def __init__(self, data: np.ndarray, windows, nwindows: int, dwindows: int, lib=None):
        # data: n x d, column-major (feature-major) like the reference (ldim = n)
        self.lib = lib or oracle_lib()
        data = np.asfortranarray(data, dtype=np.float64)
        self.n, self.d = data.shape
        self._data = data
        self._win = np.ascontiguousarray(np.asarray(windows, dtype=np.int32).ravel())
        self.nw, self.dw = nwindows, dwindows
        self.h = self.lib.orc_additive_create(_d(self._data), self.n, self.n, self.d, _i(self._win),
                                              nwindows, dwindows)

    def setup(self, kernel: int, f: float, l: float, mu: float):
        self.lib.orc_additive_setup(self.h, kernel, f, l, mu)

    def matsymv(self, x, alpha=1.0, beta=0.0, y=None, exact=False):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(self.n) if y is None else np.ascontiguousarray(y, dtype=np.float64).copy()
        self.lib.orc_additive_matsymv(self.h, self.n, alpha, _d(x), beta, _d(y), int(exact))
        return y

    def gradmatsymv(self, x, alpha=1.0, beta=0.0, y=None, exact=False):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(3 * self.n) if y is None else np.ascontiguousarray(y, dtype=np.float64).copy()
        self.lib.orc_additive_gradmatsymv(self.h, self.n, alpha, _d(x), beta, _d(y), int(exact))
        return y

    def comp_info(self, c: int):
        d = np.zeros(1, np.int32)
        s = np.zeros(1)
        sg = np.zeros(1)
        self.lib.orc_additive_comp_info(self.h, c, _i(d), _d(s), _d(sg), None, None)
        nm = 32 ** int(d[0])
        bh = np.zeros(nm)
        bhd = np.zeros(nm)
        self.lib.orc_additive_comp_info(self.h, c, _i(d), _d(s), _d(sg), _d(bh), _d(bhd))
        return dict(d=int(d[0]), scale=float(s[0]), sigma0=float(sg[0]), bhat=bh, bhat_d=bhd)

    def comp_points(self, c: int):
        info = self.comp_info(c)
        out = np.zeros(self.n * info["d"])
        self.lib.orc_additive_comp_points(self.h, c, _d(out))
        return out.reshape(self.n, info["d"])

    def __del__(self):
        try:
            self.lib.orc_additive_free(self.h)
        except Exception:
            pass


# ----------------------------------------------------------------------------------------------
# The reference's own dense path (oracle/_ref)
# ----------------------------------------------------------------------------------------------
class NfftKernelStruct(C.Structure):
    """Layout of nfft4gp_kernel, SRC/linearalg/kernels.h:65-95."""
    _fields_ = [
        ("_params", C.c_double * 5),
        ("_iparams", C.c_int * 5),
        ("_max_n", C.c_int),
        ("_omp", C.c_int),
        ("_noise_level", C.c_double),
        ("_own_buffer", C.c_int),
        ("_buffer", _dp),
        ("_own_dbuffer", C.c_int),
        ("_dbuffer", _dp),
        ("_fkernel_buffer", C.c_void_p),
        ("_ibufferp", C.c_void_p),
        ("_libufferp", C.c_void_p),
        ("_own_fkernel_buffer_params", C.c_int),
        ("_fkernel_buffer_params", C.c_void_p),
        ("_ldwork", C.c_size_t),
        ("_dwork", _dp),
        ("_external", C.c_void_p),
    ]


_rlib = None

SYMMATVEC = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_double, _dp, C.c_double, _dp)
SOLVE = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, _dp, _dp)


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def ref_lib():
    global _rlib
    if _rlib is None:
        lib = C.CDLL(REF_SO)
        lib.Nfft4GPKernelAdditiveKernelParamCreate.restype = C.c_void_p
        lib.Nfft4GPKernelAdditiveKernelParamCreate.argtypes = [_dp, C.c_int, C.c_int, C.c_int, _ip, C.c_int,
                                                              C.c_int, C.c_void_p]
        lib.Nfft4GPKernelAdditiveKernel.argtypes = [C.c_void_p, _dp, C.c_int, C.c_int, C.c_int, _ip, C.c_int,
                                                    _ip, C.c_int, C.POINTER(_dp), C.POINTER(_dp)]
        lib.Nfft4GPKernelGaussianKernel.argtypes = lib.Nfft4GPKernelAdditiveKernel.argtypes
        lib.Nfft4GPKernelParamCreate.restype = C.c_void_p
        lib.Nfft4GPKernelParamCreate.argtypes = [C.c_int, C.c_int]
        lib.Nfft4GPDenseMatSymv.argtypes = [C.c_void_p, C.c_int, C.c_double, _dp, C.c_double, _dp]
        lib.Nfft4GPDenseGradMatSymv.argtypes = [C.c_void_p, C.c_int, C.c_double, _dp, C.c_double, _dp]
        lib.Nfft4GPSolverPcg.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, _dp, _dp,
                                         C.c_int, C.c_int, C.c_double, _dp, C.POINTER(_dp), _ip, C.c_int]
        lib.Nfft4GPPrecondNysCreate.restype = C.c_void_p
        lib.Nfft4GPPrecondNysSetRank.argtypes = [C.c_void_p, C.c_int]
        lib.Nfft4GPPrecondNysSetPerm.argtypes = [C.c_void_p, _ip, C.c_int]
        lib.Nfft4GPPrecondNysSetupWithKernel.argtypes = [_dp, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                                         C.c_void_p, C.c_int, C.c_void_p]
        lib.Nfft4GPPrecondNysSolve.argtypes = [C.c_void_p, C.c_int, _dp, _dp]
        _rlib = lib
    return _rlib


class RefDenseAdditive:
    """The reference's dense additive kernel (kernels.c:3046-3494) + dense SYMV (matops.c:3-29)."""

    GAUSSIAN = "Nfft4GPKernelGaussianKernel"
    MATERN12 = "Nfft4GPKernelMatern12Kernel"

    def __init__(self, data, windows, nwindows, dwindows, kernel: int = 0):
        self.lib = ref_lib()
        data = np.asfortranarray(data, dtype=np.float64)
        self.n, self.d = data.shape
        self._data = data
        self._win = np.ascontiguousarray(np.asarray(windows, dtype=np.int32).ravel())
        fk = getattr(self.lib, self.GAUSSIAN if kernel == 0 else self.MATERN12)
        self._fk = C.cast(fk, C.c_void_p)
        self.h = self.lib.Nfft4GPKernelAdditiveKernelParamCreate(_d(self._data), self.n, self.n, self.d,
                                                                 _i(self._win), nwindows, dwindows, self._fk)
        self.st = NfftKernelStruct.from_address(self.h)

    def matrices(self, f, l, mu, grad=True):
        self.st._params[0] = f
        self.st._params[1] = l
        self.st._noise_level = mu
        K = _dp()
        dK = _dp()
        self.lib.Nfft4GPKernelAdditiveKernel(self.h, _d(self._data), self.n, self.n, self.d, None, 0, None, 0,
                                             C.byref(K), C.byref(dK) if grad else None)
        n = self.n
        Kn = np.ctypeslib.as_array(K, shape=(n * n,)).reshape(n, n, order="F").copy()
        dKn = None
        if grad:
            dKn = np.ctypeslib.as_array(dK, shape=(3 * n * n,)).reshape(3, n, n).transpose(0, 2, 1).copy()
        self._K, self._dK = K, dK
        return Kn, dKn

    def matsymv(self, x, alpha=1.0, beta=0.0, y=None):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(self.n) if y is None else np.ascontiguousarray(y, dtype=np.float64).copy()
        self.lib.Nfft4GPDenseMatSymv(C.cast(self._K, C.c_void_p), self.n, alpha, _d(x), beta, _d(y))
        return y

    def gradmatsymv(self, x, alpha=1.0, beta=0.0, y=None):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(3 * self.n) if y is None else np.ascontiguousarray(y, dtype=np.float64).copy()
        self.lib.Nfft4GPDenseGradMatSymv(C.cast(self._dK, C.c_void_p), self.n, alpha, _d(x), beta, _d(y))
        return y


def ref_pcg(matvec_py, n, b, x0=None, maxits=1000, tol=1e-6, atol=0, precond_py=None):
    """Run the reference's Nfft4GPSolverPcg (pcg.c:3-206) with Python callbacks.

    ``matvec_py(alpha, x, beta, y)`` and ``precond_py(x_out, rhs)`` operate on numpy views.
    Returns (x, rel_res, rel_res_v (list), iters).
    """
    lib = ref_lib()

    def _mv(_m, nn, alpha, xp, beta, yp):
        xv = np.ctypeslib.as_array(xp, shape=(nn,))
        yv = np.ctypeslib.as_array(yp, shape=(nn,))
        matvec_py(alpha, xv, beta, yv)
        return 0

    def _pc(_p, nn, xp, rp):
        xv = np.ctypeslib.as_array(xp, shape=(nn,))
        rv = np.ctypeslib.as_array(rp, shape=(nn,))
        precond_py(xv, rv)
        return 0

    mv_cb = SYMMATVEC(_mv)
    pc_cb = SOLVE(_pc) if precond_py is not None else None
    x = np.zeros(n) if x0 is None else np.array(x0, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    rel = C.c_double()
    relv = _dp()
    it = C.c_int()
    dummy = C.c_int(1)
    lib.Nfft4GPSolverPcg(None, n, C.cast(mv_cb, C.c_void_p), C.byref(dummy) if pc_cb else None,
                         C.cast(pc_cb, C.c_void_p) if pc_cb else None, _d(x), _d(b), maxits, atol, tol,
                         C.byref(rel), C.byref(relv), C.byref(it), 0)
    m = min(maxits, n)
    hist = np.ctypeslib.as_array(relv, shape=(m + 1,)).copy()
    return x, rel.value, hist, it.value


# ----------------------------------------------------------------------------------------------
# Nystrom preconditioner of the reference (SRC/preconds/nys.c), driven through oracle/_ref
# ----------------------------------------------------------------------------------------------
class PrecondNysStruct(C.Structure):
    """precond_nys, SRC/preconds/nys.h:24-55."""
    _fields_ = [
        ("_k_setup", C.c_int), ("_own_perm", C.c_int), ("_perm", _ip), ("_n", C.c_int), ("_tits", C.c_int),
        ("_titt", C.c_double), ("_tset", C.c_double), ("_tlogdet", C.c_double), ("_tdvp", C.c_double),
        ("_nys_opt", C.c_int), ("_k", C.c_int), ("_eta", C.c_double), ("_f2", C.c_double),
        ("_U", _dp), ("_s", _dp), ("_work", _dp), ("_K", _dp), ("_dU", _dp), ("_dK", _dp),
        ("_chol_K11", C.c_void_p), ("_dvp_nosolve", C.c_int),
    ]


class RefNystrom:
    """Nfft4GPPrecondNysSetupWithKernel (nys.c:518-660) on the reference's dense additive kernel."""

    def __init__(self, dense: "RefDenseAdditive", f, l, mu, k, perm):
        lib = ref_lib()
        self.lib = lib
        st = dense.st
        st._params[0] = f
        st._params[1] = l
        st._noise_level = mu
        self.perm = np.ascontiguousarray(np.asarray(perm, dtype=np.int32))
        self.h = lib.Nfft4GPPrecondNysCreate()
        lib.Nfft4GPPrecondNysSetRank(self.h, k)
        lib.Nfft4GPPrecondNysSetPerm(self.h, _i(self.perm), 0)
        fk = C.cast(lib.Nfft4GPKernelAdditiveKernel, C.c_void_p)
        rc = lib.Nfft4GPPrecondNysSetupWithKernel(_d(dense._data), dense.n, dense.n, dense.d, fk, dense.h, 0,
                                                  self.h)
        assert rc == 0
        self.st = PrecondNysStruct.from_address(self.h)
        self.n, self.k = dense.n, k

    def factors(self):
        n, k = self.n, self.k
        U = np.ctypeslib.as_array(self.st._U, shape=(n * k,)).reshape(n, k, order="F").copy()
        s = np.ctypeslib.as_array(self.st._s, shape=(k,)).copy()
        return U, s, self.st._eta, self.perm.copy()

    def solve(self, x, rhs):
        self.lib.Nfft4GPPrecondNysSolve(C.c_void_p(self.h), self.n, _d(x), _d(rhs))
        return x
