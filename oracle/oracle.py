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
        lib.orc_set_num_threads.argtypes = [C.c_int]
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
        lib.Nfft4GPPrecondNysDvp.argtypes = [C.c_void_p, C.c_int, _ip, _dp, C.POINTER(_dp)]
        lib.Nfft4GPPrecondNysTrace.argtypes = [C.c_void_p, C.POINTER(_dp)]
        lib.Nfft4GPPrecondNysLogdet.argtypes = [C.c_void_p]
        lib.Nfft4GPPrecondNysLogdet.restype = C.c_double
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
    """Nfft4GPPrecondNysSetupWithKernel (nys.c:518-660) on the reference's dense additive kernel; with
    grad=True (require_grad) also its Dvp / Trace / Logdet (nys.c:175-516)."""

    def __init__(self, dense: "RefDenseAdditive", f, l, mu, k, perm, grad=False):
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
        rc = lib.Nfft4GPPrecondNysSetupWithKernel(_d(dense._data), dense.n, dense.n, dense.d, fk, dense.h,
                                                  1 if grad else 0, self.h)
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

    def dvp(self, x, mask=None):
        """[M^{-1} dM/df x; M^{-1} dM/dl x; M^{-1} dM/dmu x] (3n), nys.c:175-330."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(3 * self.n)
        yp = _d(y)
        m = None if mask is None else _i(np.ascontiguousarray(mask, dtype=np.int32))
        assert self.lib.Nfft4GPPrecondNysDvp(C.c_void_p(self.h), self.n, m, _d(x), C.byref(yp)) == 0
        return y

    def trace(self):
        t = np.zeros(3)
        tp = _d(t)
        assert self.lib.Nfft4GPPrecondNysTrace(C.c_void_p(self.h), C.byref(tp)) == 0
        return t

    def logdet(self):
        return float(self.lib.Nfft4GPPrecondNysLogdet(C.c_void_p(self.h)))


# ----------------------------------------------------------------------------------------------
# FSAI preconditioner of the reference (SRC/preconds/fsai.c), driven through oracle/_ref, and the
# AFN apply (SRC/preconds/afn.c:82-143, not in the reference build) restated in numpy on top of it
# ----------------------------------------------------------------------------------------------
class PrecondFsaiStruct(C.Structure):
    """precond_fsai, SRC/preconds/fsai.h:22-39."""
    _fields_ = [
        ("_lfil", C.c_int), ("_n", C.c_int), ("_tits", C.c_int), ("_titt", C.c_double), ("_tset", C.c_double),
        ("_tlogdet", C.c_double), ("_tdvp", C.c_double), ("_L_i", _ip), ("_L_j", _ip), ("_L_a", _dp),
        ("_dL_a", _dp), ("_work", _dp),
    ]


def ref_gaussian_params(f, l, mu, max_n):
    """Nfft4GPKernelParamCreate (kernels.c:404-440) with _params = (f, l), _noise_level = mu; omp = 1 gives
    each OpenMP thread its own _dwork (the FSAI setup calls the kernel inside a parallel region)."""
    lib = ref_lib()
    h = lib.Nfft4GPKernelParamCreate(int(max_n), 1)
    st = NfftKernelStruct.from_address(h)
    st._params[0] = f
    st._params[1] = l
    st._noise_level = mu
    return h


def ref_gaussian_matrix(params, data, permr=None, permc=None):
    """The reference's Nfft4GPKernelGaussianKernel (kernels.c:680-1289): K(permr, permc) (no noise),
    K(permr, permr) + noise when permc is None (only its lower triangle is written), the full matrix f^2 (exp(-|xi - xj|^2 / 2 l^2) + mu I)
    when no permutation is given."""
    lib = ref_lib()
    data = np.asfortranarray(data, dtype=np.float64)
    n, d = data.shape
    K = _dp()
    if permr is None:
        lib.Nfft4GPKernelGaussianKernel(params, _d(data), n, n, d, None, 0, None, 0, C.byref(K), None)
        kr = kc = n
    elif permc is None:
        pr = np.ascontiguousarray(permr, dtype=np.int32)
        kr = kc = pr.size
        lib.Nfft4GPKernelGaussianKernel(params, _d(data), n, n, d, _i(pr), kr, None, 0, C.byref(K), None)
    else:
        pr = np.ascontiguousarray(permr, dtype=np.int32)
        pc = np.ascontiguousarray(permc, dtype=np.int32)
        kr, kc = pr.size, pc.size
        lib.Nfft4GPKernelGaussianKernel(params, _d(data), n, n, d, _i(pr), kr, _i(pc), kc, C.byref(K), None)
    out = np.ctypeslib.as_array(K, shape=(kr * kc,)).reshape(kr, kc, order="F").copy()
    C.CDLL(None).free(K)
    return out


class RefFsai:
    """Nfft4GPPrecondFsaiSetupWithKernel (fsai.c:302-312: KNN pattern of `data`, per-row Cholesky solves
    on kernel submatrices) and its apply Nfft4GPPrecondFsaiSolve (fsai.c:106-123), via oracle/_ref.
    ``kernel`` names a func_kernel of the reference (default its dense Gaussian kernel, kernels.c:680)
    and ``params`` its parameter handle."""

    def __init__(self, data, params, lfil, kernel="Nfft4GPKernelGaussianKernel", grad=False):
        lib = ref_lib()
        self.lib = lib
        lib.Nfft4GPPrecondFsaiCreate.restype = C.c_void_p
        lib.Nfft4GPPrecondFsaiSetLfil.argtypes = [C.c_void_p, C.c_int]
        lib.Nfft4GPPrecondFsaiSetupWithKernel.argtypes = [_dp, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                                          C.c_void_p, C.c_int, C.c_void_p]
        lib.Nfft4GPPrecondFsaiSolve.argtypes = [C.c_void_p, C.c_int, _dp, _dp]
        self._data = np.asfortranarray(data, dtype=np.float64)
        n, d = self._data.shape
        self.n = n
        self.h = lib.Nfft4GPPrecondFsaiCreate()
        lib.Nfft4GPPrecondFsaiSetLfil(self.h, lfil)
        fk = C.cast(getattr(lib, kernel), C.c_void_p)
        rc = lib.Nfft4GPPrecondFsaiSetupWithKernel(_d(self._data), n, n, d, fk, params, 1 if grad else 0, self.h)
        assert rc == 0
        self.st = PrecondFsaiStruct.from_address(self.h)
        self.grad = grad
        for name, args in (("Nfft4GPPrecondFsaiDvp", [C.c_void_p, C.c_int, _ip, _dp, C.POINTER(_dp)]),
                           ("Nfft4GPPrecondFsaiTrace", [C.c_void_p, C.POINTER(_dp)]),
                           ("Nfft4GPPrecondFsaiLogdet", [C.c_void_p]),
                           ("Nfft4GPPrecondFsaiInvL", [C.c_void_p, C.c_int, _dp, _dp]),
                           ("Nfft4GPPrecondFsaiInvLT", [C.c_void_p, C.c_int, _dp, _dp])):
            getattr(lib, name).argtypes = args
        lib.Nfft4GPPrecondFsaiLogdet.restype = C.c_double

    def csr(self):
        n = self.n
        ia = np.ctypeslib.as_array(self.st._L_i, shape=(n + 1,)).copy()
        nnz = int(ia[n])
        ja = np.ctypeslib.as_array(self.st._L_j, shape=(nnz,)).copy()
        aa = np.ctypeslib.as_array(self.st._L_a, shape=(nnz,)).copy()
        return ia, ja, aa

    def solve(self, rhs):
        rhs = np.ascontiguousarray(rhs, dtype=np.float64)
        x = np.zeros(self.n)
        self.lib.Nfft4GPPrecondFsaiSolve(C.c_void_p(self.h), self.n, _d(x), _d(rhs))
        return x

    def dl(self):
        """the gradient factors dL_a (3 nnz: f, l, mu), fsai.c:472-476"""
        nnz = int(np.ctypeslib.as_array(self.st._L_i, shape=(self.n + 1,))[self.n])
        return np.ctypeslib.as_array(self.st._dL_a, shape=(3 * nnz,)).copy()

    def inv_l(self, rhs, trans=False):
        rhs = np.ascontiguousarray(rhs, dtype=np.float64)
        x = np.zeros(self.n)
        fn = self.lib.Nfft4GPPrecondFsaiInvLT if trans else self.lib.Nfft4GPPrecondFsaiInvL
        fn(C.c_void_p(self.h), self.n, _d(x), _d(rhs))
        return x

    def dvp(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(3 * self.n)
        yp = _d(y)
        assert self.lib.Nfft4GPPrecondFsaiDvp(C.c_void_p(self.h), self.n, None, _d(x), C.byref(yp)) == 0
        return y

    def trace(self):
        t = np.zeros(3)
        tp = _d(t)
        assert self.lib.Nfft4GPPrecondFsaiTrace(C.c_void_p(self.h), C.byref(tp)) == 0
        return t

    def logdet(self):
        return float(self.lib.Nfft4GPPrecondFsaiLogdet(C.c_void_p(self.h)))


class FpsStruct(C.Structure):
    """ordering_fps, SRC/linearalg/ordering.h:27-61."""
    _fields_ = [
        ("_algorithm", C.c_int), ("_tol", C.c_double), ("_rho", C.c_double), ("_fdist", C.c_void_p),
        ("_fdist_params", C.c_void_p), ("_dist", _dp), ("_build_pattern", C.c_int), ("_pattern_lfil", C.c_int),
        ("_pattern_opt", C.c_int), ("_S_i", _ip), ("_S_j", _ip),
    ]


def ref_sort_fps(data, k, tol=0.0):
    """Nfft4GPSortFps with kFpsAlgorithmParallel1 (ordering.c:422-739) via oracle/_ref: the selected points
    and their fill distances (_dist).  k <= 0 selects until the fill distance drops below tol."""
    lib = ref_lib()
    lib.Nfft4GPOrdFpsCreate.restype = C.c_void_p
    lib.Nfft4GPOrdFpsFree.argtypes = [C.c_void_p]
    lib.Nfft4GPSortFps.argtypes = [C.c_void_p, _dp, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int),
                                   C.POINTER(_ip)]
    data = np.asfortranarray(data, dtype=np.float64)
    n, d = data.shape
    h = lib.Nfft4GPOrdFpsCreate()
    st = FpsStruct.from_address(h)
    st._algorithm = 0  # kFpsAlgorithmParallel1
    st._tol = tol
    kk = C.c_int(k)
    perm = _ip()
    assert lib.Nfft4GPSortFps(h, _d(data), n, n, d, C.byref(kk), C.byref(perm)) == 0
    m = kk.value
    p = np.ctypeslib.as_array(perm, shape=(m,)).copy()
    dist = np.ctypeslib.as_array(st._dist, shape=(m,)).copy()
    C.CDLL(None).free(perm)
    lib.Nfft4GPOrdFpsFree(h)
    return p, dist


def fps_par1(data, k, tol=0.0):
    """Nfft4GPSortFpsPar1 (ordering.c:422-711) restated in numpy: start at the point closest to the mean
    (ordering.c:467-538), give it the largest distance to it (:594-599), then repeatedly append the
    unselected point farthest from the selected set (strict >, lowest index on ties, (0, 0) when no
    distance is positive, :617-690) while fewer than k are selected and the newest one's distance is
    >= tol.  Distances as Nfft4GPDistanceEuclid (kernels.c:5-15): sqrt of the squares summed in feature
    order."""
    X = np.asarray(data, dtype=np.float64)
    n, d = X.shape
    k = n if k <= 0 else k

    def dist_to(q):
        v = np.zeros(n)
        for c in range(d):
            t = X[:, c] - q[c]
            v = v + t * t
        return np.sqrt(v)

    mean = np.zeros(d)
    for c in range(d):
        mean[c] = np.sum(X[:, c] / n)
    i1 = int(np.argmin(dist_to(mean)))
    dc = dist_to(X[i1])
    i2 = int(np.argmax(dc)) if dc.max() > 0 else 0
    dmax = dc[i2] if dc.max() > 0 else 0.0
    marker = np.full(n, -1)
    perm, dist = [i1], [dmax]
    dc[i1] = dmax
    marker[i1] = 0
    if dmax < tol or len(perm) >= k:
        return np.array(perm, dtype=np.int32), np.array(dist)
    i1 = i2
    marker[i1] = 1
    perm.append(i1)
    dist.append(dmax)
    while len(perm) < k and dc[i1] >= tol:
        free = marker < 0
        dc[free] = np.minimum(dc[free], dist_to(X[i1])[free])
        cand = np.where(free, dc, -1.0)
        i2 = int(np.argmax(cand))
        if cand[i2] > 0:
            dmax = cand[i2]
        else:
            i2, dmax = 0, 0.0
        i1 = i2
        marker[i1] = len(perm)
        perm.append(i1)
        dist.append(dmax)
    return np.array(perm, dtype=np.int32), np.array(dist)


def expand_perm(perm, n):
    """Nfft4GPExpandPerm (utils.c:208-245): perm, then the unused indices in ascending order."""
    used = np.zeros(n, dtype=bool)
    used[perm] = True
    return np.concatenate([np.asarray(perm, dtype=np.int32), np.flatnonzero(~used).astype(np.int32)])


class RankestStruct(C.Structure):
    """rankest, SRC/linearalg/rankest.h:13-23."""
    _fields_ = [
        ("_nsample", C.c_int), ("_nsample_r", C.c_int), ("_max_rank", C.c_int), ("_full_tol", C.c_double),
        ("_kernel_func", C.c_void_p), ("_kernel_str", C.c_void_p), ("_ordering_str", C.c_void_p), ("_perm", _ip),
    ]


def ref_rankest(data, params, max_rank, nsample=500, nsample_r=5, which="scaled", seed=None):
    """Nfft4GPRankestNysScaled (rankest.c:354-391) or Nfft4GPRankestDefault (:132-181) of the reference on its
    dense Gaussian kernel (params: an nfft4gp_kernel handle), via oracle/_ref; srand(seed) first when given.
    Returns the rank (and, for "default", the selected points)."""
    lib = ref_lib()
    lib.Nfft4GPRankestStrCreate.restype = C.c_void_p
    lib.Nfft4GPRankestStrFree.argtypes = [C.c_void_p]
    fn = lib.Nfft4GPRankestNysScaled if which == "scaled" else lib.Nfft4GPRankestDefault
    fn.argtypes = [C.c_void_p, _dp, C.c_int, C.c_int, C.c_int]
    fn.restype = C.c_int
    data = np.asfortranarray(data, dtype=np.float64)
    n, d = data.shape
    h = lib.Nfft4GPRankestStrCreate()
    st = RankestStruct.from_address(h)
    st._max_rank = max_rank
    st._nsample = nsample
    st._nsample_r = nsample_r
    st._kernel_func = C.cast(lib.Nfft4GPKernelGaussianKernel, C.c_void_p).value
    st._kernel_str = params
    if seed is not None:
        C.CDLL(None).srand(seed)
    r = fn(h, _d(data), n, n, d)
    perm = None
    if which != "scaled":
        perm = np.ctypeslib.as_array(st._perm, shape=(r,)).copy() if r > 0 else np.zeros(0, np.int32)
    lib.Nfft4GPRankestStrFree(h)
    return r if which == "scaled" else (r, perm)


def ref_schur_params(data, perm, k, chol_K11, gauss_params):
    """Nfft4GPKernelSchurCombineKernelParamCreate (kernels.c:3496-3596, no gradient): the kernel of the
    Schur complement K22 - K21 K11^{-1} K12 the reference's AFN setup hands to FSAI (afn.c:473)."""
    lib = ref_lib()
    f = lib.Nfft4GPKernelSchurCombineKernelParamCreate
    f.restype = C.c_void_p
    f.argtypes = [_dp, C.c_int, C.c_int, C.c_int, _ip, C.c_int, _dp, _dp, C.c_void_p, C.c_void_p, C.c_int,
                  C.c_int]
    data = np.asfortranarray(data, dtype=np.float64)
    n, d = data.shape
    perm = np.ascontiguousarray(perm, dtype=np.int32)
    L = np.asfortranarray(chol_K11, dtype=np.float64)
    fk = C.cast(lib.Nfft4GPKernelGaussianKernel, C.c_void_p)
    keep = (data, perm, L)
    return f(_d(data), n, n, d, _i(perm), k, _d(L), None, fk, gauss_params, 1, 0), keep


def csr_mv(ia, ja, aa, x, trans=False):
    """Nfft4GPCsrMv (matops.c:139-272) with alpha = 1, beta = 0: y = L x ('N') or L^T x ('T')."""
    n = ia.size - 1
    rows = np.repeat(np.arange(n), np.diff(ia))
    nnz = int(ia[n])
    prod = aa[:nnz] * (x[rows] if trans else x[ja[:nnz]])
    y = np.zeros(n)
    np.add.at(y, ja[:nnz] if trans else rows, prod)
    return y


def fsai_apply(ia, ja, aa, rhs):
    """Nfft4GPPrecondFsaiSolve (fsai.c:106-123): x = L^T (L rhs)."""
    return csr_mv(ia, ja, aa, csr_mv(ia, ja, aa, rhs), trans=True)


def gaussian_block(X, f, l, rows, cols):
    """f^2 exp(-|x_r - x_c|^2 / 2 l^2), the off-diagonal blocks of kernels.c:680-1289."""
    A, B = X[rows], X[cols]
    D = ((A[:, None, :] - B[None, :, :]) ** 2).sum(-1)
    return f * f * np.exp(-D / (2.0 * l * l))


def afn_apply(perm, L11, K12, schur_solve, rhs):
    """Nfft4GPPrecondAFNSolve (afn.c:82-143) restated: [rp; rp2] = rhs(perm); y = A11 \\ rp (A11 = L11
    L11^T); rp2 -= K12^T y; y2 = S^{-1} rp2; rp -= K12 y2; y = A11 \\ rp; x(perm) = [y; y2].
    k = 0 applies schur_solve to rhs; k = n solves with A11 on the unpermuted rhs (afn.c:101-110)."""
    import scipy.linalg as sl
    n = rhs.shape[0]
    k = L11.shape[0]
    if k == 0:
        return schur_solve(rhs)
    if k == n:
        return sl.cho_solve((L11, True), rhs)
    rp = rhs[perm].copy()
    y = sl.cho_solve((L11, True), rp[:k])
    rp2 = rp[k:] - K12.T @ y
    y2 = schur_solve(rp2)
    r1 = rp[:k] - K12 @ y2
    y = sl.cho_solve((L11, True), r1)
    x = np.empty(n)
    x[perm] = np.concatenate([y, y2])
    return x


# ----------------------------------------------------------------------------------------------
# FGMRES (fgmres.c), Lanczos quadrature (lanczos.c:421-610) and the GP loss (gp_loss.c:96-307) of the
# reference, driven through oracle/_ref with its dense operator and Nystrom preconditioner
# ----------------------------------------------------------------------------------------------
def _host_cb(matvec_py, nout=1):
    def _mv(_m, nn, alpha, xp, beta, yp):
        xv = np.ctypeslib.as_array(xp, shape=(nn,))
        yv = np.ctypeslib.as_array(yp, shape=(nout * nn,))
        matvec_py(alpha, xv, beta, yv)
        return 0
    return SYMMATVEC(_mv)


def ref_fgmres(matvec_py, n, b, kdim, maxits, tol, atol=0, precond_py=None, x0=None):
    """Nfft4GPSolverFgmres (fgmres.c:3-252) with Python callbacks; returns (x, rel_res, hist, iters)."""
    lib = ref_lib()
    lib.Nfft4GPSolverFgmres.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, _dp, _dp, C.c_int,
                                        C.c_int, C.c_int, C.c_double, _dp, C.POINTER(_dp), _ip, C.c_int]
    mv_cb = _host_cb(matvec_py)

    def _pc(_p, nn, xp, rp):
        precond_py(np.ctypeslib.as_array(xp, shape=(nn,)), np.ctypeslib.as_array(rp, shape=(nn,)))
        return 0

    pc_cb = SOLVE(_pc) if precond_py is not None else None
    x = np.zeros(n) if x0 is None else np.array(x0, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    rel, relv, it, dummy = C.c_double(), _dp(), C.c_int(), C.c_int(1)
    lib.Nfft4GPSolverFgmres(None, n, C.cast(mv_cb, C.c_void_p), C.byref(dummy) if pc_cb else None,
                            C.cast(pc_cb, C.c_void_p) if pc_cb else None, _d(x), _d(b), kdim, maxits, atol, tol,
                            C.byref(rel), C.byref(relv), C.byref(it), -1)
    hist = np.ctypeslib.as_array(relv, shape=(maxits + 1,)).copy()
    return x, rel.value, hist, it.value


def ref_logdet_quadrature(matvec_py, dmatvec_py, n, maxits, nvecs, radamacher):
    """Nfft4GPLanczosQuadratureLogdet (lanczos.c:421-610), no preconditioner, fixed Rademacher probes."""
    lib = ref_lib()
    f = lib.Nfft4GPLanczosQuadratureLogdet
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                  C.c_void_p, C.c_void_p, C.c_int, C.c_int, _dp, C.c_int, _dp, C.POINTER(_dp)]
    mv_cb = _host_cb(matvec_py)
    dmv_cb = _host_cb(dmatvec_py, 3)
    R = np.asfortranarray(radamacher, dtype=np.float64)
    val = C.c_double()
    dval = _dp()
    rc = f(None, None, n, C.cast(mv_cb, C.c_void_p), C.cast(dmv_cb, C.c_void_p), None, None, None, None, None,
           maxits, nvecs, _d(R), -1, C.byref(val), C.byref(dval))
    assert rc == 0
    return val.value, np.ctypeslib.as_array(dval, shape=(3,)).copy()


class RefGpLoss:
    """Nfft4GPGpLoss (gp_loss.c:96-307) of the reference on its dense additive kernel (kernels.c:3099-3494,
    Gaussian), Nfft4GPDenseMatSymv / Nfft4GPDenseGradMatSymv (matops.c:3-29) and, optionally, its Nystrom
    preconditioner with gradients (nys.c:175-660).  ``args(lib_fn)`` gives the argument tuple with the
    reference's own function pointers, so the same call can be made on this library's Nfft4GPGpLoss."""

    def __init__(self, X, windows, nw, dw, k=0, perm=None):
        lib = ref_lib()
        self.lib = lib
        self.X = np.asfortranarray(X, dtype=np.float64)
        self.n, self.d = self.X.shape
        self.win = np.ascontiguousarray(np.asarray(windows, dtype=np.int32).ravel())
        fk = C.cast(lib.Nfft4GPKernelGaussianKernel, C.c_void_p)
        mk = lambda: lib.Nfft4GPKernelAdditiveKernelParamCreate(_d(self.X), self.n, self.n, self.d, _i(self.win),
                                                                  nw, dw, fk)
        self.kh = mk()
        self.pkh = mk()
        self.k = k
        self.nys = None
        if k > 0:
            self.perm = np.ascontiguousarray(np.asarray(perm, dtype=np.int32))
            self.nys = lib.Nfft4GPPrecondNysCreate()
            lib.Nfft4GPPrecondNysSetRank(self.nys, k)
            lib.Nfft4GPPrecondNysSetPerm(self.nys, _i(self.perm), 0)
        self.dwork = np.zeros(4 * self.n * self.n + 4 * self.n)

    def fn(self, name):
        return C.cast(getattr(self.lib, name), C.c_void_p).value

    def args(self, hyper, label, maxits, nvecs, radamacher, tol=1e-8, transform=0):
        x = np.ascontiguousarray(hyper, dtype=np.float64)
        lab = np.ascontiguousarray(label, dtype=np.float64)
        R = np.asfortranarray(radamacher, dtype=np.float64)
        self._keep = (x, lab, R)
        nys = self.k > 0
        P = lambda name: self.fn(name) if nys else None
        return (x.ctypes.data, self.X.ctypes.data, lab.ctypes.data, self.n, self.n, self.d,
                self.fn("Nfft4GPKernelAdditiveKernel"), self.kh, None, self.fn("Nfft4GPDenseMatSymv"),
                self.fn("Nfft4GPDenseGradMatSymv"), self.fn("Nfft4GPKernelAdditiveKernel"), self.pkh, None,
                P("Nfft4GPPrecondNysSetupWithKernel"), P("Nfft4GPPrecondNysSolve"), P("Nfft4GPPrecondNysTrace"),
                P("Nfft4GPPrecondNysLogdet"), P("Nfft4GPPrecondNysDvp"), P("Nfft4GPPrecondNysReset"),
                self.nys if nys else None, 0, tol, maxits, maxits, nvecs, R.ctypes.data, transform, None, 0,
                self.dwork.ctypes.data)

    ARGTYPES = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_double, C.c_int, C.c_int, C.c_int,
                C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, _dp, _dp]

    def run(self, fn, *a, **kw):
        """fn = a Nfft4GPGpLoss entry point (the reference's, or this library's); returns (loss, grad)."""
        fn.argtypes = self.ARGTYPES
        fn.restype = C.c_int
        loss = np.zeros(1)
        grad = np.zeros(3)
        rc = fn(*self.args(*a, **kw), _d(loss), _d(grad))
        assert rc == 0, rc
        return float(loss[0]), grad

    def reference(self, *a, **kw):
        return self.run(self.lib.Nfft4GPGpLoss, *a, **kw)


FUNC_KERNEL = C.CFUNCTYPE(C.c_int, C.c_void_p, _dp, C.c_int, C.c_int, C.c_int, _ip, C.c_int, _ip, C.c_int,
                          C.POINTER(_dp), C.POINTER(_dp))


def ref_gp_loss_nfft(X, windows, nw, dw, label, hyper, maxits, nvecs, radamacher, tol=1e-8):
    """The reference's Nfft4GPGpLoss (gp_loss.c:96-307, compiled in oracle/_ref) driven by this oracle's
    NFFT operator (the CPU restatement of nfft_interface.c): the kernel setup callback reads f, l, mu from
    the kernel struct the loss writes (gp_loss.c:143-150) and sets the oracle up; matvec / grad matvec
    are the oracle's (no preconditioner).  Returns (loss, grad)."""
    lib = ref_lib()
    X = np.asfortranarray(X, dtype=np.float64)
    n, d = X.shape
    o = OracleAdditiveNFFT(X, np.asarray(windows, dtype=np.int32), nw, dw)
    kh = lib.Nfft4GPKernelParamCreate(n, 0)
    st = NfftKernelStruct.from_address(kh)

    def fk(_s, _data, _n, _ldim, _d, _pr, _kr, _pc, _kc, Kp, dKp):
        o.setup(0, st._params[0], st._params[1], st._noise_level)
        Kp[0] = C.cast(C.c_void_p(kh), _dp)
        dKp[0] = C.cast(C.c_void_p(kh), _dp)
        return 0

    fk_cb = FUNC_KERNEL(fk)
    mv_cb = _host_cb(lambda a, xv, b, yv: yv.__setitem__(slice(None), o.matsymv(xv.copy(), a, b, yv.copy())))
    dmv_cb = _host_cb(lambda a, xv, b, yv: yv.__setitem__(slice(None), o.gradmatsymv(xv.copy(), a, b, yv.copy())),
                      3)
    x = np.ascontiguousarray(hyper, dtype=np.float64)
    lab = np.ascontiguousarray(label, dtype=np.float64)
    R = np.asfortranarray(radamacher, dtype=np.float64)
    loss = np.zeros(1)
    grad = np.zeros(3)
    fn = lib.Nfft4GPGpLoss
    fn.argtypes = RefGpLoss.ARGTYPES
    fn.restype = C.c_int
    V = lambda cb: C.cast(cb, C.c_void_p).value
    pkh = lib.Nfft4GPKernelParamCreate(n, 0)  # gp_loss.c:145-150 writes the preconditioner's kernel struct too
    rc = fn(x.ctypes.data, X.ctypes.data, lab.ctypes.data, n, n, d, V(fk_cb), kh, None, V(mv_cb), V(dmv_cb),
            None, pkh, None, None, None, None, None, None, None, None, 0, tol, maxits, maxits, nvecs,
            R.ctypes.data, 0, None, -1, None, _d(loss), _d(grad))
    assert rc == 0
    return float(loss[0]), grad


def ref_nfft_gp_predict(X, Xp, windows, nw, dw, label, hyper, maxits, tol, with_std=True, atol=0):
    """Nfft4GPAdditiveNFFTGpPredict (nfft_interface.c:873-1068) restated over the reference's own FGMRES
    (fgmres.c, oracle/_ref) and this oracle's NFFT operator, softplus transform (transform.c:20-37):
    mean = (K_all [K11^{-1} y; 0])[n:], std_i = sqrt|K22_ii - K21_i K11^{-1} K12_i| with one FGMRES
    (restart n, maxits n) per prediction point.  Returns (mean, std or None)."""
    tv = np.where(np.asarray(hyper) > 20, hyper, np.log1p(np.exp(np.minimum(hyper, 20))))
    f, l, mu = (float(v) for v in tv)
    X = np.asfortranarray(X, dtype=np.float64)
    n = X.shape[0]
    Xa = np.asfortranarray(np.vstack([X, np.asarray(Xp, dtype=np.float64)]))
    na = Xa.shape[0]
    o11 = OracleAdditiveNFFT(X, windows, nw, dw)
    o11.setup(0, f, l, mu)
    oa = OracleAdditiveNFFT(Xa, windows, nw, dw)
    oa.setup(0, f, l, mu)

    def mv11(a, xv, b, yv):
        yv[:] = o11.matsymv(xv.copy(), a, b, yv.copy())

    iKY, _, _, _ = ref_fgmres(mv11, n, np.asarray(label, dtype=np.float64), maxits, maxits, tol, atol=atol)
    helper = oa.matsymv(np.concatenate([iKY, np.zeros(na - n)]))
    mean = helper[n:].copy()
    if not with_std:
        return mean, None
    std = np.zeros(na - n)
    for i in range(na - n):
        e = np.zeros(na)
        e[n + i] = 1.0
        h = oa.matsymv(e)
        sol, _, _, _ = ref_fgmres(mv11, n, h[:n].copy(), n, n, tol, atol=atol)
        std[i] = np.sqrt(abs(h[n + i] - np.dot(h[:n], sol)))
    return mean, std
