"""Krylov solve and preconditioner front-ends over the C ABI.

``pcg``         Nfft4GPSolverPcg (SRC/solvers/pcg.c:3-206) with an NFFT operator and an optional
                Nystrom preconditioner, both passed to the C solver as C function pointers (no
                Python in the iteration loop).
``NystromPrecond``  Nfft4GPAmdNys* -- the apply of SRC/preconds/nys.c:115-173 on factors U, s, eta,
                perm produced by the reference's Nfft4GPPrecondNysSetupWithKernel (nys.c:518-660).
``FsaiPrecond`` Nfft4GPAmdFsai* -- the apply of SRC/preconds/fsai.c:106-123 on the reference's CSR factor.
``AfnPrecond``  Nfft4GPAmdAfn* -- the apply of SRC/preconds/afn.c:82-143.
``fgmres``      Nfft4GPSolverFgmres (SRC/solvers/fgmres.c:3-252).
``logdet``      Nfft4GPLanczosQuadratureLogdet (SRC/solvers/lanczos.c:421-610), no preconditioner.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .nfft import _check_len, _ptr


class NystromPrecond:
    """M^{-1} of the reference's Nystrom preconditioner (nys.c:115-173) held in HBM.

    ``NystromPrecond(U, s, eta, perm)`` takes factors from anywhere (e.g. the reference's own setup);
    ``NystromPrecond.from_additive(op, perm, k)`` builds them on the GPU from the dense additive kernel of
    an NFFTAdditiveKernel's data and hyperparameters (Nfft4GPAmdNysSetupAdditive, nys.c:518-660)."""

    @classmethod
    def from_additive(cls, op, perm, k: int, k11: str = "reference"):
        """k11 = "reference": the reference's K11 exactly (built from slices of the kernel's window
        buffer, see include/nfft4gp_amd.h); "landmarks": K(perm[:k], perm[:k]) as the method intends."""
        mode = {"reference": 0, "landmarks": 1}[k11]
        perm = np.ascontiguousarray(np.asarray(perm, dtype=np.int32))
        if perm.size != op.n:
            raise ValueError("perm must be a permutation of the handle's n points")
        self = cls.__new__(cls)
        self.n, self.k = op.n, int(k)
        self.h = _lib.lib().Nfft4GPAmdNysSetupAdditive(op.h, perm.ctypes.data, int(k), mode)
        if not self.h:
            raise RuntimeError("Nfft4GPAmdNysSetupAdditive failed (see stderr)")
        eta = C.c_double()
        _lib.lib().Nfft4GPAmdNysFactors(self.h, None, None, None, C.byref(eta))
        self.eta = eta.value
        return self

    def set_storage(self, bits: int):
        """U read by the apply in fp64 (64, the reference's) or as an fp32 copy (32; fp64 accumulation)."""
        if _lib.lib().Nfft4GPAmdNysSetStorage(self.h, int(bits)):
            raise ValueError("storage bits must be 32 or 64")
        return self

    def setup_times(self):
        """hipEvent ms of the GPU setup's panel, U1 = Kp G^T, Gram U1^T U1 and U = U1 W kernels."""
        ms = np.zeros(4)
        _lib.lib().Nfft4GPAmdNysSetupTimes(self.h, ms.ctypes.data)
        return {"panel": ms[0], "gemm1": ms[1], "gram": ms[2], "gemm2": ms[3]}

    def factors(self, perm=None):
        """(U, s, eta) with U's rows in the order of ``perm`` (the reference keeps them permuted)."""
        U = np.zeros((self.n, self.k), order="F")
        s = np.zeros(self.k)
        eta = C.c_double()
        p = None if perm is None else np.ascontiguousarray(np.asarray(perm, dtype=np.int32))
        _lib.lib().Nfft4GPAmdNysFactors(self.h, p.ctypes.data if p is not None else None, U.ctypes.data,
                                        s.ctypes.data, C.byref(eta))
        return U, s, eta.value

    def __init__(self, U, s, eta: float, perm=None):
        U = np.asfortranarray(np.asarray(U, dtype=np.float64))
        n, k = U.shape
        s = np.ascontiguousarray(np.asarray(s, dtype=np.float64))
        p = None if perm is None else np.ascontiguousarray(np.asarray(perm, dtype=np.int32))
        self.n, self.k, self.eta = n, k, float(eta)
        self.h = _lib.lib().Nfft4GPAmdNysCreate(n, k, U.ctypes.data, s.ctypes.data, float(eta),
                                                p.ctypes.data if p is not None else None)
        if not self.h:
            raise RuntimeError("Nfft4GPAmdNysCreate failed")

    def solve(self, x, rhs):
        _check_len("x", x, self.n)
        _check_len("rhs", rhs, self.n)
        rc = _lib.lib().Nfft4GPAmdNysSolve(self.h, self.n, _ptr(x)[0], _ptr(rhs)[0])
        if rc:
            raise RuntimeError("Nfft4GPAmdNysSolve failed")
        return x

    @property
    def solve_fnptr(self) -> int:
        return _lib.fnptr("Nfft4GPAmdNysSolve")

    def free(self):
        if getattr(self, "h", None):
            _lib.lib().Nfft4GPAmdNysFree(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class ReferenceNystrom:
    """A precond_nys built by the reference's own Nfft4GPPrecondNysSetupWithKernel (nys.c:518-660), applied
    on the GPU through this library's Nfft4GPPrecondNysSolve (the reference's name, nys.c:115-173), which
    reads the struct's _n, _k, _perm, _eta, _U, _s (nys.h:24-55) and mirrors the factors into HBM once.
    ``ptr`` is the struct's address; the struct stays the caller's."""

    def __init__(self, ptr: int, n: int):
        self.h, self.n = int(ptr), int(n)

    def solve(self, x, rhs):
        _check_len("x", x, self.n)
        _check_len("rhs", rhs, self.n)
        if _lib.lib().Nfft4GPPrecondNysSolve(self.h, self.n, _ptr(x)[0], _ptr(rhs)[0]):
            raise RuntimeError("Nfft4GPPrecondNysSolve failed")
        return x

    @property
    def solve_fnptr(self) -> int:
        return _lib.fnptr("Nfft4GPPrecondNysSolve")

    def free(self):
        """drop the HBM mirror (the struct itself is the reference's to free)"""
        if self.h:
            _lib.lib().Nfft4GPAmdPrecondNysMirrorRelease(self.h)


class _Apply:
    """Common part of the HBM-resident preconditioner handles (func_solve + free)."""

    _solve = _free = ""

    def solve(self, x, rhs):
        _check_len("x", x, self.n)
        _check_len("rhs", rhs, self.n)
        rc = getattr(_lib.lib(), self._solve)(self.h, self.n, _ptr(x)[0], _ptr(rhs)[0])
        if rc:
            raise RuntimeError(f"{self._solve} failed")
        return x

    @property
    def solve_fnptr(self) -> int:
        return _lib.fnptr(self._solve)

    def free(self):
        if getattr(self, "h", None):
            getattr(_lib.lib(), self._free)(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class FsaiPrecond(_Apply):
    """M^{-1} = L^T L of the reference's FSAI preconditioner (fsai.c:106-123) held in HBM.

    ``L_i, L_j, L_a`` are precond_fsai's CSR arrays (fsai.h:22-39) as produced by
    Nfft4GPPrecondFsaiSetupWithKernel (fsai.c:302-...)."""

    _solve, _free = "Nfft4GPAmdFsaiSolve", "Nfft4GPAmdFsaiFree"

    def __init__(self, L_i, L_j, L_a):
        ia = np.ascontiguousarray(np.asarray(L_i, dtype=np.int32))
        ja = np.ascontiguousarray(np.asarray(L_j, dtype=np.int32))
        aa = np.ascontiguousarray(np.asarray(L_a, dtype=np.float64))
        n = ia.size - 1
        if n <= 0 or ja.size < ia[-1] or aa.size < ia[-1]:
            raise ValueError("L_i must have n+1 entries and L_j, L_a at least L_i[n]")
        if ia[-1] and (ja[: ia[-1]].min() < 0 or ja[: ia[-1]].max() >= n):
            raise ValueError("L_j has column indices outside [0, n)")
        self.n = n
        self.h = _lib.lib().Nfft4GPAmdFsaiCreate(n, ia.ctypes.data, ja.ctypes.data, aa.ctypes.data)
        if not self.h:
            raise RuntimeError("Nfft4GPAmdFsaiCreate failed (see stderr)")


class AfnPrecond(_Apply):
    """The reference's AFN apply (afn.c:82-143) held in HBM: perm (n), L11 the lower Cholesky factor of
    A11 = K(perm[:k], perm[:k]) (k x k), K12 = K(perm[:k], perm[k:]) (k x (n-k)) and ``schur`` an
    FsaiPrecond of size n-k (kept alive by this object)."""

    _solve, _free = "Nfft4GPAmdAfnSolve", "Nfft4GPAmdAfnFree"

    def __init__(self, perm, L11, K12, schur: FsaiPrecond | None):
        L11 = np.asfortranarray(np.asarray(L11, dtype=np.float64))
        k = L11.shape[0]
        p = np.ascontiguousarray(np.asarray(perm, dtype=np.int32))
        n = p.size
        K12 = np.asfortranarray(np.asarray(K12, dtype=np.float64).reshape(k, n - k))
        if schur is not None and schur.n != n - k:
            raise ValueError("schur must be an FsaiPrecond of size n - k")
        self.n, self.k, self.schur = n, k, schur
        self.h = _lib.lib().Nfft4GPAmdAfnCreate(n, k, p.ctypes.data, L11.ctypes.data, K12.ctypes.data,
                                                schur.h if schur is not None else None)
        if not self.h:
            raise RuntimeError("Nfft4GPAmdAfnCreate failed (see stderr)")

    @classmethod
    def setup(cls, X, k: int, f: float, l: float, mu: float, perm_opt: str = "fps", perm=None,
              schur_lfil: int = 20, kernel: int = 0, op=None, schur: str = "fsai"):
        """Nfft4GPAmdAfnSetup: the AFN of the plain Gaussian (kernel 0) / Matern-1/2 (1) kernel of the
        points X (n x d) built on the GPU with rank k (afn.c:161-489, schur_opt 3).  perm_opt: "identity"
        (afn.c:245-256), "fps" (farthest points, afn.c:196-209) or "perm" (``perm`` given, n entries).
        With ``op`` (an NFFTAdditiveKernel after its setup) the kernel is the dense additive kernel of
        op's windows and hyperparameters (f, l, mu are then op's).  ``schur``: "fsai" (schur_opt 3, the
        reference's default) or "noise" (schur_opt 0: S^{-1} = I / mu, afn.c:451-459)."""
        L = _lib.lib()
        X = np.asfortranarray(np.asarray(X, dtype=np.float64))
        n, d = X.shape
        opt = {"identity": 0, "fps": 1, "perm": 2}[perm_opt]
        p = None if perm is None else np.ascontiguousarray(np.asarray(perm, dtype=np.int32))
        if opt == 2 and (p is None or p.size != n):
            raise ValueError("perm_opt 'perm' needs a permutation of the n points")
        params = op.h if op is not None else _lib.kernel_params(f, l, mu, n)
        self = cls.__new__(cls)
        self.n, self.schur = n, None
        self.h = L.Nfft4GPAmdAfnSetupSchur(X.ctypes.data, n, n, d, int(k), opt, None if p is None else p.ctypes.data,
                                           {"fsai": 3, "noise": 0}[schur], int(schur_lfil), int(kernel), params)
        if op is None:
            L.Nfft4GPKernelParamFree(params)
        if not self.h:
            raise RuntimeError("Nfft4GPAmdAfnSetup failed (see stderr)")
        kk = C.c_int()
        L.Nfft4GPAmdAfnInfo(self.h, C.byref(kk), None, None, None, None)
        self.k = kk.value
        return self

    def set_storage(self, bits: int):
        """K12 read by the apply's two passes in fp64 (64, the reference's) or as an fp32 copy (32; fp64
        accumulation), Nfft4GPAmdAfnSetStorage."""
        if _lib.lib().Nfft4GPAmdAfnSetStorage(self.h, int(bits)):
            raise ValueError("storage bits must be 32 or 64")
        return self

    def set_operator(self, op):
        """K12^T y and K12 y2 as matvecs of ``op`` (the NFFTAdditiveKernel this AFN was built from, after its
        setup) instead of passes over the stored K12 -- the kernel part of the same operator, to its NFFT accuracy;
        None: back to the stored K12.  Nfft4GPAmdAfnSetOperator; ``op`` must outlive this object's applies."""
        if _lib.lib().Nfft4GPAmdAfnSetOperator(self.h, op.h if op is not None else None):
            raise ValueError("Nfft4GPAmdAfnSetOperator failed (see stderr)")
        self._op = op
        return self

    def info(self):
        """(k, perm, (ia, ja, aa) of the Schur complement's FSAI or None)"""
        L = _lib.lib()
        perm = np.zeros(self.n, np.int32)
        nnz = L.Nfft4GPAmdAfnInfo(self.h, None, perm.ctypes.data, None, None, None)
        if nnz <= 0:
            return self.k, perm, None
        ia = np.zeros(self.n - self.k + 1, np.int32)
        ja = np.zeros(nnz, np.int32)
        aa = np.zeros(nnz)
        L.Nfft4GPAmdAfnInfo(self.h, None, None, ia.ctypes.data, ja.ctypes.data, aa.ctypes.data)
        return self.k, perm, (ia, ja, aa)


class PrecondAFN(_Apply):
    """Nfft4GPPrecondAFNSetup (afn.c:161-489) as the reference runs it (Nfft4GPAmdPrecondAFNSetup): rank
    estimation and ordering, then the AFN when the estimate reaches max_k (or k is 0 or n), the rank-k
    Nystrom on the estimated landmarks when 0 < k < max_k (afn.c:294-304), and MATLAB's RAN fallback -- a
    Nystrom on the same order -- when the AFN's factors break down (afn_setup.m:93-98).

    ``kind`` is "afn", "nystrom" or "ran" (with require_grad also "fsai" at k = 0 and "nystrom_full" at k = n,
    the gradient-capable equivalents of afn.c:263-284's branches); ``k`` the rank.  The kernel is the plain Gaussian / Matern-1/2 of X
    (f, l, mu), or with ``op`` (an NFFTAdditiveKernel after its setup) the dense additive kernel of op's
    windows and hyperparameters.  perm_opt: "random" (0) or "fps" (1); schur: "fsai" (schur_opt 3) or
    "noise" (0).  max_k <= 0: the predefined rank -max_k in natural order, no estimation (afn.c:245-256).
    require_grad: keep the gradient pieces (MATLAB afn_dvp.m / afn_trace.m / afn_logdet.m; the Nystrom
    branches need ``op``) for ``dvp`` (M^{-1} dM/dtheta_g x, g = f, l, mu), ``trace`` and ``logdet``."""

    _solve, _free = "Nfft4GPAmdPrecondAFNSolve", "Nfft4GPAmdPrecondAFNFree"
    KINDS = ("afn", "nystrom", "ran", "fsai", "nystrom_full")

    def __init__(self, X, max_k: int, f: float = 1.0, l: float = 1.0, mu: float = 0.01, perm_opt: str = "random",
                 schur: str = "fsai", schur_lfil: int = 20, nsamples: int = 500, kernel: int = 0, op=None,
                 require_grad: bool = False):
        L = _lib.lib()
        X = np.asfortranarray(np.asarray(X, dtype=np.float64))
        n, d = X.shape
        params = op.h if op is not None else _lib.kernel_params(f, l, mu, n)
        self.n = n
        self.h = L.Nfft4GPAmdPrecondAFNSetup(X.ctypes.data, n, n, d, int(max_k), {"random": 0, "fps": 1}[perm_opt],
                                             {"fsai": 3, "noise": 0}[schur], int(schur_lfil), int(nsamples),
                                             int(kernel), params, int(bool(require_grad)))
        if op is None:
            L.Nfft4GPKernelParamFree(params)
        if not self.h:
            raise RuntimeError("Nfft4GPAmdPrecondAFNSetup failed (see stderr)")
        kind, k = C.c_int(), C.c_int()
        L.Nfft4GPAmdPrecondAFNInfo(self.h, C.byref(kind), C.byref(k), None, None)
        self.kind, self.k = self.KINDS[kind.value], k.value
        self.require_grad = bool(require_grad)

    def set_storage(self, bits: int):
        """The AFN's K12 / the Nystrom branch's U read in fp64 (64) or as an fp32 copy (32; fp64 accumulation),
        Nfft4GPAmdPrecondAFNSetStorage; the gradient-capable branches keep fp64."""
        if _lib.lib().Nfft4GPAmdPrecondAFNSetStorage(self.h, int(bits)):
            raise ValueError("storage bits must be 32 or 64")
        return self

    def set_operator(self, op):
        """The AFN branch's K12 products as matvecs of ``op`` (AfnPrecond.set_operator); no effect on the
        Nystrom / FSAI branches, nor with require_grad (as set_storage: Dvp, Trace and Logdet describe the stored
        factors, so the solve keeps them).  Nfft4GPAmdPrecondAFNInfo + Nfft4GPAmdAfnSetOperator."""
        if self.require_grad:
            return self
        L = _lib.lib()
        kind, afn = C.c_int(), C.c_void_p()
        L.Nfft4GPAmdPrecondAFNInfo(self.h, C.byref(kind), None, C.byref(afn), None)
        if kind.value == 0 and afn.value:
            if L.Nfft4GPAmdAfnSetOperator(afn, op.h if op is not None else None):
                raise ValueError("Nfft4GPAmdAfnSetOperator failed (see stderr)")
            self._op = op
        return self

    def dvp(self, x, mask=None):
        """[M^{-1} dM/df x, M^{-1} dM/dl x, M^{-1} dM/dmu x] (3 n, host numpy or a GPU tensor like x)."""
        _check_len("x", x, self.n)
        y = x.new_zeros(3 * self.n) if hasattr(x, "data_ptr") else np.zeros(3 * self.n)
        yp = C.c_void_p(_ptr(y)[0])
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.int32)
        if _lib.lib().Nfft4GPAmdPrecondAFNDvp(self.h, self.n, None if m is None else m.ctypes.data, _ptr(x)[0],
                                              C.byref(yp)):
            raise RuntimeError("Nfft4GPAmdPrecondAFNDvp failed (setup without require_grad?)")
        return y

    def trace(self):
        """tr(M^{-1} dM/dtheta_g), g = f, l, mu."""
        t = np.zeros(3)
        tp = C.c_void_p(t.ctypes.data)
        if _lib.lib().Nfft4GPAmdPrecondAFNTrace(self.h, C.byref(tp)):
            raise RuntimeError("Nfft4GPAmdPrecondAFNTrace failed (setup without require_grad?)")
        return t

    def logdet(self):
        return float(_lib.lib().Nfft4GPAmdPrecondAFNLogdet(self.h))

    def free(self):
        if getattr(self, "h", None):
            _lib.lib().Nfft4GPAmdPrecondAFNFree(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def afn_rank_estimate(X, max_k: int, f: float = 1.0, l: float = 1.0, mu: float = 0.01, perm_opt: str = "fps",
                      nsamples: int = 500, kernel: int = 0, op=None):
    """Nfft4GPAmdAfnRankEstimate -- the rank / ordering step of Nfft4GPPrecondAFNSetup (afn.c:165-256) on
    the GPU: (k, perm).  k == max_k: build ``AfnPrecond.setup(X, k, ..., perm_opt="perm", perm=perm)``;
    0 < k < max_k: the reference switches to a rank-k Nystrom (afn.c:287-296) -- ``PrecondAFN`` makes that
    choice.  With ``op`` the kernel is op's dense additive kernel.  Draws libc rand()."""
    L = _lib.lib()
    X = np.asfortranarray(np.asarray(X, dtype=np.float64))
    n, d = X.shape
    perm = np.zeros(n, np.int32)
    params = op.h if op is not None else _lib.kernel_params(f, l, mu, n)
    k = L.Nfft4GPAmdAfnRankEstimate(X.ctypes.data, n, n, d, int(max_k), {"random": 0, "fps": 1}[perm_opt],
                                    int(nsamples), int(kernel), params, perm.ctypes.data)
    if op is None:
        L.Nfft4GPKernelParamFree(params)
    if k < 0:
        raise RuntimeError("Nfft4GPAmdAfnRankEstimate failed (see stderr)")
    return k, perm


def sort_fps(X, k: int, tol: float = 0.0):
    """Nfft4GPAmdSortFps -- Nfft4GPSortFps with kFpsAlgorithmParallel1 (ordering.c:422-739) on the GPU:
    (selected points, fill distances).  X: n x d numpy array or a torch GPU tensor of shape (d, n)
    (column-major n x d).  k <= 0 selects until the fill distance drops below tol."""
    L = _lib.lib()
    if hasattr(X, "data_ptr"):
        d, n = X.shape
        src, keep = X.data_ptr(), X
    else:
        keep = np.asfortranarray(np.asarray(X, dtype=np.float64))
        n, d = keep.shape
        src = keep.ctypes.data
    m = n if k <= 0 else min(k, n)
    kk = C.c_int(int(k))
    perm = np.zeros(m, np.int32)
    dist = np.zeros(m)
    if L.Nfft4GPAmdSortFps(src, n, n, d, C.byref(kk), float(tol), perm.ctypes.data, dist.ctypes.data):
        raise RuntimeError("Nfft4GPAmdSortFps failed (see stderr)")
    del keep
    return perm[:kk.value], dist[:kk.value]


def pcg(op, b, x=None, maxits=1000, tol=1e-6, atol=False, precond=None, print_level=0):
    """Nfft4GPSolverPcg(op, n, matvec, precond, precondfunc, x, b, maxits, atol, tol, ...).

    ``op`` is an NFFTAdditiveKernel (its C matvec is used) and ``precond`` a NystromPrecond, FsaiPrecond,
    AfnPrecond or None.
    ``b``/``x`` are numpy arrays or torch GPU tensors.  Returns (x, rel_res, rel_res_v, iters) with the
    reference's reporting semantics (iters = 0 when not converged, pcg.c:19,197).
    """
    if x is None:
        x = b * 0
    n = op.n
    _check_len("b", b, n)
    _check_len("x", x, n)
    rel = C.c_double()
    relv = _lib.dp()
    it = C.c_int()
    L = _lib.lib()
    rc = L.Nfft4GPSolverPcg(op.h, n, op.matvec_fnptr, precond.h if precond else None,
                            precond.solve_fnptr if precond else None, _ptr(x)[0], _ptr(b)[0], int(maxits),
                            int(bool(atol)), float(tol), C.byref(rel), C.byref(relv), C.byref(it), int(print_level))
    if rc:
        raise RuntimeError("Nfft4GPSolverPcg failed")
    length = L.Nfft4GPAmdPcgHistoryLength()
    hist = np.ctypeslib.as_array(relv, shape=(length,)).copy()
    C.CDLL(None).free(relv)
    return x, rel.value, hist, it.value


def fgmres(op, b, x=None, kdim=50, maxits=1000, tol=1e-6, atol=False, precond=None, print_level=-1):
    """Nfft4GPSolverFgmres(op, n, matvec, precond, precondfunc, x, b, kdim, maxits, atol, tol, ...).
    Returns (x, rel_res, rel_res_v, iters)."""
    if x is None:
        x = b * 0
    n = op.n
    _check_len("b", b, n)
    _check_len("x", x, n)
    rel = C.c_double()
    relv = _lib.dp()
    it = C.c_int()
    L = _lib.lib()
    rc = L.Nfft4GPSolverFgmres(op.h, n, op.matvec_fnptr, precond.h if precond else None,
                               precond.solve_fnptr if precond else None, _ptr(x)[0], _ptr(b)[0], int(kdim),
                               int(maxits), int(bool(atol)), float(tol), C.byref(rel), C.byref(relv), C.byref(it),
                               int(print_level))
    if rc:
        raise RuntimeError("Nfft4GPSolverFgmres failed")
    hist = np.ctypeslib.as_array(relv, shape=(int(maxits) + 1,)).copy()
    C.CDLL(None).free(relv)
    return x, rel.value, hist, it.value


def logdet(op, maxits, nvecs, rademacher=None, print_level=-1):
    """Stochastic Lanczos quadrature of logdet(K)/n and its gradient (Nfft4GPLanczosQuadratureLogdet,
    lanczos.c:421-610) for an operator with ``matvec_fnptr`` and ``gradmatvec_fnptr``."""
    val = C.c_double()
    dval = _lib.dp()
    R = None if rademacher is None else np.asfortranarray(np.asarray(rademacher, dtype=np.float64))
    rc = _lib.lib().Nfft4GPLanczosQuadratureLogdet(op.h, op.h, op.n, op.matvec_fnptr, op.gradmatvec_fnptr, None,
                                                   None, None, None, None, int(maxits), int(nvecs),
                                                   R.ctypes.data if R is not None else None, int(print_level),
                                                   C.byref(val), C.byref(dval))
    if rc:
        raise RuntimeError("Nfft4GPLanczosQuadratureLogdet failed")
    g = np.ctypeslib.as_array(dval, shape=(3,)).copy()
    C.CDLL(None).free(dval)
    return val.value, g
