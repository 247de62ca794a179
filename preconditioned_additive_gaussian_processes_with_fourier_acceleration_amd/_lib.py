"""ctypes binding of ``libnfft4gp_amd.so`` (the C ABI declared in ``include/nfft4gp_amd.h``).

The library is built in-tree by ``csrc/Makefile`` (``__graft_entry__.build()``).  Importing this
module never falls back to anything: if the shared object is missing, ``lib()`` raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libnfft4gp_amd.so")
HEADER = os.path.join(os.path.dirname(PKG_DIR), "include", "nfft4gp_amd.h")

dp = C.POINTER(C.c_double)
ip = C.POINTER(C.c_int)
vp = C.c_void_p

SYMMATVEC = C.CFUNCTYPE(C.c_int, vp, C.c_int, C.c_double, vp, C.c_double, vp)
SOLVE = C.CFUNCTYPE(C.c_int, vp, C.c_int, vp, vp)
ALLREDUCE = C.CFUNCTYPE(C.c_int, vp, vp, C.c_longlong)  # Nfft4GPAmdAllreduceFn


class NfftKernelStruct(C.Structure):
    """nfft4gp_kernel, field layout of SRC/linearalg/kernels.h:65-95."""
    _fields_ = [
        ("_params", C.c_double * 5),
        ("_iparams", C.c_int * 5),
        ("_max_n", C.c_int),
        ("_omp", C.c_int),
        ("_noise_level", C.c_double),
        ("_own_buffer", C.c_int),
        ("_buffer", dp),
        ("_own_dbuffer", C.c_int),
        ("_dbuffer", dp),
        ("_fkernel_buffer", vp),
        ("_ibufferp", vp),
        ("_libufferp", vp),
        ("_own_fkernel_buffer_params", C.c_int),
        ("_fkernel_buffer_params", vp),
        ("_ldwork", C.c_size_t),
        ("_dwork", dp),
        ("_external", vp),
    ]


_SIGS = {
    # name: (restype, argtypes)
    "Nfft4GPKernelParamCreate": (vp, [C.c_int, C.c_int]),
    "Nfft4GPKernelParamFree": (None, [vp]),
    "Nfft4GPNFFTKernelParamCreate": (vp, [C.c_int, C.c_int]),
    "Nfft4GPNFFTKernelParamFree": (None, [vp]),
    "Nfft4GPNFFTKernelFree": (None, [vp]),
    "Nfft4GPNFFTKernelParamFreeNFFTKernel": (C.c_int, [vp]),
    "Nfft4GPNFFTKernelParamRemovePoints": (C.c_int, [vp]),
    "Nfft4GPNFFTKernelGaussianKernel": (C.c_int, [vp, vp, C.c_int, C.c_int, C.c_int, ip, C.c_int, ip, C.c_int,
                                                  C.POINTER(vp), C.POINTER(vp)]),
    "Nfft4GPNFFTKernelMatern12Kernel": (C.c_int, [vp, vp, C.c_int, C.c_int, C.c_int, ip, C.c_int, ip, C.c_int,
                                                  C.POINTER(vp), C.POINTER(vp)]),
    "Nfft4GPNFFTMatSymv": (C.c_int, [vp, C.c_int, C.c_double, vp, C.c_double, vp]),
    "Nfft4GPNFFTGradMatSymv": (C.c_int, [vp, C.c_int, C.c_double, vp, C.c_double, vp]),
    "Nfft4GPNFFTAdditiveKernelParamCreate": (vp, [vp, C.c_int, C.c_int, C.c_int, vp, C.c_int, C.c_int]),
    "Nfft4GPNFFTAdditiveKernelGaussianKernel": (C.c_int, [vp, vp, C.c_int, C.c_int, C.c_int, ip, C.c_int, ip,
                                                          C.c_int, C.POINTER(vp), C.POINTER(vp)]),
    "Nfft4GPNFFTAdditiveKernelMatern12Kernel": (C.c_int, [vp, vp, C.c_int, C.c_int, C.c_int, ip, C.c_int, ip,
                                                          C.c_int, C.POINTER(vp), C.POINTER(vp)]),
    "Nfft4GPAdditiveNFFTMatSymv": (C.c_int, [vp, C.c_int, C.c_double, vp, C.c_double, vp]),
    "Nfft4GPAdditiveNFFTGradMatSymv": (C.c_int, [vp, C.c_int, C.c_double, vp, C.c_double, vp]),
    "Nfft4GPAdditiveNFFTKernelFree": (None, [vp]),
    "Nfft4GPNFFTAppendData": (vp, [vp, C.c_int, C.c_int, C.c_int, vp, C.c_int, C.c_int]),
    "Nfft4GPVecNorm2": (C.c_double, [vp, C.c_int]),
    "Nfft4GPVecDdot": (C.c_double, [vp, C.c_int, vp]),
    "Nfft4GPVecFill": (None, [vp, C.c_size_t, C.c_double]),
    "Nfft4GPVecScale": (None, [vp, C.c_size_t, C.c_double]),
    "Nfft4GPVecAxpy": (None, [C.c_double, vp, C.c_size_t, vp]),
    "Nfft4GPSolverPcg": (C.c_int, [vp, C.c_int, vp, vp, vp, vp, vp, C.c_int, C.c_int, C.c_double, dp,
                                   C.POINTER(dp), ip, C.c_int]),
    "Nfft4GPAmdPcgHistoryLength": (C.c_int, []),
    "Nfft4GPSolverFgmres": (C.c_int, [vp, C.c_int, vp, vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_double, dp,
                                      C.POINTER(dp), ip, C.c_int]),
    "Nfft4GPSolverLanczos": (C.c_int, [vp, C.c_int, vp, vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_double, dp,
                                       C.POINTER(dp), ip, ip, C.POINTER(dp), C.POINTER(dp), C.c_int]),
    "Nfft4GPLanczosQuadratureLogdet": (C.c_int, [vp, vp, C.c_int, vp, vp, vp, vp, vp, vp, vp, C.c_int, C.c_int, vp,
                                                 C.c_int, dp, C.POINTER(dp)]),
    "Nfft4GPTransform": (C.c_int, [C.c_int, C.c_double, C.c_int, dp, dp]),
    "Nfft4GPVecRand": (None, [vp, C.c_int]),
    "Nfft4GPVecRadamacher": (None, [vp, C.c_int]),
    "Nfft4GPAmdSetCallbackPointerMode": (None, [C.c_int]),
    "Nfft4GPAmdNysCreate": (vp, [C.c_int, C.c_int, vp, vp, C.c_double, vp]),
    "Nfft4GPAmdNysSolve": (C.c_int, [vp, C.c_int, vp, vp]),
    "Nfft4GPAmdNysFree": (None, [vp]),
    "Nfft4GPAmdNysSetupAdditive": (vp, [vp, vp, C.c_int, C.c_int]),
    "Nfft4GPAmdNysFactors": (C.c_int, [vp, vp, vp, vp, dp]),
    "Nfft4GPAmdNysSetupTimes": (C.c_int, [vp, vp]),
    "Nfft4GPAmdNysSetStorage": (C.c_int, [vp, C.c_int]),
    "Nfft4GPAmdPrecondFsaiCreate": (vp, []),
    "Nfft4GPAmdPrecondFsaiFree": (None, [vp]),
    "Nfft4GPAmdPrecondFsaiReset": (None, [vp]),
    "Nfft4GPAmdPrecondFsaiSetLfil": (None, [vp, C.c_int]),
    "Nfft4GPAmdPrecondFsaiSetKernel": (None, [vp, C.c_int]),
    "Nfft4GPAmdPrecondFsaiSetupWithKernel": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, vp, vp, C.c_int, vp]),
    "Nfft4GPAmdPrecondFsaiSetCsr": (C.c_int, [vp, C.c_int, vp, vp, vp, vp]),
    "Nfft4GPAmdPrecondFsaiCsr": (C.c_int, [vp, vp, vp, vp, vp]),
    "Nfft4GPAmdPrecondFsaiSolve": (C.c_int, [vp, C.c_int, vp, vp]),
    "Nfft4GPAmdPrecondFsaiInvL": (C.c_int, [vp, C.c_int, vp, vp]),
    "Nfft4GPAmdPrecondFsaiInvLT": (C.c_int, [vp, C.c_int, vp, vp]),
    "Nfft4GPAmdPrecondFsaiDvp": (C.c_int, [vp, C.c_int, vp, vp, vp]),
    "Nfft4GPAmdPrecondFsaiTrace": (C.c_int, [vp, vp]),
    "Nfft4GPAmdPrecondFsaiLogdet": (C.c_double, [vp]),
    "Nfft4GPAmdPrecondNysCreate": (vp, []),
    "Nfft4GPAmdPrecondNysFree": (None, [vp]),
    "Nfft4GPAmdPrecondNysReset": (None, [vp]),
    "Nfft4GPAmdPrecondNysSetRank": (None, [vp, C.c_int]),
    "Nfft4GPAmdPrecondNysSetPerm": (None, [vp, vp, C.c_int]),
    "Nfft4GPAmdPrecondNysSetK11Mode": (None, [vp, C.c_int]),
    "Nfft4GPAmdPrecondNysSetupWithKernel": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, vp, vp, C.c_int, vp]),
    "Nfft4GPAmdPrecondNysSolve": (C.c_int, [vp, C.c_int, vp, vp]),
    "Nfft4GPAmdPrecondNysDvp": (C.c_int, [vp, C.c_int, vp, vp, vp]),
    "Nfft4GPAmdPrecondNysTrace": (C.c_int, [vp, vp]),
    "Nfft4GPAmdPrecondNysLogdet": (C.c_double, [vp]),
    "Nfft4GPPrecondNysSolve": (C.c_int, [vp, C.c_int, vp, vp]),
    "Nfft4GPAmdPrecondNysMirrorRelease": (C.c_int, [vp]),
    "Nfft4GPAmdFsaiCreate": (vp, [C.c_int, vp, vp, vp]),
    "Nfft4GPAmdFsaiSolve": (C.c_int, [vp, C.c_int, vp, vp]),
    "Nfft4GPAmdFsaiFree": (None, [vp]),
    "Nfft4GPAmdAfnCreate": (vp, [C.c_int, C.c_int, vp, vp, vp, vp]),
    "Nfft4GPAmdAfnSolve": (C.c_int, [vp, C.c_int, vp, vp]),
    "Nfft4GPAmdAfnFree": (None, [vp]),
    "Nfft4GPAmdAfnSetup": (vp, [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_int, C.c_int, vp]),
    "Nfft4GPAmdAfnSetupSchur": (vp, [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_int, C.c_int, C.c_int,
                                     vp]),
    "Nfft4GPAmdAfnInfo": (C.c_int, [vp, vp, vp, vp, vp, vp]),
    "Nfft4GPAmdSortFps": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, vp, C.c_double, vp, vp]),
    "Nfft4GPAmdRankestNysScaled": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_int, C.c_int, C.c_int]),
    "Nfft4GPAmdRankestDefault": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_int, C.c_int, C.c_int,
                                           C.c_double, vp]),
    "Nfft4GPAmdAfnRankEstimate": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp,
                                            vp]),
    "Nfft4GPAmdSetStream": (None, [vp]),
    "Nfft4GPAmdGetStream": (vp, []),
    "Nfft4GPAmdDeviceAvailable": (C.c_int, []),
    "Nfft4GPAmdVersion": (C.c_char_p, []),
    "Nfft4GPAmdAdditiveLayoutInfo": (C.c_int, [vp, C.POINTER(C.c_longlong), C.c_int]),
    "Nfft4GPAmdTimingEnable": (C.c_int, [vp, C.c_int]),
    "Nfft4GPAmdTimingQuery": (C.c_int, [vp, dp, C.POINTER(C.c_longlong)]),
    "Nfft4GPAmdKernelBench": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, vp, vp, dp]),
    "Nfft4GPAmdAdditiveShardCreate": (vp, [vp, C.c_int, C.c_int, C.c_int, vp, C.c_int, C.c_int, C.c_int, C.c_int]),
    "Nfft4GPAmdShardSpread": (C.c_int, [vp, vp, vp]),
    "Nfft4GPAmdShardFinish": (C.c_int, [vp, vp, C.c_int, C.c_double, vp, C.c_double, vp]),
    "Nfft4GPAmdShardGridSize": (C.c_longlong, [vp]),
    "Nfft4GPAmdPrecondAFNSetup": (vp, [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.c_int, vp, C.c_int]),
    "Nfft4GPAmdAdditiveMatSymvMulti": (C.c_int, [vp, C.c_int, C.c_int, C.c_double, vp, C.c_longlong, C.c_double, vp,
                                               C.c_longlong]),
    "Nfft4GPAmdPrecondAFNCreate": (vp, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
    "Nfft4GPAmdPrecondAFNSetupWithKernel": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, vp, vp, C.c_int, vp]),
    "Nfft4GPAmdPrecondAFNDvp": (C.c_int, [vp, C.c_int, vp, vp, vp]),
    "Nfft4GPAmdPrecondAFNTrace": (C.c_int, [vp, vp]),
    "Nfft4GPAmdPrecondAFNLogdet": (C.c_double, [vp]),
    "Nfft4GPAmdPrecondAFNReset": (None, [vp]),
    "Nfft4GPAmdPrecondAFNSolve": (C.c_int, [vp, C.c_int, vp, vp]),
    "Nfft4GPAmdPrecondAFNInfo": (C.c_int, [vp, ip, ip, C.POINTER(vp), C.POINTER(vp)]),
    "Nfft4GPAmdPrecondAFNFree": (None, [vp]),
    "Nfft4GPAmdCommRcclAvailable": (C.c_int, []),
    "Nfft4GPAmdCommUniqueId": (C.c_int, [vp]),
    "Nfft4GPAmdCommCreateRccl": (vp, [C.c_int, C.c_int, vp]),
    "Nfft4GPAmdCommCreateCallback": (vp, [C.c_int, C.c_int, ALLREDUCE, vp, vp, C.c_longlong]),
    "Nfft4GPAmdCommAllreduce": (C.c_int, [vp, vp, C.c_longlong]),
    "Nfft4GPAmdCommFree": (None, [vp]),
    "Nfft4GPAmdCommRanks": (C.c_int, [vp]),
    "Nfft4GPAmdSetDeterministic": (C.c_int, [vp, C.c_int]),
    "Nfft4GPAmdSetPrecision": (C.c_int, [vp, C.c_int]),
    "Nfft4GPAmdDistTimingEnable": (C.c_int, [vp, C.c_int]),
    "Nfft4GPAmdDistTimingQuery": (C.c_int, [vp, dp, C.POINTER(C.c_longlong)]),
    "Nfft4GPAmdAdditiveComponentShard": (C.c_int, [vp, C.c_int, C.c_int]),
    "Nfft4GPAmdDistCreate": (vp, [vp, C.c_int, vp]),
    "Nfft4GPAmdDistFree": (None, [vp]),
    "Nfft4GPAmdDistMatSymv": (C.c_int, [vp, C.c_int, C.c_double, vp, C.c_double, vp]),
    "Nfft4GPAmdDistSetChunks": (C.c_int, [vp, C.c_int]),
    "Nfft4GPAmdDistPeerEnable": (C.c_int, [vp]),
    "Nfft4GPAmdDistPeerActive": (C.c_int, [vp]),
    "Nfft4GPAmdDistPeerDisable": (C.c_int, [vp]),
    "Nfft4GPAmdDistCheck": (C.c_int, [vp]),
    "Nfft4GPAmdSetFgmresOrtho": (None, [C.c_int]),
    "Nfft4GPAmdFgmresSecondPasses": (C.c_longlong, []),
    "Nfft4GPAmdDistGradMatSymv": (C.c_int, [vp, C.c_int, C.c_double, vp, C.c_double, vp]),
    "Nfft4GPAmdDistGaussianKernel": (C.c_int, [vp, vp, C.c_int, C.c_int, C.c_int, vp, C.c_int, vp, C.c_int, vp,
                                              vp]),
    "Nfft4GPAmdDistMatern12Kernel": (C.c_int, [vp, vp, C.c_int, C.c_int, C.c_int, vp, C.c_int, vp, C.c_int, vp,
                                              vp]),
    "Nfft4GPAmdNysShard": (vp, [vp, C.c_int, C.c_int, vp]),
    "Nfft4GPAmdNysShardSetupAdditive": (vp, [vp, vp, C.c_int, C.c_int]),
    "Nfft4GPAmdAfnShard": (vp, [vp, C.c_int, C.c_int, vp]),
    "Nfft4GPAmdAfnShardSetup": (vp, [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_int, C.c_int, C.c_int,
                                    vp, C.c_int, C.c_int, vp]),
    "Nfft4GPAmdAfnShardInfo": (C.c_int, [vp, ip, ip, C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)]),
    "Nfft4GPAmdAfnSetStorage": (C.c_int, [vp, C.c_int]),
    "Nfft4GPAmdAfnSetOperator": (C.c_int, [vp, vp]),
    "Nfft4GPAmdPrecondAFNSetStorage": (C.c_int, [vp, C.c_int]),
    "Nfft4GPAmdDistAfnSolve": (C.c_int, [vp, C.c_int, vp, vp]),
    "Nfft4GPAmdDistAfnFree": (None, [vp]),
    "Nfft4GPAmdDistNysSolve": (C.c_int, [vp, C.c_int, vp, vp]),
    "Nfft4GPAmdDistNysFree": (None, [vp]),
    "Nfft4GPAmdHostTapPoly": (C.c_int, [vp]),
    "Nfft4GPAmdHostCirculant": (C.c_int, [C.c_int, C.c_double, C.c_double, vp, vp]),
    "Nfft4GPAmdHostPrepare": (C.c_double, [vp, C.c_int, vp]),
    "Nfft4GPAmdHostSymEig": (C.c_int, [vp, C.c_int, vp, vp]),
    "Nfft4GPAmdHostCholInverse": (C.c_int, [vp, C.c_int, C.c_double, vp]),
    "Nfft4GPAmdHostLayout": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_longlong), vp, vp,
                                       vp, vp]),
    "Nfft4GPAmdDeviceLayout": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_longlong), vp, vp,
                                         vp, vp]),
    "Nfft4GPAmdHostLayoutRec": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_longlong),
                                          vp, vp, vp, vp]),
    "Nfft4GPAmdDeviceLayoutRec": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                            C.POINTER(C.c_longlong), vp, vp, vp, vp]),
}

_lib = None


class ExtensionMissing(RuntimeError):
    pass


def header_symbols(path: str = HEADER) -> list[str]:
    """Every function name declared in include/nfft4gp_amd.h."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"\b(Nfft4GP\w+)\s*\(", txt)
    return sorted(set(names))


def lib():
    """Load the HIP C-ABI library (raises ExtensionMissing if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ExtensionMissing(
                f"{LIB_PATH} not found: build it with `make -C {os.path.join(PKG_DIR, 'csrc')}` "
                "(or __graft_entry__.build()). There is no CPU fallback.")
        # One HIP runtime per process.  PyTorch-ROCm bundles its own libamdhip64.so.7; when torch is
        # installed it is loaded FIRST, so this library's libamdhip64.so.7 dependency binds to that
        # already-loaded runtime.  Loading /opt/rocm's copy first instead puts two HIP/HSA runtimes in
        # the process and whichever initialises second loses the device.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def fnptr(name: str) -> int:
    """Address of an exported C function (to pass as func_symmatvec / func_solve)."""
    return C.cast(getattr(lib(), name), vp).value


def kernel_params(f: float, l: float, mu: float, max_n: int) -> int:
    """An nfft4gp_kernel (Nfft4GPKernelParamCreate, kernels.c:404-440) with _params = (f, l) and
    _noise_level = mu, as the reference's callers fill it (gp_loss.c:143-150).  Free with
    Nfft4GPKernelParamFree."""
    h = lib().Nfft4GPKernelParamCreate(int(max_n), 0)
    st = NfftKernelStruct.from_address(h)
    st._params[0] = f
    st._params[1] = l
    st._noise_level = mu
    return h
