"""MI355X-native NFFT-accelerated additive Gaussian-process kernel operator.

Drop-in for the hot path of Hitenze/Preconditioned_Additive_Gaussian_Processes_with_Fourier_Acceleration
(SRC/external/nfft_interface.c + SRC/solvers/pcg.c + SRC/preconds/nys.c apply): hand-written HIP
kernels for gfx950 behind the C ABI of include/nfft4gp_amd.h (libnfft4gp_amd.so, built in-tree).
"""
from ._lib import ExtensionMissing, header_symbols, lib  # noqa: F401
from .data import read_features, read_labels, read_windows  # noqa: F401
from .gp import gp_loss, gp_predict  # noqa: F401
from .nfft import GAUSSIAN, MATERN12, NFFTAdditiveKernel, NFFTKernel  # noqa: F401
from .solvers import (AfnPrecond, FsaiPrecond, NystromPrecond, PrecondAFN, ReferenceNystrom, afn_rank_estimate, fgmres,  # noqa: F401
                      logdet, pcg, sort_fps)

__version__ = "0.1.0"
