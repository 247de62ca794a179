// kernel_eval.hpp -- kernel entries of the preconditioner setups (FSAI, AFN, rank estimation).
//
// The reference's plain kernels, f^2 exp(-r^2 / 2 l^2) (Nfft4GPKernelGaussianKernel, kernels.c:680-1289)
// and f^2 exp(-r / l) (Nfft4GPKernelMatern12Kernel, :2390-3033), and its dense additive kernel
// (Nfft4GPKernelAdditiveKernel, :3099-3494): f^2 (1/nw) sum_w exp(-r_w^2 / 2 l^2) over windows of dw
// coordinates (the last one last_dw), coordinates packed window after window as in the kernel's
// gathered buffer.  The plain kernel is the one-window case.  Diagonal: f^2 (1 + mu) (kernels.c:695).
#pragma once

#include <hip/hip_runtime.h>

#include "internal.h"

namespace nfft4gp_amd {

struct KernelParams {
   int kernel = 0;  // 0 Gaussian, 1 Matern-1/2
   double f2 = 1.0, inv = 0.5, mu = 0.0;
   double df_scale = 2.0;  // 2/f
   double dl_scale = 1.0;  // f^2 / l^3 (Gaussian) or f^2 / l^2 (Matern)
   int nw = 1, dw = 1, last_dw = 1;
   double inv_nw = 1.0;
};

inline KernelParams kernel_params_of(const KernelSpec& K, int d)
{
   KernelParams P;
   const double f = K.f, l = K.l;
   P.kernel = K.kernel ? 1 : 0;
   P.f2 = f * f;
   P.inv = (P.kernel == 0) ? 1.0 / (2.0 * l * l) : 1.0 / l;
   P.mu = K.mu;
   P.df_scale = 2.0 / f;
   P.dl_scale = (P.kernel == 0) ? P.f2 / (l * l * l) : P.f2 / (l * l);
   if (K.Xk) {
      P.nw = K.nw;
      P.dw = K.dw;
      P.last_dw = K.last_dw;
   } else {
      P.nw = 1;
      P.dw = P.last_dw = d;
   }
   P.inv_nw = 1.0 / P.nw;
   return P;
}

// K(x_a, x_b) and its three derivative entries (f, l, mu; fsai.c:530 dK_a); diag: a and b are one point
__device__ __forceinline__ void kern_pair(const KernelParams& P, const double* __restrict__ X, long long ldim, int a,
                                          int b, bool diag, double& K, double* dK)
{
   if (diag) {
      K = P.f2 + P.f2 * P.mu;
      dK[0] = P.df_scale * K;
      dK[1] = 0.0;
      dK[2] = P.f2;
      return;
   }
   double acc = 0.0, accl = 0.0;
   int c = 0;
   for (int w = 0; w < P.nw; w++) {
      const int dims = (w == P.nw - 1) ? P.last_dw : P.dw;
      double s = 0.0;
      for (int t = 0; t < dims; t++, c++) {
         const double df = X[(size_t)c * ldim + a] - X[(size_t)c * ldim + b];
         s = fma(df, df, s);
      }
      const double r = (P.kernel == 0) ? s : sqrt(s);
      const double e = exp(-r * P.inv);
      acc += e;
      accl = fma(r, e, accl);
   }
   K = P.f2 * acc * P.inv_nw;
   dK[0] = P.df_scale * K;
   dK[1] = P.dl_scale * accl * P.inv_nw;
   dK[2] = 0.0;
}

}  // namespace nfft4gp_amd
