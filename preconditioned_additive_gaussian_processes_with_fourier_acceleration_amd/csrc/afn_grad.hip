// afn_grad.hip -- the AFN preconditioner's gradient pieces for the GP loss (MATLAB afn_dvp.m, afn_trace.m,
// afn_logdet.m; the reference's C afn.c has none: Nfft4GPPrecondAFNTrace returns 0).
//
// The setup (afn_setup.hip, afn_setup_impl with gradients) keeps L, L^{-1}, L^{-T}, dL_g = L Phi(L^{-1}
// dK11_g L^{-T}), K12, dK12_g and the Schur FSAI G with dG_g.  afn_dvp.m forms (dM/dtheta_g) x for the
// AFN's M; the library's loss follows lanczos.c, whose func_dvp returns M^{-1} (dM/dtheta_g) x (as the
// reference's nys.c and fsai.c do), so the result goes through the AFN apply once more.  Every product is
// a device kernel: k x k matrix-vector products, the k x n2 panels K12 / dK12_g (a wave per column, or
// column-block partials with a fixed-order reduction), the FSAI's CSR products and level-scheduled
// triangular solves.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>

#include "callbacks.hpp"
#include "internal.h"

namespace nfft4gp_amd {

namespace {

constexpr int kT = 256;

// y = beta y + alpha A x, A k x k column-major (a thread per row: coalesced over the column)
__global__ __launch_bounds__(kT) void k_mv_n(const double* __restrict__ A, int k, const double* __restrict__ x,
                                             double* __restrict__ y, double alpha, double beta)
{
   const int i = blockIdx.x * kT + threadIdx.x;
   if (i >= k) return;
   double r = 0.0;
   for (int j = 0; j < k; j++) r = fma(A[i + (size_t)j * k], x[j], r);
   y[i] = (beta == 0.0 ? 0.0 : beta * y[i]) + alpha * r;
}

// y = beta y + alpha A^T x for A with `rows` rows (ld rows) and `cols` columns: one wave per column
__global__ __launch_bounds__(kT) void k_mv_t(const double* __restrict__ A, int rows, int cols,
                                             const double* __restrict__ x, double* __restrict__ y, double alpha,
                                             double beta)
{
   const int lane = threadIdx.x & 63;
   const long long j = (long long)blockIdx.x * (kT / 64) + (threadIdx.x >> 6);
   if (j >= cols) return;
   const double* col = A + j * rows;
   double r = 0.0;
   for (int i = lane; i < rows; i += 64) r = fma(col[i], x[i], r);
   for (int off = 32; off > 0; off >>= 1) r += __shfl_down(r, off, 64);
   if (lane == 0) y[j] = (beta == 0.0 ? 0.0 : beta * y[j]) + alpha * r;
}

// part[b][i] = sum_{j in block b} A[i + j k] x_j  (A k x n2); then y = beta y + alpha sum_b part[b]
constexpr int kPanelBlocks = 1024;
__global__ __launch_bounds__(kT) void k_pn_part(const double* __restrict__ A, int k, int n2, int cols,
                                                const double* __restrict__ x, double* __restrict__ part)
{
   const int j0 = blockIdx.x * cols, j1 = min(n2, j0 + cols);
   for (int i = threadIdx.x; i < k; i += kT) {
      double r = 0.0;
      for (int j = j0; j < j1; j++) r = fma(A[i + (size_t)j * k], x[j], r);
      part[(size_t)blockIdx.x * k + i] = r;
   }
}

__global__ __launch_bounds__(kT) void k_pn_reduce(const double* __restrict__ part, int nblk, int k,
                                                  double* __restrict__ y, double alpha, double beta)
{
   const int i = blockIdx.x * kT + threadIdx.x;
   if (i >= k) return;
   double r = 0.0;
   for (int b = 0; b < nblk; b++) r += part[(size_t)b * k + i];
   y[i] = (beta == 0.0 ? 0.0 : beta * y[i]) + alpha * r;
}

__global__ void k_axpby(int n, double a, const double* __restrict__ x, double b, double* __restrict__ y)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) y[i] = a * x[i] + (b == 0.0 ? 0.0 : b * y[i]);
}

__global__ void k_perm_gather(const double* __restrict__ src, const int* __restrict__ perm, int n,
                              double* __restrict__ dst)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) dst[i] = src[perm[i]];
}

__global__ void k_perm_scatter(const double* __restrict__ src, const int* __restrict__ perm, int n,
                               double* __restrict__ dst)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) dst[perm[i]] = src[i];
}

inline int g1(int n) { return std::max(1, (n + kT - 1) / kT); }

struct Ops {
   AfnGrad* G;
   hipStream_t s;
   double* part;
   int nblk, cols;
   void mv_n(const double* A, const double* x, double* y, double a = 1.0, double b = 0.0)
   {
      hipLaunchKernelGGL(k_mv_n, dim3(g1(G->k)), dim3(kT), 0, s, A, G->k, x, y, a, b);
   }
   void mv_t(const double* A, const double* x, double* y, double a = 1.0, double b = 0.0)
   {
      hipLaunchKernelGGL(k_mv_t, dim3((G->k + 3) / 4), dim3(kT), 0, s, A, G->k, G->k, x, y, a, b);
   }
   void panel_t(const double* A, const double* x, double* y, double a = 1.0, double b = 0.0)  // y (n2) = A^T x
   {
      hipLaunchKernelGGL(k_mv_t, dim3((G->n2 + 3) / 4), dim3(kT), 0, s, A, G->k, G->n2, x, y, a, b);
   }
   void panel_n(const double* A, const double* x, double* y, double a = 1.0, double b = 0.0)  // y (k) = A x
   {
      hipLaunchKernelGGL(k_pn_part, dim3(nblk), dim3(kT), 0, s, A, G->k, G->n2, cols, x, part);
      hipLaunchKernelGGL(k_pn_reduce, dim3(g1(G->k)), dim3(kT), 0, s, part, nblk, G->k, y, a, b);
   }
   void axpby(int n, double a, const double* x, double b, double* y)
   {
      hipLaunchKernelGGL(k_axpby, dim3(g1(n)), dim3(kT), 0, s, n, a, x, b, y);
   }
   int fsai(int op, int g, const double* x, double* y) { return fsai_grad_op(G->S, op, g, x, y, s); }
};

}  // namespace

void afn_grad_free(AfnGrad* G)
{
   if (!G) return;
   (void)hipStreamSynchronize(current_stream());
   for (void* p : {(void*)G->perm, (void*)G->L, (void*)G->Linv, (void*)G->LinvT, (void*)G->dL, (void*)G->dK12,
                   (void*)G->work})
      (void)hipFree(p);
   fsai_grad_free(G->S);
   delete G;
}

int afn_grad_dvp(AfnGrad* G, const int* mask, const double* x, double* y, hipStream_t s)
{
   const int n = G->n, k = G->k, n2 = G->n2;
   const size_t kk = (size_t)k * k, kn2 = (size_t)k * n2;
   Ops o{G, s, nullptr, 0, 0};
   if (!G->S || !G->afn) return -1;
   o.cols = std::max(16, (n2 + kPanelBlocks - 1) / kPanelBlocks);
   o.nblk = (n2 + o.cols - 1) / o.cols;
   // scratch: n-vectors P, YP, Z1L.., k-vectors; the panel partials after them
   double* w = G->work;
   double* P = w;                   // permuted x (n): xu = P, xl = P + k
   double* YP = P + n;              // permuted (dM/dtheta) x (n): yu = YP, yl = YP + k
   double* Z1L = YP + n;            // n2
   double* E = Z1L + n2;            // n2
   double* F = E + n2;              // n2
   double* R = F + n2;              // n2 (also z2l)
   double* kv = w + 6 * (size_t)n;  // k-vectors (2 n + 4 n2 <= 6 n before them)
   double *T1 = kv, *LT1 = kv + k, *Z1U = kv + 2 * k, *TZ = kv + 3 * k, *B1 = kv + 4 * k, *B2 = kv + 5 * k,
          *S1 = kv + 6 * k, *Z2U = kv + 7 * k;
   if (!o.part) {
      static double* part = nullptr;
      static size_t part_cap = 0;
      const size_t need = (size_t)o.nblk * k;
      if (need > part_cap) {
         (void)hipStreamSynchronize(s);
         (void)hipFree(part);
         NFFT4GP_HIP_CHECK(hipMalloc((void**)&part, sizeof(double) * need));
         part_cap = need;
      }
      o.part = part;
   }
   double* xu = P;
   double* xl = P + k;
   double* yu = YP;
   double* yl = YP + k;
   if (mask) NFFT4GP_HIP_CHECK(hipMemsetAsync(y, 0, sizeof(double) * 3 * (size_t)n, s));  // masked gradients: 0
   hipLaunchKernelGGL(k_perm_gather, dim3(g1(n)), dim3(kT), 0, s, x, G->perm, n, P);
   // afn_dvp.m, the parts shared by the gradients
   o.panel_n(G->K12, xl, T1);             // K12 xl
   o.mv_n(G->Linv, T1, LT1);              // L \ (K12 xl)
   o.mv_t(G->L, xu, Z1U);                 // z1u = L' xu + L \ (K12 xl)
   o.axpby(k, 1.0, LT1, 1.0, Z1U);
   if (o.fsai(3, 0, xl, Z1L)) return -1;  // z1l = G' \ xl
   if (o.fsai(2, 0, Z1L, E)) return -1;   // G \ z1l
   o.mv_n(G->LinvT, Z1U, TZ);             // L' \ z1u
   for (int g = 0; g < 3; g++) {
      if (mask && !mask[g]) continue;
      const double* dL = G->dL + g * kk;
      const double* dK12 = g < 2 ? G->dK12 + g * kn2 : nullptr;  // dK12_mu = 0
      // y1u = dL z1u;  y1l = dK12' t - K12' (L' \ (dL' t)) - G \ (dG (G \ z1l)),  t = L' \ z1u
      o.mv_n(dL, Z1U, yu);
      if (dK12)
         o.panel_t(dK12, TZ, yl);
      else
         (void)hipMemsetAsync(yl, 0, sizeof(double) * n2, s);
      o.mv_t(dL, TZ, B1);
      o.mv_n(G->LinvT, B1, B2);
      o.panel_t(G->K12, B2, yl, -1.0, 1.0);
      if (o.fsai(4, g, E, F) || o.fsai(2, 0, F, R)) return -1;
      o.axpby(n2, -1.0, R, 1.0, yl);
      // z2l = -G' \ (dG' (G' \ xl)) (G' \ xl = z1l);  y2ui = dK12 xl - dL (L \ (K12 xl));
      // z2u = dL' xu + L \ y2ui;  y2u = L z2u;  y2l = K12' (L' \ z2u) + G \ z2l
      if (o.fsai(5, g, Z1L, F) || o.fsai(3, 0, F, R)) return -1;  // R = -z2l
      if (dK12)
         o.panel_n(dK12, xl, S1);
      else
         (void)hipMemsetAsync(S1, 0, sizeof(double) * k, s);
      o.mv_n(dL, LT1, S1, -1.0, 1.0);
      o.mv_t(dL, xu, Z2U);
      o.mv_n(G->Linv, S1, Z2U, 1.0, 1.0);
      o.mv_n(G->L, Z2U, yu, 1.0, 1.0);
      o.mv_n(G->LinvT, Z2U, B1);
      o.panel_t(G->K12, B1, yl, 1.0, 1.0);
      if (o.fsai(2, 0, R, F)) return -1;  // G \ (-z2l)
      o.axpby(n2, -1.0, F, 1.0, yl);
      // unpermute (dM/dtheta_g) x, then the library's func_dvp convention: M^{-1} (dM/dtheta_g) x
      double* yg = y + (size_t)g * n;
      hipLaunchKernelGGL(k_perm_scatter, dim3(g1(n)), dim3(kT), 0, s, YP, G->perm, n, yg);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      if (Nfft4GPAmdAfnSolve(G->afn, n, yg, yg)) return -1;  // the apply gathers its rhs before writing x
   }
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

}  // namespace nfft4gp_amd
