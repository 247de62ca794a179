// nystrom.hip -- Nystrom ("RAN") preconditioner setup on the GPU.
//
// Restates Nfft4GPPrecondNysSetupWithKernel (SRC/preconds/nys.c:518-660) for the dense additive kernel
// of an additive handle's data / windows / hyperparameters (SRC/linearalg/kernels.c:3099-3494, Gaussian
// kernels.c:680-1289 and Matern-1/2 :2390-3033, "when have permc we do not add noise"):
//
//   Kp  = K(perm, perm[:k])                   n x k panel, rows in permuted order   (k_nys_panel, VALU)
//   K11 (see below), + sqrt(k) ulp(|K11|_F) I, L = chol(K11), G = L^{-1}     (host, k x k; chol.c:428-467)
//   U1  = Kp G^T                              (k_gemm_f64, MFMA; matops.c Nfft4GPTrilNystromMm)
//   AA  = U1^T U1 = V diag(w1) V^T            (k_gemm_f64 split over rows, MFMA; host eigensolve;
//                                              matops.c Nfft4GPTrilNystromSvd)
//   U   = U1 V(:, reversed) diag(1/sqrt(w1 reversed))   (k_gemm_f64, rows scattered to natural order)
//   s   = max(1/(w + eta), 0), eta = mu f^2   (nys.c:641-647)
//
// The three n x k x k products (6 n k^2 flops, 1.6 TFLOP at n = 1e6, k = 512) run on v_mfma_f64_16x16x4;
// the k x k Cholesky / inverse / eigensolve (O(k^3), ~0.1-0.5 s at k = 512) run on the host.
//
// K11: the reference builds it by calling the additive kernel on the k x d sub-data, but that kernel
// reads its own gathered buffer with the stride of the n it is given (kernels.c:3160), so its K11 is the
// kernel matrix of buffer slices, not of the landmarks perm[:k] (checked against the compiled reference
// to 1e-11).  k11_mode 0 reproduces that (parity); k11_mode 1 uses K(perm[:k], perm[:k]), the matrix the
// method intends, which is what makes the preconditioner effective.
#include <cstdlib>
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rocsolver/rocsolver.h>  // types and prototypes only: the library is dlopen'ed on first use

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "internal.h"

namespace nfft4gp_amd {

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));

// ---- panel: Kp[jj + ii*n] = (f^2/nw) sum_c kern(|xr_c[jj] - xc_c[ii]|), jj < n, ii < k ------------------
// xr: the rows' window coordinates (n x D, column t of window w at t = w*dw + dd, ld n), xc: the landmarks'
// (k x D, ld k).  The reference's panel rows are perm-ordered (nys.c:566-567); a natural-order panel gives
// the same U1^T U1 (a sum over rows) and lands U in natural row order directly, so the final product needs
// no row scatter and the apply reads U as stored.  A row shard passes its own rows as xr.
constexpr int kPanelRows = 64, kPanelCols = 64, kPanelThreads = 256;
constexpr int kPanelMaxDims = 128;  // window dimensions summed over all windows (nw * dw)

// GRAD: also the two hyperparameter derivatives of the noise-free panel (kernels.c:680-1289 Gaussian,
// :2390-3033 Matern-1/2, averaged over windows by kernels.c:3099-3494), written as blocks 2 and 3 at
// Kp + n k and Kp + 2 n k:  dK/df = (2/f) K,  dK/dl = (f^2/nw) sum_c r_c^2/l^3 e^{-r_c^2/2l^2} (Gaussian)
// or (f^2/nw) sum_c r_c/l^2 e^{-r_c/l} (Matern-1/2), over the first grad_nw windows: with a padded last
// window (skip_last > 0) the reference's rectangular K(permr, permc) adds the last window to K but not to
// dK (kernels.c:3169 passes NULL for its dK), while its square no-permutation matrix (the K11 of
// nys.c:569) keeps it (kernels.c:3398); grad_nw = nw - 1 reproduces the former.
template <int KERNEL, bool GRAD>  // KERNEL 0 Gaussian exp(-r^2 / 2l^2), 1 Matern-1/2 exp(-r / l)
__global__ __launch_bounds__(kPanelThreads) void k_nys_panel(const double* __restrict__ xr, int n, int nw, int dw,
                                                             int last_dw, const double* __restrict__ xc, int k,
                                                             double scale, double inv, double* __restrict__ Kp,
                                                             int grad_nw, double df_scale, double dl_scale)
{
   extern __shared__ double sm[];
   const int D = (nw - 1) * dw + last_dw;
   double* s_r = sm;                     // [D][kPanelRows]
   double* s_c = sm + D * kPanelRows;    // [D][kPanelCols]
   const int r0 = blockIdx.x * kPanelRows, c0 = blockIdx.y * kPanelCols;
   for (int e = threadIdx.x; e < D * kPanelRows; e += kPanelThreads) {
      const int t = e / kPanelRows, i = e % kPanelRows;
      const int w = min(t / dw, nw - 1), dd = t - w * dw;  // window w, its dimension dd
      const size_t col = (size_t)w * dw + dd;               // windows packed at stride n*dw (kernels.c:3160)
      s_r[e] = (r0 + i < n) ? xr[col * n + r0 + i] : 0.0;
      s_c[e] = (c0 + i < k) ? xc[col * k + c0 + i] : 0.0;
   }
   __syncthreads();
   // thread -> 4 rows x 4 columns, rows fastest so stores are coalesced per column
   const int tr = threadIdx.x & 15, tc = threadIdx.x >> 4;
   double acc[4][4] = {}, accf[4][4] = {}, accl[4][4] = {};
   for (int w = 0; w < nw; w++) {
      const int dims = (w == nw - 1) ? last_dw : dw;
      double r2[4][4] = {};
      for (int dd = 0; dd < dims; dd++) {
         const int t = w * dw + dd;
         double xr[4], xc[4];
#pragma unroll
         for (int a = 0; a < 4; a++) xr[a] = s_r[t * kPanelRows + tr + 16 * a];
#pragma unroll
         for (int b = 0; b < 4; b++) xc[b] = s_c[t * kPanelCols + tc + 16 * b];
#pragma unroll
         for (int a = 0; a < 4; a++)
#pragma unroll
            for (int b = 0; b < 4; b++) {
               const double df = xr[a] - xc[b];
               r2[a][b] = fma(df, df, r2[a][b]);
            }
      }
      const bool gw = GRAD && w < grad_nw;
#pragma unroll
      for (int a = 0; a < 4; a++)
#pragma unroll
         for (int b = 0; b < 4; b++) {
            const double r = (KERNEL == 0) ? r2[a][b] : sqrt(r2[a][b]);
            const double e = (KERNEL == 0) ? exp(-r * inv) : exp(-r * inv);
            acc[a][b] += e;
            if (gw) {
               accf[a][b] += e;
               accl[a][b] = fma(r, e, accl[a][b]);
            }
         }
   }
   const size_t blk = (size_t)n * k;
#pragma unroll
   for (int b = 0; b < 4; b++) {
      const int c = c0 + tc + 16 * b;
      if (c >= k) continue;
#pragma unroll
      for (int a = 0; a < 4; a++) {
         const int r = r0 + tr + 16 * a;
         if (r >= n) continue;
         Kp[(size_t)c * n + r] = scale * acc[a][b];
         if (GRAD) {
            Kp[blk + (size_t)c * n + r] = df_scale * accf[a][b];
            Kp[2 * blk + (size_t)c * n + r] = dl_scale * accl[a][b];
         }
      }
   }
}

// launch the panel variant for (kernel, grad)
void launch_panel(int kernel, bool grad, dim3 grid, size_t lds, hipStream_t s, const double* xr, int n, int nw, int dw,
                  int last_dw, const double* xc, int k, double f, double l, double* Kp, int grad_nw)
{
   const double f2nw = f * f / nw;
   const double inv = (kernel == 0) ? 1.0 / (2.0 * l * l) : 1.0 / l;
   const double df_scale = 2.0 / f * f2nw;
   const double dl_scale = (kernel == 0) ? f2nw / (l * l * l) : f2nw / (l * l);
#define NYS_PANEL(KK, GG)                                                                                        \
   hipLaunchKernelGGL((k_nys_panel<KK, GG>), grid, dim3(kPanelThreads), lds, s, xr, n, nw, dw, last_dw, xc, k, \
                      f2nw, inv, Kp, grad_nw, df_scale, dl_scale)
   if (kernel == 0) {
      if (grad) NYS_PANEL(0, true); else NYS_PANEL(0, false);
   } else {
      if (grad) NYS_PANEL(1, true); else NYS_PANEL(1, false);
   }
#undef NYS_PANEL
}

// ---- C = op(A) B on MFMA f64 ---------------------------------------------------------------------
// op(A) is M x K: A column-major (lda) or, with TRANSA, A^T of a column-major K x M array.  B is K x N
// column-major (ldb).  128 x 128 output tile per workgroup: 4 waves in 2 x 2, each 64 x 64 = 4 x 4
// blocks of v_mfma_f64_16x16x4_f64 (64 doubles of accumulator per lane).  K advances in steps of 16
// through a double-buffered LDS tile: step i's MFMAs read buffer i & 1 while step i + 1's global loads
// (issued before them) are in flight; their registers then go to the other buffer, one barrier per step.
// The MFMA operands are swapped (B feeds the A-operand slot) so a lane's accumulators hold 16 consecutive
// ROWS of C: every store instruction writes 4 full 128-B column segments of the column-major C instead of
// 16 scattered 32-B pieces.  Tile order: the N tiles of one M tile are consecutive and run on one XCD
// (workgroup id % 8), so the A rows they share are read from HBM once and then from that XCD's L2.
// ksplit < K splits K into chunks (tile order z-major); chunk z writes its partial product at
// C + z * split_stride (summed by k_sum_splits).  sym: C is symmetric (the Gram U^T U), only tiles with
// tile_n <= tile_m are computed (k_sum_splits mirrors the rest).  The accumulation order over K is the
// same as a single-buffered step loop: results do not depend on the tile order.
constexpr int kGemmTile = 128, kGemmK = 16, kGemmThreads = 256, kGemmPad = 1;
constexpr int kGemmLd = kGemmTile + kGemmPad;
constexpr size_t kGemmLds = sizeof(double) * 2 * 2 * kGemmK * kGemmLd;  // [buffer][A | B][kk][row]

template <bool TRANSA>
__global__ __launch_bounds__(kGemmThreads) void k_gemm_f64(int M, int N, int K, const double* __restrict__ A,
                                                           long long lda, const double* __restrict__ B,
                                                           long long ldb, double* __restrict__ C, long long ldc,
                                                           long long split_stride, int ksplit, int sym)
{
   extern __shared__ double g_smem[];
   const int mt = (M + kGemmTile - 1) / kGemmTile, nt = (N + kGemmTile - 1) / kGemmTile;
   const int nz = (K + ksplit - 1) / ksplit;
   const long long total = (long long)mt * nt * nz;
   const long long per = (total + 7) / 8;
   const long long tpos = (long long)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
   if (tpos >= total) return;
   const int zi = (int)(tpos / ((long long)mt * nt));
   const int rem = (int)(tpos % ((long long)mt * nt));
   const int tm = rem / nt, tn = rem % nt;
   if (sym && tn > tm) return;
   const int m0 = tm * kGemmTile, n0 = tn * kGemmTile;
   const int kbeg = zi * ksplit, kend = min(K, kbeg + ksplit);
   const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
   const int wm = (wave & 1) * 64, wn = (wave >> 1) * 64;
   constexpr int kPer = kGemmK * kGemmTile / kGemmThreads;  // 8 elements of each operand per thread
   constexpr int kBuf = 2 * kGemmK * kGemmLd;                // doubles per buffer (A then B)
   d4 acc[4][4];
#pragma unroll
   for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
   double av[kPer], bv[kPer];
   auto fetch = [&](int k0) {
#pragma unroll
      for (int u = 0; u < kPer; u++) {
         const int e = tid + u * kGemmThreads;
         int r, kk;
         if (!TRANSA) {
            r = e & (kGemmTile - 1);
            kk = e >> 7;
         } else {
            kk = e & (kGemmK - 1);
            r = e >> 4;
         }
         const int gr = m0 + r, gk = k0 + kk;
         av[u] = (gr < M && gk < kend) ? (TRANSA ? A[gk + (long long)gr * lda] : A[gr + (long long)gk * lda]) : 0.0;
         const int bk = e & (kGemmK - 1), bc = e >> 4;
         const int gbk = k0 + bk, gbc = n0 + bc;
         bv[u] = (gbk < kend && gbc < N) ? B[gbk + (long long)gbc * ldb] : 0.0;
      }
   };
   auto store = [&](double* buf) {
      double* As = buf;
      double* Bs = buf + kGemmK * kGemmLd;
#pragma unroll
      for (int u = 0; u < kPer; u++) {
         const int e = tid + u * kGemmThreads;
         if (!TRANSA)
            As[(e >> 7) * kGemmLd + (e & (kGemmTile - 1))] = av[u];
         else
            As[(e & (kGemmK - 1)) * kGemmLd + (e >> 4)] = av[u];
         Bs[(e & (kGemmK - 1)) * kGemmLd + (e >> 4)] = bv[u];
      }
   };
   fetch(kbeg);
   store(g_smem);
   __syncthreads();
   int cur = 0;
   for (int k0 = kbeg; k0 < kend; k0 += kGemmK) {
      const bool more = k0 + kGemmK < kend;
      if (more) fetch(k0 + kGemmK);  // in flight during this step's MFMAs
      const double* As = g_smem + cur * kBuf;
      const double* Bs = As + kGemmK * kGemmLd;
#pragma unroll
      for (int k4 = 0; k4 < kGemmK / 4; k4++) {
         const int kk = 4 * k4 + (lane >> 4);
         double a[4], b[4];
#pragma unroll
         for (int i = 0; i < 4; i++) a[i] = As[kk * kGemmLd + wm + 16 * i + (lane & 15)];
#pragma unroll
         for (int j = 0; j < 4; j++) b[j] = Bs[kk * kGemmLd + wn + 16 * j + (lane & 15)];
#pragma unroll
         for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < 4; j++) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(b[j], a[i], acc[i][j], 0, 0, 0);
      }
      if (more) store(g_smem + (cur ^ 1) * kBuf);  // the other buffer: nobody reads it during this step
      __syncthreads();
      cur ^= 1;
   }
   // D map of v_mfma_f64_16x16x4_f64: D col = lane & 15 (B-operand index = row of C here),
   // D row = (lane >> 4) + 4 * reg (A-operand index = column of C here)
   double* Cz = C + (size_t)zi * split_stride;
#pragma unroll
   for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
         for (int rg = 0; rg < 4; rg++) {
            const int gr = m0 + wm + 16 * i + (lane & 15);
            const int gc = n0 + wn + 16 * j + (lane >> 4) + 4 * rg;
            if (gr < M && gc < N) Cz[gr + (long long)gc * ldc] = acc[i][j][rg];
         }
}

// the launch grid of k_gemm_f64: one workgroup per (M tile, N tile, K chunk), rounded up to a multiple of 8
static unsigned gemm_blocks(int M, int N, int K, int ksplit)
{
   const long long total = (long long)((M + kGemmTile - 1) / kGemmTile) * ((N + kGemmTile - 1) / kGemmTile) *
                           ((K + ksplit - 1) / ksplit);
   return (unsigned)(((total + 7) / 8) * 8);
}

static void gemm_attr_once()
{
   static const bool done = []() {
      for (const void* f : {(const void*)k_gemm_f64<false>, (const void*)k_gemm_f64<true>})
         (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kGemmLds);
      (void)hipGetLastError();
      return true;
   }();
   (void)done;
}

// C[i] = sum_z part[z * stride + i] in z order.  sym (square C of order ld): elements of tiles above the
// tile diagonal were not computed and are read from the transposed position.
__global__ void k_sum_splits(const double* __restrict__ part, int nsplit, long long stride, long long count,
                             double* __restrict__ C, int sym, int ld)
{
   const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
   if (i >= count) return;
   long long src = i;
   if (sym) {
      const long long r = i % ld, c = i / ld;
      if (c / kGemmTile > r / kGemmTile) src = c + r * ld;
   }
   double v = 0.0;
   for (int z = 0; z < nsplit; z++) v += part[z * stride + src];
   C[i] = v;
}

int gemm(bool transA, int M, int N, int K, const double* A, long long lda, const double* B, long long ldb, double* C,
         long long ldc, hipStream_t s)
{
   if (M <= 0 || N <= 0) return 0;
   gemm_attr_once();
   const int ks = std::max(K, 1);
   const dim3 grid(gemm_blocks(M, N, ks, ks));
   if (transA)
      hipLaunchKernelGGL(k_gemm_f64<true>, grid, dim3(kGemmThreads), kGemmLds, s, M, N, K, A, lda, B, ldb, C, ldc, 0LL,
                         ks, 0);
   else
      hipLaunchKernelGGL(k_gemm_f64<false>, grid, dim3(kGemmThreads), kGemmLds, s, M, N, K, A, lda, B, ldb, C, ldc, 0LL,
                         ks, 0);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

// ---- host k x k linear algebra (column-major, k <= a few thousand) --------------------------------
// lower Cholesky in place (LAPACK dpotrf 'L' semantics); returns 0 or the failing column + 1
int chol_lower(std::vector<double>& a, int k)
{
   for (int j = 0; j < k; j++) {
      double d = a[j + (size_t)j * k];
      for (int p = 0; p < j; p++) d -= a[j + (size_t)p * k] * a[j + (size_t)p * k];
      if (!(d > 0.0)) return j + 1;
      d = std::sqrt(d);
      a[j + (size_t)j * k] = d;
      for (int i = j + 1; i < k; i++) {
         double v = a[i + (size_t)j * k];
         for (int p = 0; p < j; p++) v -= a[i + (size_t)p * k] * a[j + (size_t)p * k];
         a[i + (size_t)j * k] = v / d;
      }
   }
   for (int j = 0; j < k; j++)
      for (int i = 0; i < j; i++) a[i + (size_t)j * k] = 0.0;
   return 0;
}

// inverse of a lower-triangular matrix in place (dtrtri 'L' 'N')
void trtri_lower(std::vector<double>& L, int k)
{
   std::vector<double> G((size_t)k * k, 0.0);
   for (int j = 0; j < k; j++) {
      G[j + (size_t)j * k] = 1.0 / L[j + (size_t)j * k];
      for (int i = j + 1; i < k; i++) {
         double v = 0.0;
         for (int m = j; m < i; m++) v += L[i + (size_t)m * k] * G[m + (size_t)j * k];
         G[i + (size_t)j * k] = -v / L[i + (size_t)i * k];
      }
   }
   L.swap(G);
}

// symmetric eigensolve (dsyev 'V' semantics: ascending w, orthonormal eigenvectors as columns of V):
// Householder tridiagonalisation, then implicit-shift QL with the transformations accumulated
int sym_eig(const std::vector<double>& A, int n, std::vector<double>& w, std::vector<double>& V)
{
   std::vector<double> a(A);  // a[i + j*n] = a(i, j); symmetric, so a(i, j) = a[i*n + j] too
   auto at = [&](int i, int j) -> double& { return a[(size_t)i * n + j]; };
   std::vector<double> d(n), e(n);
   for (int i = n - 1; i > 0; i--) {
      const int l = i - 1;
      double h = 0.0, scale = 0.0;
      if (l > 0) {
         for (int kk = 0; kk <= l; kk++) scale += std::fabs(at(i, kk));
         if (scale == 0.0) {
            e[i] = at(i, l);
         } else {
            for (int kk = 0; kk <= l; kk++) {
               at(i, kk) /= scale;
               h += at(i, kk) * at(i, kk);
            }
            double f = at(i, l);
            double g = (f >= 0.0) ? -std::sqrt(h) : std::sqrt(h);
            e[i] = scale * g;
            h -= f * g;
            at(i, l) = f - g;
            f = 0.0;
            for (int j = 0; j <= l; j++) {
               at(j, i) = at(i, j) / h;
               g = 0.0;
               for (int kk = 0; kk <= j; kk++) g += at(j, kk) * at(i, kk);
               for (int kk = j + 1; kk <= l; kk++) g += at(kk, j) * at(i, kk);
               e[j] = g / h;
               f += e[j] * at(i, j);
            }
            const double hh = f / (h + h);
            for (int j = 0; j <= l; j++) {
               f = at(i, j);
               e[j] = g = e[j] - hh * f;
               for (int kk = 0; kk <= j; kk++) at(j, kk) -= (f * e[kk] + g * at(i, kk));
            }
         }
      } else {
         e[i] = at(i, l);
      }
      d[i] = h;
   }
   d[0] = 0.0;
   e[0] = 0.0;
   for (int i = 0; i < n; i++) {
      const int l = i - 1;
      if (d[i] != 0.0) {
         for (int j = 0; j <= l; j++) {
            double g = 0.0;
            for (int kk = 0; kk <= l; kk++) g += at(i, kk) * at(kk, j);
            for (int kk = 0; kk <= l; kk++) at(kk, j) -= g * at(kk, i);
         }
      }
      d[i] = at(i, i);
      at(i, i) = 1.0;
      for (int j = 0; j <= l; j++) at(j, i) = at(i, j) = 0.0;
   }
   // z^T (rows = eigenvector slots) so the QL rotations touch contiguous memory
   std::vector<double> zt((size_t)n * n);
   for (int i = 0; i < n; i++)
      for (int kk = 0; kk < n; kk++) zt[(size_t)i * n + kk] = at(kk, i);
   for (int i = 1; i < n; i++) e[i - 1] = e[i];
   if (n > 0) e[n - 1] = 0.0;
   for (int l = 0; l < n; l++) {
      int iter = 0, m;
      do {
         for (m = l; m < n - 1; m++) {
            const double dd = std::fabs(d[m]) + std::fabs(d[m + 1]);
            if (std::fabs(e[m]) <= DBL_EPSILON * dd) break;
         }
         if (m != l) {
            if (iter++ == 200) return -1;
            double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
            double r = std::hypot(g, 1.0);
            g = d[m] - d[l] + e[l] / (g + std::copysign(r, g));
            double s = 1.0, c = 1.0, p = 0.0;
            int i;
            for (i = m - 1; i >= l; i--) {
               double f = s * e[i];
               const double b = c * e[i];
               e[i + 1] = (r = std::hypot(f, g));
               if (r == 0.0) {
                  d[i + 1] -= p;
                  e[m] = 0.0;
                  break;
               }
               s = f / r;
               c = g / r;
               g = d[i + 1] - p;
               r = (d[i] - g) * s + 2.0 * c * b;
               d[i + 1] = g + (p = s * r);
               g = c * r - b;
               double* z0 = zt.data() + (size_t)i * n;
               double* z1 = zt.data() + (size_t)(i + 1) * n;
               for (int kk = 0; kk < n; kk++) {
                  f = z1[kk];
                  z1[kk] = s * z0[kk] + c * f;
                  z0[kk] = c * z0[kk] - s * f;
               }
            }
            if (r == 0.0 && i >= l) continue;
            d[l] -= p;
            e[l] = g;
            e[m] = 0.0;
         }
      } while (m != l);
   }
   std::vector<int> order(n);
   for (int i = 0; i < n; i++) order[i] = i;
   std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return d[x] < d[y]; });
   w.resize(n);
   V.assign((size_t)n * n, 0.0);
   for (int c = 0; c < n; c++) {
      w[c] = d[order[c]];
      memcpy(V.data() + (size_t)c * n, zt.data() + (size_t)order[c] * n, sizeof(double) * n);
   }
   return 0;
}

// ---- k x k helpers on the device -------------------------------------------------------------------
__global__ void k_add_diag(double* A, int k, double nu)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < k) A[i + (size_t)i * k] += nu;
}

// G = lower part of A (strict upper zeroed)
__global__ void k_clean_lower(const double* __restrict__ A, int k, double* __restrict__ G)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
   if (i < k) G[i + (size_t)j * k] = (i >= j) ? A[i + (size_t)j * k] : 0.0;
}

// Gt = (lower part of G)^T
__global__ void k_transpose_lower(const double* __restrict__ G, int k, double* __restrict__ Gt)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
   if (i < k) Gt[i + (size_t)j * k] = (j >= i) ? G[j + (size_t)i * k] : 0.0;
}

// W[:, c] = V[:, k-1-c] / sqrt(w1[k-1-c]) (x 1e12 when sqrt(w1) < 1e-12), s[c] = max(1/(w^2 + eta), 0)
// (matops.c Nfft4GPTrilNystromSvd, nys.c:641-647; NFFT4GP_MAX maps NaN to 0)
// robust (k11_mode 1): eigenvalues of U1'U1 at rounding level (<= k eps max w1, or negative from
// rounding, where the reference's sqrt gives NaN factors) drop their column instead
__global__ void k_nys_scale(const double* __restrict__ V, const double* __restrict__ w1, int k, double eta,
                            double* __restrict__ W, double* __restrict__ s, int robust)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x, c = blockIdx.y;
   const int src = k - 1 - c;
   if (robust && !(w1[src] > (double)k * 2.220446049250313e-16 * w1[k - 1])) {
      if (i < k) W[i + (size_t)c * k] = 0.0;
      if (i == 0) s[c] = 0.0;
      return;
   }
   const double wi = sqrt(w1[src]);
   if (i < k) W[i + (size_t)c * k] = V[i + (size_t)src * k] * ((wi < 1e-12) ? 1e12 : 1.0 / wi);
   if (i == 0) {
      const double v = 1.0 / (wi * wi + eta);
      s[c] = (v >= 0.0) ? v : 0.0;
   }
}

// rocSOLVER (dpotrf / dtrtri / dsyevd) loaded on first use: with PyTorch in the process it binds to the
// copy PyTorch already loaded (one ROCm runtime per process); without it, to /opt/rocm.  If it cannot be
// loaded the k x k steps run on the host instead (NFFT4GP_AMD_NO_ROCSOLVER=1 forces that).
struct RocSolver {
   bool ok = false;
   rocblas_handle h = nullptr;
   decltype(&rocblas_set_stream) set_stream = nullptr;
   decltype(&rocsolver_dpotrf) potrf = nullptr;
   decltype(&rocsolver_dtrtri) trtri = nullptr;
   decltype(&rocsolver_dsyevd) syevd = nullptr;
};

// first loadable of the given names, or nullptr with the dlerror of each attempt appended to `why`.  The
// versioned sonames come first: they match a copy already mapped into the process (PyTorch's bundled
// rocBLAS / rocSOLVER carry the sonames librocblas.so.5 / librocsolver.so.0), so the process keeps one copy
void* dlopen_first(const char* const* names, std::string& why)
{
   for (const char* const* p = names; *p; ++p) {
      if (void* h = dlopen(*p, RTLD_NOW | RTLD_GLOBAL)) return h;
      const char* e = dlerror();
      why += std::string("\n  ") + (e ? e : *p);
   }
   return nullptr;
}

RocSolver& rocsolver()
{
   static RocSolver R;
   static bool tried = false;
   if (tried) return R;
   tried = true;
   if (getenv("NFFT4GP_AMD_NO_ROCSOLVER") && atoi(getenv("NFFT4GP_AMD_NO_ROCSOLVER")) > 0) {
      fprintf(stderr, "nfft4gp_amd: NFFT4GP_AMD_NO_ROCSOLVER set: k x k Cholesky / inverse / eigensolves run on "
                      "the host.\n");
      return R;
   }
   static const char* const blas_names[] = {"librocblas.so.5", "librocblas.so.4", "librocblas.so",
                                            "/opt/rocm/lib/librocblas.so.5", "/opt/rocm/lib/librocblas.so", nullptr};
   static const char* const solver_names[] = {"librocsolver.so.0", "librocsolver.so",
                                              "/opt/rocm/lib/librocsolver.so.0", "/opt/rocm/lib/librocsolver.so",
                                              nullptr};
   std::string why;
   // rocBLAS / rocSOLVER draw libc rand() while they initialise (measured: the first rank estimation after an
   // srand() then picked other subsamples than the second).  The reference's draws (Nfft4GPRandPerm,
   // rankest.c) must see the caller's sequence, so the loading, the handle and one warm-up call of each
   // routine run on a private random() state (initstate / setstate: rand() is random() in glibc).
   static char priv_state[256];
   char* caller_state = initstate(20240807u, priv_state, sizeof(priv_state));
   struct Restore {
      char* s;
      ~Restore() { setstate(s); }
   } restore{caller_state};
   void* hb = dlopen_first(blas_names, why);
   void* hs = hb ? dlopen_first(solver_names, why) : nullptr;
   auto create = hb ? (decltype(&rocblas_create_handle))dlsym(hb, "rocblas_create_handle") : nullptr;
   if (hb && hs) {
      R.set_stream = (decltype(&rocblas_set_stream))dlsym(hb, "rocblas_set_stream");
      R.potrf = (decltype(&rocsolver_dpotrf))dlsym(hs, "rocsolver_dpotrf");
      R.trtri = (decltype(&rocsolver_dtrtri))dlsym(hs, "rocsolver_dtrtri");
      R.syevd = (decltype(&rocsolver_dsyevd))dlsym(hs, "rocsolver_dsyevd");
      if (!create || !R.set_stream || !R.potrf || !R.trtri || !R.syevd)
         why += "\n  a rocBLAS / rocSOLVER entry point is missing";
      else if (create(&R.h) != rocblas_status_success)
         why += "\n  rocblas_create_handle failed";
      else
         R.ok = true;
   }
   if (R.ok) {
      // first calls initialise the libraries' internals (inside the private random() state)
      double* A = nullptr;
      int* info = nullptr;
      if (hipMalloc((void**)&A, sizeof(double) * 8) == hipSuccess && hipMalloc((void**)&info, sizeof(int)) == hipSuccess) {
         const double one[4] = {1.0, 0.0, 0.0, 1.0};
         (void)hipMemcpy(A, one, sizeof(one), hipMemcpyHostToDevice);
         (void)R.potrf(R.h, rocblas_fill_lower, 2, A, 2, info);
         (void)R.trtri(R.h, rocblas_fill_lower, rocblas_diagonal_non_unit, 2, A, 2, info);
         (void)hipMemcpy(A, one, sizeof(one), hipMemcpyHostToDevice);
         (void)R.syevd(R.h, rocblas_evect_none, rocblas_fill_lower, 2, A, 2, A + 4, A + 6, info);
         (void)hipDeviceSynchronize();
      }
      (void)hipFree(A);
      (void)hipFree(info);
   }
   if (!R.ok)
      fprintf(stderr, "nfft4gp_amd: rocSOLVER could not be loaded; k x k Cholesky / inverse / eigensolves run on "
                      "the host (slower, same results to rounding):%s\n", why.c_str());
   return R;
}

template <class T>
int dalloc(T** p, size_t count)
{
   NFFT4GP_HIP_CHECK(hipMalloc((void**)p, sizeof(T) * std::max<size_t>(1, count)));
   return 0;
}

}  // namespace

int gemm_f64(bool transA, int M, int N, int K, const double* A, long long lda, const double* B, long long ldb,
             double* C, long long ldc, hipStream_t s)
{
   return gemm(transA, M, N, K, A, lda, B, ldb, C, ldc, s);
}

int sym_eig_host(const std::vector<double>& A, int n, std::vector<double>& w, std::vector<double>& V)
{
   return sym_eig(A, n, w, V);
}

// eigenvalues (ascending) of the symmetric n x n device matrix A (lower triangle read, A overwritten):
// rocSOLVER dsyevd without vectors; the host tridiagonal QL when rocSOLVER did not load
int sym_eigvals_dev(double* A, int n, std::vector<double>& w, hipStream_t s)
{
   w.assign(n, 0.0);
   RocSolver& R = rocsolver();
   if (R.ok) {
      double *d_w = nullptr, *d_e = nullptr;
      int* d_info = nullptr;
      int info = 0;
      int rc = -1;
      if (dalloc(&d_w, n) == 0 && dalloc(&d_e, n) == 0 && dalloc(&d_info, 1) == 0) {
         R.set_stream(R.h, s);
         if (R.syevd(R.h, rocblas_evect_none, rocblas_fill_lower, n, A, n, d_w, d_e, d_info) == rocblas_status_success &&
             hipMemcpyAsync(w.data(), d_w, sizeof(double) * n, hipMemcpyDeviceToHost, s) == hipSuccess &&
             hipMemcpyAsync(&info, d_info, sizeof(int), hipMemcpyDeviceToHost, s) == hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess)
            rc = info ? -1 : 0;
      }
      (void)hipFree(d_w);
      (void)hipFree(d_e);
      (void)hipFree(d_info);
      return rc;
   }
   std::vector<double> h((size_t)n * n), V;
   if (hipMemcpyAsync(h.data(), A, sizeof(double) * h.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
       hipStreamSynchronize(s) != hipSuccess)
      return -1;
   for (int j = 0; j < n; j++)
      for (int i = 0; i < j; i++) h[i + (size_t)j * n] = h[j + (size_t)i * n];
   return sym_eig(h, n, w, V);
}

// L^{-1} of chol(A) (lower) in place; returns 0 or the failing column + 1
int chol_inverse_host(std::vector<double>& A, int k)
{
   if (int info = chol_lower(A, k)) return info;
   trtri_lower(A, k);
   return 0;
}

// G = L^{-1} (clean lower triangle) and Gt = G^T of L = chol(A + shift I), A k x k on the device (A is
// overwritten).  rocSOLVER potrf + trtri when it loaded, the host Cholesky otherwise.  Returns 0, the
// failing column + 1 when A + shift is not positive definite, or -1.
int chol_inverse_dev(double* A, int k, double shift, double* G, double* Gt, int* d_info, hipStream_t s)
{
   RocSolver& R = rocsolver();
   if (R.ok) {
      int info = 0;
      R.set_stream(R.h, s);
      if (shift != 0.0) hipLaunchKernelGGL(k_add_diag, dim3((k + 255) / 256), dim3(256), 0, s, A, k, shift);
      if (R.potrf(R.h, rocblas_fill_lower, k, A, k, d_info) != rocblas_status_success ||
          hipMemcpyAsync(&info, d_info, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
         return -1;
      if (info) return info;
      if (R.trtri(R.h, rocblas_fill_lower, rocblas_diagonal_non_unit, k, A, k, d_info) != rocblas_status_success)
         return -1;
      hipLaunchKernelGGL(k_transpose_lower, dim3((k + 255) / 256, k), dim3(256), 0, s, A, k, Gt);
      if (G) hipLaunchKernelGGL(k_clean_lower, dim3((k + 255) / 256, k), dim3(256), 0, s, A, k, G);
      return hipGetLastError() == hipSuccess ? 0 : -1;
   }
   std::vector<double> h((size_t)k * k);
   if (hipMemcpyAsync(h.data(), A, sizeof(double) * h.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
       hipStreamSynchronize(s) != hipSuccess)
      return -1;
   for (int j = 0; j < k; j++) h[j + (size_t)j * k] += shift;
   if (int info = chol_lower(h, k)) return info;
   trtri_lower(h, k);
   std::vector<double> ht((size_t)k * k);
   for (int j = 0; j < k; j++)
      for (int i = 0; i < k; i++) {
         ht[i + (size_t)j * k] = (j >= i) ? h[j + (size_t)i * k] : 0.0;
         if (i < j) h[i + (size_t)j * k] = 0.0;
      }
   if (hipMemcpy(Gt, ht.data(), sizeof(double) * ht.size(), hipMemcpyHostToDevice)) return -1;
   if (G && hipMemcpy(G, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice)) return -1;
   return 0;
}

__global__ void k_zero_upper(double* A, int k)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
   if (i < j && i < k) A[i + (size_t)j * k] = 0.0;
}

int chol_factor_dev(double* A, int k, int* d_info, hipStream_t s)
{
   RocSolver& R = rocsolver();
   if (R.ok) {
      int info = 0;
      R.set_stream(R.h, s);
      if (R.potrf(R.h, rocblas_fill_lower, k, A, k, d_info) != rocblas_status_success ||
          hipMemcpyAsync(&info, d_info, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
         return -1;
      if (info) return info;
      hipLaunchKernelGGL(k_zero_upper, dim3((k + 255) / 256, k), dim3(256), 0, s, A, k);
      return hipGetLastError() == hipSuccess ? 0 : -1;
   }
   std::vector<double> h((size_t)k * k);
   if (hipMemcpyAsync(h.data(), A, sizeof(double) * h.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
       hipStreamSynchronize(s) != hipSuccess)
      return -1;
   if (int info = chol_lower(h, k)) return info;
   for (int j = 0; j < k; j++)
      for (int i = 0; i < j; i++) h[i + (size_t)j * k] = 0.0;
   return hipMemcpy(A, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}

// C (M x N, ld ldc) = A^T B with A K x M (lda) and B K x N (ldb), K split over row chunks (fixed-order sum,
// deterministic); sym: C symmetric with A == B (only tiles on and below the diagonal are computed)
int gram_tn(int M, int N, int K, const double* A, long long lda, const double* B, long long ldb, double* C, int sym,
            hipStream_t s)
{
   const int nsplit = std::max(1, std::min(256, K / 8192));
   const int ksplit = ((K + nsplit - 1) / nsplit + kGemmK - 1) / kGemmK * kGemmK;
   const int nsplit_used = (K + ksplit - 1) / ksplit;
   double* part = nullptr;
   if (dalloc(&part, (size_t)nsplit_used * M * N)) return -1;
   gemm_attr_once();
   const dim3 grid(gemm_blocks(M, N, K, ksplit));
   hipLaunchKernelGGL(k_gemm_f64<true>, grid, dim3(kGemmThreads), kGemmLds, s, M, N, K, A, lda, B, ldb, part,
                      (long long)M, (long long)M * N, ksplit, sym);
   const long long cnt = (long long)M * N;
   hipLaunchKernelGGL(k_sum_splits, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, part, nsplit_used, cnt, cnt,
                      C, sym, M);
   const bool ok = hipGetLastError() == hipSuccess;
   (void)hipStreamSynchronize(s);
   (void)hipFree(part);
   return ok ? 0 : -1;
}

// ------------------------------------------------------------------------------------------------
// rank 0's count doubles at d on every rank (the others contribute zeros to the sum)
static int bcast_root(Comm* comm, double* d, size_t count, hipStream_t s)
{
   if (comm->rank != 0) NFFT4GP_HIP_CHECK(hipMemsetAsync(d, 0, sizeof(double) * count, s));
   return comm->allreduce(d, count, s);
}

// Row shards (shard != nullptr): the collectives below (the L^{-T} broadcast, the Gram all-reduce, the
// eigenbasis broadcast) are entered by every rank in the same order.  A rank-local failure between them
// (an allocation, an upload, a rocSOLVER error) returns on that rank only, and the other ranks then wait in
// their next collective: under a communicator any setup error is fatal to the whole group, and the caller
// must tear the group down (the replicated steps -- K11, its Cholesky -- fail on every rank
// alike).
NysDev* nys_setup_additive(const double* xw_host, int n, int nw, int dw, int skip_last, int kernel, double f,
                           double l, double mu, const int* perm, int k, int k11_mode, bool with_grad,
                           const NysShard* shard)
{
   // the gathered buffer holds n_all rows per window column; this setup's rows are [rb, rb + n)
   const int n_all = shard ? shard->n_global : n;
   const int rb = shard ? shard->row_begin : 0;
   Comm* comm = shard ? shard->comm : nullptr;
   const int last_dw = dw - skip_last;
   const int D = (nw - 1) * dw + last_dw;
   // NFFT4GP_AMD_VERBOSE=1: per-phase wall times on stderr
   const bool verbose = getenv("NFFT4GP_AMD_VERBOSE") && atoi(getenv("NFFT4GP_AMD_VERBOSE")) > 0;
   auto tic = std::chrono::steady_clock::now();
   auto phase = [&](const char* name) {
      if (!verbose) return;
      (void)hipStreamSynchronize(current_stream());
      const auto now = std::chrono::steady_clock::now();
      fprintf(stderr, "nfft4gp_amd: nystrom %-10s %8.3f ms\n", name,
              std::chrono::duration<double, std::milli>(now - tic).count());
      tic = now;
   };
   if (k <= 0 || k > n_all || D > kPanelMaxDims || last_dw <= 0 || (shard && (with_grad || !comm))) {
      fprintf(stderr, "nfft4gp_amd: Nystrom setup needs 0 < k <= n, <= %d window dimensions (and no gradients on "
                      "row shards)\n", kPanelMaxDims);
      return nullptr;
   }
   hipStream_t s = current_stream();
   const int nblk = with_grad ? 3 : 1;  // panel blocks: K (and dK/df, dK/dl)
   double *d_xw = nullptr, *d_xk = nullptr, *d_x11 = nullptr, *d_Kp = nullptr, *d_U1 = nullptr, *d_B = nullptr, *d_AA = nullptr;
   double *d_K11 = nullptr, *d_w1 = nullptr, *d_e = nullptr, *d_s = nullptr, *d_T = nullptr;
   int* d_info = nullptr;
   NysDev* N = new NysDev();
   N->n = n;
   N->k = k;
   auto release = [&]() {
      for (double* p : {d_xw, d_xk, d_x11, d_Kp, d_U1, d_B, d_AA, d_K11, d_w1, d_e, d_s, d_T}) (void)hipFree(p);
      (void)hipFree(d_info);
   };
   auto fail = [&](const char* what) -> NysDev* {
      if (what) fprintf(stderr, "nfft4gp_amd: Nystrom setup: %s\n", what);
      (void)hipStreamSynchronize(s);
      release();
      nys_free(N);
      return nullptr;
   };
   // hipEvents around the four big kernels (panel, gemm1, gram, gemm2) for the MFMA report
   hipEvent_t ev[8];
   for (auto& e : ev) (void)hipEventCreate(&e);
   struct EvGuard {
      hipEvent_t* e;
      ~EvGuard()
      {
         for (int i = 0; i < 8; i++) (void)hipEventDestroy(e[i]);
      }
   } ev_guard{ev};
   const size_t nk = (size_t)n * k, kk = (size_t)k * k;
   if (dalloc(&d_xw, (size_t)n * D) || dalloc(&d_xk, (size_t)k * D) || dalloc(&d_x11, (size_t)k * D) ||
       dalloc(&d_info, 1) ||
       dalloc(&d_Kp, nk * nblk) || dalloc(&d_U1, nk) || dalloc(&d_B, kk) || dalloc(&d_AA, kk))
      return fail("allocation");
   // this setup's rows (n x D, ld n), the landmarks perm[:k] (k x D, ld k) and the K11 points: the
   // landmarks (mode 1), or the reference's K11 rows (mode 0: nys.c:569 hands the k x d sub-data to
   // Nfft4GPKernelAdditiveKernel, which ignores it and reads window i of its own gathered buffer at offset
   // i*n*dwindows with n = k, kernels.c:3160 -- the columns of a buffer of k rows: column t of that buffer
   // starts at t*k of ours)
   {
      std::vector<double> xk((size_t)k * D), x11((size_t)k * D);
      for (int t = 0; t < D; t++)
         for (int a = 0; a < k; a++) {
            xk[(size_t)t * k + a] = xw_host[(size_t)t * n_all + perm[a]];
            x11[(size_t)t * k + a] = k11_mode == 1 ? xk[(size_t)t * k + a] : xw_host[(size_t)t * k + a];
         }
      if ((n > 0 && hipMemcpy2D(d_xw, sizeof(double) * n, xw_host + rb, sizeof(double) * n_all, sizeof(double) * n, D,
                                hipMemcpyHostToDevice)) ||
          hipMemcpy(d_xk, xk.data(), sizeof(double) * xk.size(), hipMemcpyHostToDevice) ||
          hipMemcpy(d_x11, x11.data(), sizeof(double) * x11.size(), hipMemcpyHostToDevice))
         return fail("upload");
   }

   // 1. panel K(perm, perm[:k]) (noise-free, nys.c:566-567 / kernels.c "when have permc"), rows in natural
   //    order; with gradients also dK/df and dK/dl (nys.c:597-601)
   const double f2 = f * f;
   const int nw_grad_panel = (k11_mode == 0 && skip_last > 0) ? nw - 1 : nw;
   const size_t lds = sizeof(double) * (size_t)D * (kPanelRows + kPanelCols);
   dim3 pgrid((n + kPanelRows - 1) / kPanelRows, (k + kPanelCols - 1) / kPanelCols);
   (void)hipEventRecord(ev[0], s);
   if (n > 0)
      launch_panel(kernel, with_grad, pgrid, lds, s, d_xw, n, nw, dw, last_dw, d_xk, k, f, l, d_Kp, nw_grad_panel);
   if (hipGetLastError() != hipSuccess) return fail("panel launch");
   (void)hipEventRecord(ev[1], s);

   phase("panel");
   // 2. K11 (and dK11) on the device: the panel kernel on the K11 points against themselves (mode 1: the
   //    landmark rows of the whole panel, entry for entry the same arithmetic; mode 0: the reference's
   //    buffer rows, all windows in dK11, kernels.c:3398)
   if (dalloc(&d_K11, kk * nblk)) return fail("allocation");
   {
      dim3 kgrid((k + kPanelRows - 1) / kPanelRows, (k + kPanelCols - 1) / kPanelCols);
      launch_panel(kernel, with_grad, kgrid, lds, s, d_x11, k, nw, dw, last_dw, d_x11, k, f, l, d_K11,
                   k11_mode == 1 ? nw_grad_panel : nw);
   }
   // stable shift nu = sqrt(k) ulp(|K11|_F) (chol.c:449-465; dlansy 'F' 'L' = the full-matrix norm)
   std::vector<double> K11(kk);
   if (hipMemcpyAsync(K11.data(), d_K11, sizeof(double) * kk, hipMemcpyDeviceToHost, s) != hipSuccess ||
       hipStreamSynchronize(s) != hipSuccess)
      return fail("K11 download");
   double fro = 0.0;
   for (int j = 0; j < k; j++) {
      fro += K11[j + (size_t)j * k] * K11[j + (size_t)j * k];
      for (int i = j + 1; i < k; i++) fro += 2.0 * K11[i + (size_t)j * k] * K11[i + (size_t)j * k];
   }
   fro = std::sqrt(fro);
   const double nu = std::sqrt((double)k) * (std::nextafter(fro, fro + 1.0) - fro);
   // L = chol(K11 + nu I), G = L^{-1} (kept with gradients), Gt = G^T in d_B
   if (with_grad && (dalloc(&N->G, kk) || dalloc(&N->Gt, kk))) return fail("allocation");
   {
      const int info = chol_inverse_dev(d_K11, k, nu, with_grad ? N->G : nullptr, d_B, d_info, s);
      if (info > 0) {
         fprintf(stderr, "nfft4gp_amd: Nystrom setup: K11 + shift is not positive definite (column %d)\n", info);
         return fail(nullptr);
      }
      if (info < 0) return fail("Cholesky / triangular inverse of K11");
      // every row shard multiplies its rows by rank 0's factor (bitwise the same U1 rows as one GPU's)
      if (comm && bcast_root(comm, d_B, kk, s)) return fail("broadcast of L^{-T}");
   }
   if (with_grad) {
      // GdKG_g = L^{-1} dK11_g L^{-T} for g = f, l (chol.c:512-523)
      if (hipMemcpyAsync(N->Gt, d_B, sizeof(double) * kk, hipMemcpyDeviceToDevice, s) != hipSuccess ||
          dalloc(&N->GdKG, 2 * kk) || dalloc(&d_T, kk))
         return fail("allocation");
      for (int g = 0; g < 2; g++) {
         if (gemm(false, k, k, k, d_K11 + (g + 1) * kk, k, N->Gt, k, d_T, k, s) ||
             gemm(false, k, k, k, N->G, k, d_T, k, N->GdKG + g * kk, k, s))
            return fail("gemm");
      }
   }

   phase("k11+chol");
   // 3. U1 = Kp G^T  (dtrmm 'R' 'L' 'T', matops.c Nfft4GPTrilNystromMm)
   (void)hipEventRecord(ev[2], s);
   if (n > 0 && gemm(false, n, k, k, d_Kp, n, d_B, k, d_U1, n, s)) return fail("gemm");
   (void)hipEventRecord(ev[3], s);

   phase("gemm1");
   // 4. AA = U1^T U1, split over rows (fixed-order sum, deterministic); with gradients D = AA is kept
   (void)hipEventRecord(ev[4], s);
   if (n > 0 && gram_tn(k, k, n, d_U1, n, d_U1, n, d_AA, 1, s)) return fail("gram");
   if (n == 0 && hipMemsetAsync(d_AA, 0, sizeof(double) * kk, s) != hipSuccess) return fail("gram");
   // the Gram is a sum over rows (matops.c:65-137): the row shards' partial Grams add up to the whole one
   if (comm && comm->allreduce(d_AA, kk, s)) return fail("all-reduce of the Gram");
   (void)hipEventRecord(ev[5], s);
   if (with_grad) {
      if (dalloc(&N->D, kk) ||
          hipMemcpyAsync(N->D, d_AA, sizeof(double) * kk, hipMemcpyDeviceToDevice, s) != hipSuccess)
         return fail("allocation");
   }
   phase("gram");
   // 5. eig(AA) = V diag(w1) V^T (dsyev: ascending); W = V(:, reversed) diag(w1^-1/2) with the
   //    reference's 1e12 factor for sqrt(w1) < 1e-12 (matops.c Nfft4GPTrilNystromSvd); s (nys.c:641-647)
   const double eta = mu * f2;
   if (dalloc(&d_w1, (size_t)k) || dalloc(&d_e, (size_t)k) || dalloc(&d_s, (size_t)k)) return fail("allocation");
   RocSolver& R = rocsolver();
   if (R.ok) {
      int info = 0;
      R.set_stream(R.h, s);
      if (R.syevd(R.h, rocblas_evect_original, rocblas_fill_lower, k, d_AA, k, d_w1, d_e, d_info) !=
              rocblas_status_success ||
          hipMemcpyAsync(&info, d_info, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess || info)
         return fail("rocsolver_dsyevd");
   } else {
      std::vector<double> AA(kk);
      if (hipMemcpyAsync(AA.data(), d_AA, sizeof(double) * kk, hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
         return fail("gram download");
      std::vector<double> w1, V;
      if (sym_eig(AA, k, w1, V)) return fail("eigensolver did not converge");
      if (hipMemcpy(d_AA, V.data(), sizeof(double) * V.size(), hipMemcpyHostToDevice) ||
          hipMemcpy(d_w1, w1.data(), sizeof(double) * k, hipMemcpyHostToDevice))
         return fail("upload");
   }
   hipLaunchKernelGGL(k_nys_scale, dim3((k + 255) / 256, k), dim3(256), 0, s, d_AA, d_w1, k, eta, d_B, d_s,
                      k11_mode == 1 ? 1 : 0);
   // one eigenbasis for all row shards: rank 0's (an eigensolver may differ in signs or rounding elsewhere)
   if (comm && (bcast_root(comm, d_B, kk, s) || bcast_root(comm, d_s, (size_t)k, s)))
      return fail("broadcast of the eigenbasis");
   phase("eig");
   // 6. U = U1 W.  Without gradients the panel's storage is reused for U; with them the panel (K, dK/df,
   //    dK/dl) and U1 (= dU, nys.c:611-615) stay, for Dvp and Trace.
   if (with_grad) {
      if (dalloc(&N->U, nk)) return fail("allocation");
   } else {
      N->U = d_Kp;
      d_Kp = nullptr;
   }
   (void)hipEventRecord(ev[6], s);
   if (n > 0 && gemm(false, n, k, k, d_U1, n, d_B, k, N->U, n, s)) return fail("gemm");
   (void)hipEventRecord(ev[7], s);
   N->eta = eta;
   N->s = d_s;
   d_s = nullptr;
   if (with_grad) {
      N->grad = true;
      N->f2 = f2;
      N->Kall = d_Kp;
      d_Kp = nullptr;
      N->dU = d_U1;
      d_U1 = nullptr;
      if (dalloc(&N->vk, 8 * (size_t)k) || dalloc(&N->vn, (size_t)n)) return fail("allocation");
   }
   N->hs.resize(k);
   if (hipMemcpyAsync(N->hs.data(), N->s, sizeof(double) * k, hipMemcpyDeviceToHost, s) != hipSuccess ||
       nys_alloc_scratch(N) || hipStreamSynchronize(s) != hipSuccess)
      return fail("sync");
   phase("gemm2");
   for (int i = 0; i < 4; i++) {
      float ms = 0.0f;
      if (hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]) == hipSuccess) N->setup_ms[i] = ms;
   }
   release();
   return N;
}

}  // namespace nfft4gp_amd

extern "C" {

int Nfft4GPAmdNysSetupTimes(void* nys, double* ms4)
{
   nfft4gp_amd::NysDev* N = (nfft4gp_amd::NysDev*)nys;
   if (!N || !ms4) return -1;
   for (int i = 0; i < 4; i++) ms4[i] = N->setup_ms[i];
   return 0;
}

int Nfft4GPAmdNysFactors(void* nys, const int* perm, double* U, double* s, double* eta)
{
   nfft4gp_amd::NysDev* N = (nfft4gp_amd::NysDev*)nys;
   if (!N) return -1;
   const int n = N->n, k = N->k;
   if (U) {
      std::vector<double> h((size_t)n * k);
      NFFT4GP_HIP_CHECK(hipMemcpy(h.data(), N->U, sizeof(double) * h.size(), hipMemcpyDeviceToHost));
      for (int c = 0; c < k; c++)
         for (int i = 0; i < n; i++) U[i + (size_t)c * n] = h[(perm ? perm[i] : i) + (size_t)c * n];
   }
   if (s) NFFT4GP_HIP_CHECK(hipMemcpy(s, N->s, sizeof(double) * k, hipMemcpyDeviceToHost));
   if (eta) *eta = N->eta;
   return 0;
}

}  // extern "C"

// ---- host-only helpers for the CPU test-suite (no GPU needed) ------------------------------------
extern "C" int Nfft4GPAmdHostSymEig(const double* A, int n, double* w, double* V)
{
   std::vector<double> a(A, A + (size_t)n * n), wv, Vv;
   if (nfft4gp_amd::sym_eig_host(a, n, wv, Vv)) return -1;
   memcpy(w, wv.data(), sizeof(double) * n);
   memcpy(V, Vv.data(), sizeof(double) * (size_t)n * n);
   return 0;
}

extern "C" int Nfft4GPAmdHostCholInverse(const double* A, int k, double shift, double* G)
{
   std::vector<double> a(A, A + (size_t)k * k);
   for (int j = 0; j < k; j++) a[j + (size_t)j * k] += shift;
   const int info = nfft4gp_amd::chol_inverse_host(a, k);
   if (info) return info;
   memcpy(G, a.data(), sizeof(double) * (size_t)k * k);
   return 0;
}

// ---- device test hooks (tests/ only): the MFMA GEMM and the panel kernel in isolation ---------------
extern "C" int Nfft4GPAmdDebugGemm(int transA, int M, int N, int K, const double* A, long long lda, const double* B,
                                   long long ldb, double* C, long long ldc)
{
   if (nfft4gp_amd::gemm_f64(transA != 0, M, N, K, A, lda, B, ldb, C, ldc, nfft4gp_amd::current_stream()))
      return -1;
   NFFT4GP_HIP_CHECK(hipStreamSynchronize(nfft4gp_amd::current_stream()));
   return 0;
}
