// afn_setup.hip -- farthest-point ordering and the AFN preconditioner's setup in HBM.
//
//   Nfft4GPAmdSortFps   Nfft4GPSortFps with kFpsAlgorithmParallel1 (ordering.c:422-711, :713-739): start at
//                       the point closest to the mean, then repeatedly add the unselected point farthest
//                       from the selected set, until k points or the fill distance drops below tol.
//                       One launch per added point (k_fps_step): every workgroup updates its points'
//                       distance to the newest point, the last workgroup to finish (a ticket) reduces the
//                       per-workgroup maxima in a fixed order and appends the winner.  Control stays on the
//                       device; the host reads the count once at the end.  Distances are the reference's
//                       sqrt(sum_c (x_ic - y_c)^2) summed over c in order with unfused multiply and add
//                       (kernels.c:5-15), ties go to the lowest index as in its serial loop, so the order
//                       and the fill distances are bitwise the reference's (the start point depends on the
//                       mean, summed here in a fixed blocked order).
//   Nfft4GPAmdAfnSetup  Nfft4GPPrecondAFNSetup (afn.c:161-489) with a given rank k, its default Schur
//                       option (kernel FSAI, schur_opt 3, afn.c:430-480) and ordering:
//                         perm_opt 0: identity (afn.c:245-256, max_k < 0: predefined rank),
//                         perm_opt 1: FPS (afn.c:196-209),  perm_opt 2: the caller's permutation
//                       (e.g. the reference's Nfft4GPRandPerm, afn.c:210-218).
//                       K11 = K(X1) + noise -> L11 (rocSOLVER potrf) -> L11^{-1} (trtri);
//                       K12 = K(X1, X2) (k x n2); W = L11^{-1} K12 (MFMA f64 GEMM, the reference's dtrtrs);
//                       FSAI of the Schur complement K(X2) - W'W (Nfft4GPKernelSchurCombineKernel,
//                       kernels.c:3496-3760) on X2's KNN pattern (fsai_setup.hip).  k = 0: FSAI of K alone;
//                       k = n: A11 alone on the unpermuted data (afn.c:263-284).
//   The rank estimation (rankest.c, afn.c:178-243: libc rand() subsamples of 500 points) is not part of
//   this library: the caller picks k.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "callbacks.hpp"
#include "internal.h"

using namespace nfft4gp_amd;

namespace {

constexpr int kFpsThreads = 256;
constexpr int kFpsMaxBlocks = 2048;
constexpr int kFpsMaxDims = 256;

struct FpsState {
   int i1;        // newest selected point
   int count;     // points selected
   int stop;
   int first;     // the next pass is the initial one (ordering.c:545-607)
   unsigned int ticket;
};

// sqrt(sum_c (x_ic - q_c)^2), c in order, unfused (Nfft4GPDistanceEuclid, kernels.c:5-15)
__device__ __forceinline__ double dist_to(const double* __restrict__ X, long long ldim, int d, const double* q, int i)
{
#pragma clang fp contract(off)
   double v = 0.0;
   for (int c = 0; c < d; c++) {
      const double t = X[(size_t)c * ldim + i] - q[c];
      v += t * t;
   }
   return sqrt(v);
}

// (v, i) beats (w, j): larger value, then lower index (max mode); smaller value, then lower index (min)
__device__ __forceinline__ bool beats(double v, int i, double w, int j, bool max_mode)
{
   if (i < 0) return false;
   if (j < 0) return true;
   if (v != w) return max_mode ? (v > w) : (v < w);
   return i < j;
}

__device__ void block_best(double& v, int& i, bool max_mode)
{
   __shared__ double sv[kFpsThreads / 64];
   __shared__ int si[kFpsThreads / 64];
   for (int off = 32; off > 0; off >>= 1) {
      const double ov = __shfl_down(v, off, 64);
      const int oi = __shfl_down(i, off, 64);
      if (beats(ov, oi, v, i, max_mode)) {
         v = ov;
         i = oi;
      }
   }
   const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
   if (lane == 0) {
      sv[wave] = v;
      si[wave] = i;
   }
   __syncthreads();
   if (threadIdx.x == 0) {
      for (int w = 1; w < kFpsThreads / 64; w++)
         if (beats(sv[w], si[w], v, i, max_mode)) {
            v = sv[w];
            i = si[w];
         }
   }
}

// the last workgroup to finish (ticket) reduces every workgroup's (value, index) with all its threads;
// returns true in that workgroup, with the winner in (v, i) on thread 0
__device__ bool last_block_best(double bv, int bi, double* pv, int* pi, unsigned int* ticket, bool max_mode,
                                double& v, int& i)
{
   __shared__ int s_last;
   block_best(bv, bi, max_mode);
   if (threadIdx.x == 0) {
      pv[blockIdx.x] = bv;
      pi[blockIdx.x] = bi;
      __threadfence();
      s_last = (atomicAdd(ticket, 1u) == gridDim.x - 1) ? 1 : 0;
   }
   __syncthreads();
   if (!s_last) return false;
   __threadfence();
   v = 0.0;
   i = -1;
   for (int g = threadIdx.x; g < (int)gridDim.x; g += kFpsThreads) {
      const double gv = __hip_atomic_load(&pv[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int gi = __hip_atomic_load(&pi[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (beats(gv, gi, v, i, max_mode)) {
         v = gv;
         i = gi;
      }
   }
   __syncthreads();  // block_best's LDS is reused
   block_best(v, i, max_mode);
   return true;
}

// per-column mean of data / n (ordering.c:467-506), blocked fixed-order sums
__global__ __launch_bounds__(kFpsThreads) void k_col_mean(const double* __restrict__ X, long long ldim, int n,
                                                          double* __restrict__ mean)
{
   __shared__ double s[kFpsThreads];
   const int c = blockIdx.x;
   double acc = 0.0;
   for (int i = threadIdx.x; i < n; i += kFpsThreads) acc += X[(size_t)c * ldim + i] / n;
   s[threadIdx.x] = acc;
   __syncthreads();
   for (int w = kFpsThreads / 2; w > 0; w >>= 1) {
      if (threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
      __syncthreads();
   }
   if (threadIdx.x == 0) mean[c] = s[0];
}

// the point closest to the mean (ordering.c:509-538): strict <, lowest index on ties
__global__ __launch_bounds__(kFpsThreads) void k_fps_center(const double* __restrict__ X, long long ldim, int n, int d,
                                                            const double* __restrict__ mean, double* __restrict__ pv,
                                                            int* __restrict__ pi, FpsState* st)
{
   __shared__ double q[kFpsMaxDims];
   for (int c = threadIdx.x; c < d; c += kFpsThreads) q[c] = mean[c];
   __syncthreads();
   double bv = 0.0;
   int bi = -1;
   for (int i = blockIdx.x * kFpsThreads + threadIdx.x; i < n; i += gridDim.x * kFpsThreads) {
      const double v = dist_to(X, ldim, d, q, i);
      if (beats(v, i, bv, bi, false)) {
         bv = v;
         bi = i;
      }
   }
   double v;
   int b;
   if (!last_block_best(bv, bi, pv, pi, &st->ticket, false, v, b) || threadIdx.x != 0) return;
   st->i1 = b;
   st->ticket = 0u;
}

// one FPS pass against the newest point st->i1 (ordering.c:545-694)
__global__ __launch_bounds__(kFpsThreads) void k_fps_step(const double* __restrict__ X, long long ldim, int n, int d,
                                                          double* dc, int* marker, double* __restrict__ pv,
                                                          int* __restrict__ pi, FpsState* st, int* perm,
                                                          double* dist, int k, double tol)
{
   __shared__ double q[kFpsMaxDims];
   __shared__ int s_stop, s_i1, s_first;
   if (threadIdx.x == 0) {
      s_stop = st->stop;
      s_i1 = st->i1;
      s_first = st->first;
   }
   __syncthreads();
   if (s_stop) return;
   const int i1 = s_i1;
   const bool first = s_first != 0;
   for (int c = threadIdx.x; c < d; c += kFpsThreads) q[c] = X[(size_t)c * ldim + i1];
   __syncthreads();
   double bv = 0.0;
   int bi = -1;
   for (int i = blockIdx.x * kFpsThreads + threadIdx.x; i < n; i += gridDim.x * kFpsThreads) {
      if (!first && marker[i] >= 0) continue;
      const double di = dist_to(X, ldim, d, q, i);
      const double v = first ? di : (dc[i] <= di ? dc[i] : di);  // NFFT4GP_MIN (memory.h:26-33)
      dc[i] = v;
      if (beats(v, i, bv, bi, true)) {
         bv = v;
         bi = i;
      }
   }
   double v;
   int b;
   if (!last_block_best(bv, bi, pv, pi, &st->ticket, true, v, b) || threadIdx.x != 0) return;
   // the reference keeps (dmax, i2) = (0, 0) unless some distance is strictly positive
   double dmax = 0.0;
   int i2 = 0;
   if (b >= 0 && v > 0.0) {
      dmax = v;
      i2 = b;
   }
   int cnt = st->count;
   if (first) {
      // ordering.c:594-607: i1 enters with the largest distance, stop if that is below tol
      __hip_atomic_store(&dc[i1], dmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      marker[i1] = cnt;
      if (dist) dist[cnt] = dmax;
      perm[cnt++] = i1;
      st->first = 0;
      if (dmax < tol || cnt >= k) {
         st->count = cnt;
         st->stop = 1;
         st->ticket = 0u;
         return;
      }
   }
   marker[i2] = cnt;
   if (dist) dist[cnt] = dmax;
   perm[cnt++] = i2;
   st->i1 = i2;
   st->count = cnt;
   const double di2 = __hip_atomic_load(&dc[i2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
   st->stop = (cnt < k && di2 >= tol) ? 0 : 1;  // ordering.c:617 loop condition
   st->ticket = 0u;
}

// out[i + j*ldo] = K(A_i, B_j) (+ f^2 mu on the diagonal when diag_noise), A: ma points (lda), B: nb
// points (ldb), both column-major with d features.  The plain Gaussian / Matern-1/2 of kernels.c:680-1289,
// :2390-3033 (f^2 exp(-r^2 / 2 l^2), f^2 exp(-r / l)).
__global__ __launch_bounds__(256) void k_kmat(const double* __restrict__ A, long long lda, int ma,
                                              const double* __restrict__ B, long long ldb, int nb, int d, int kernel,
                                              double f2, double inv, double noise, int diag_noise,
                                              double* __restrict__ out, long long ldo)
{
   const int i = blockIdx.x * 256 + threadIdx.x;
   const int j = blockIdx.y;
   if (i >= ma) return;
   double s = 0.0;
   for (int c = 0; c < d; c++) {
      const double t = A[(size_t)c * lda + i] - B[(size_t)c * ldb + j];
      s = fma(t, t, s);
   }
   double v;
   if (diag_noise && i == j)
      v = f2 + noise;
   else
      v = f2 * exp(-(kernel == 0 ? s : sqrt(s)) * inv);
   out[(size_t)j * ldo + i] = v;
}

__global__ void k_gather_points(const double* __restrict__ X, long long ldim, int n, int d, const int* __restrict__ perm,
                                double* __restrict__ Xp)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   const int c = blockIdx.y;
   if (i < n && c < d) Xp[(size_t)c * n + i] = X[(size_t)c * ldim + perm[i]];
}

template <class T>
int dalloc(T** p, size_t count)
{
   *p = nullptr;
   return hipMalloc((void**)p, sizeof(T) * std::max<size_t>(1, count)) == hipSuccess ? 0 : -1;
}

// FPS on device coordinates; perm / dist: host arrays of at least k entries; returns the count or -1
int fps_device(const double* dX, long long ldim, int n, int d, int k, double tol, int* perm, double* dist,
               hipStream_t s)
{
   if (n <= 0 || d <= 0 || d > kFpsMaxDims) {
      fprintf(stderr, "nfft4gp_amd: FPS needs n > 0 and 1 <= d <= %d\n", kFpsMaxDims);
      return -1;
   }
   if (k <= 0 || k > n) k = n;  // ordering.c:425 (and at most n distinct points)
   const int grid = std::min(kFpsMaxBlocks, (n + kFpsThreads - 1) / kFpsThreads);
   double *dc = nullptr, *pv = nullptr, *mean = nullptr, *ddist = nullptr;
   int *marker = nullptr, *pi = nullptr, *dperm = nullptr;
   FpsState* st = nullptr;
   auto done = [&](int rc) {
      (void)hipStreamSynchronize(s);
      for (void* p : {(void*)dc, (void*)pv, (void*)mean, (void*)ddist, (void*)marker, (void*)pi, (void*)dperm,
                      (void*)st})
         (void)hipFree(p);
      return rc;
   };
   if (dalloc(&dc, n) || dalloc(&pv, grid) || dalloc(&mean, d) || dalloc(&ddist, k) || dalloc(&marker, n) ||
       dalloc(&pi, grid) || dalloc(&dperm, k) || dalloc(&st, 1))
      return done(-1);
   FpsState h0{0, 0, 0, 1, 0u};
   if (hipMemsetAsync(marker, 0xff, sizeof(int) * n, s) != hipSuccess ||
       hipMemcpyAsync(st, &h0, sizeof(h0), hipMemcpyHostToDevice, s) != hipSuccess)
      return done(-1);
   hipLaunchKernelGGL(k_col_mean, dim3(d), dim3(kFpsThreads), 0, s, dX, ldim, n, mean);
   hipLaunchKernelGGL(k_fps_center, dim3(grid), dim3(kFpsThreads), 0, s, dX, ldim, n, d, mean, pv, pi, st);
   // the first pass adds the centre and the farthest point; every later pass adds one point
   for (int it = 0; it < std::max(1, k - 1); it++)
      hipLaunchKernelGGL(k_fps_step, dim3(grid), dim3(kFpsThreads), 0, s, dX, ldim, n, d, dc, marker, pv, pi, st,
                         dperm, ddist, k, tol);
   FpsState h;
   if (hipGetLastError() != hipSuccess || hipMemcpyAsync(&h, st, sizeof(h), hipMemcpyDeviceToHost, s) != hipSuccess ||
       hipStreamSynchronize(s) != hipSuccess)
      return done(-1);
   if (hipMemcpy(perm, dperm, sizeof(int) * h.count, hipMemcpyDeviceToHost) != hipSuccess ||
       (dist && hipMemcpy(dist, ddist, sizeof(double) * h.count, hipMemcpyDeviceToHost) != hipSuccess))
      return done(-1);
   return done(h.count);
}

// Nfft4GPExpandPerm (utils.c:208-245): the k selected points, then the others in ascending order
std::vector<int> expand_perm(const int* perm, int k, int n)
{
   std::vector<int> out(perm, perm + k);
   std::vector<char> used(n, 0);
   for (int i = 0; i < k; i++) used[perm[i]] = 1;
   for (int i = 0; i < n; i++)
      if (!used[i]) out.push_back(i);
   return out;
}

}  // namespace

extern "C" {

int Nfft4GPAmdSortFps(const double* data, int n, int ldim, int d, int* k, double tol, int* perm, double* dist)
{
   if (!need_device("Nfft4GPAmdSortFps")) return -1;
   if (!data || !k || !perm || n <= 0 || ldim < n || d <= 0) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdSortFps needs data (ldim >= n), k and perm\n");
      return -1;
   }
   hipStream_t s = current_stream();
   const double* dX = data;
   double* owned = nullptr;
   if (!is_device_ptr(data)) {
      if (dalloc(&owned, (size_t)ldim * d) ||
          hipMemcpy(owned, data, sizeof(double) * (size_t)ldim * d, hipMemcpyHostToDevice) != hipSuccess) {
         (void)hipFree(owned);
         return -1;
      }
      dX = owned;
   }
   const int cnt = fps_device(dX, ldim, n, d, *k, tol, perm, dist, s);
   (void)hipFree(owned);
   if (cnt < 0) return -1;
   *k = cnt;
   return 0;
}

void* Nfft4GPAmdAfnSetup(const double* data, int n, int ldim, int d, int k, int perm_opt, const int* perm,
                         int schur_lfil, int kernel, void* fkernel_params)
{
   if (!need_device("Nfft4GPAmdAfnSetup")) return nullptr;
   const nfft4gp_kernel* kp = (const nfft4gp_kernel*)fkernel_params;
   if (!data || !kp || n <= 0 || ldim < n || d <= 0 || k < 0 || k > n || perm_opt < 0 || perm_opt > 2 ||
       (perm_opt == 2 && !perm)) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnSetup needs data (ldim >= n), kernel parameters, 0 <= k <= n, "
                      "perm_opt 0 (identity), 1 (FPS) or 2 (perm given)\n");
      return nullptr;
   }
   kernel = kernel ? 1 : 0;
   const double f = kp->_params[0], l = kp->_params[1], mu = kp->_noise_level;
   const double f2 = f * f, inv = (kernel == 0) ? 1.0 / (2.0 * l * l) : 1.0 / l;
   hipStream_t s = current_stream();
   const int n2 = n - k;
   double *dX = nullptr, *Xp = nullptr, *K11 = nullptr, *G = nullptr, *Gt = nullptr, *K12 = nullptr, *W = nullptr;
   int *dperm = nullptr, *dinfo = nullptr;
   void* S = nullptr;
   auto fail = [&](const char* what) -> void* {
      if (what) fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnSetup: %s failed\n", what);
      (void)hipStreamSynchronize(s);
      for (void* p : {(void*)dX, (void*)Xp, (void*)K11, (void*)G, (void*)Gt, (void*)K12, (void*)W, (void*)dperm,
                      (void*)dinfo})
         (void)hipFree(p);
      if (S) Nfft4GPAmdFsaiFree(S);
      return nullptr;
   };
   if (dalloc(&dX, (size_t)ldim * d)) return fail("allocation");
   const hipMemcpyKind kind = is_device_ptr(data) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
   if (hipMemcpy(dX, data, sizeof(double) * (size_t)ldim * d, kind) != hipSuccess) return fail("upload");
   // ordering (afn.c:196-256); k = n keeps the data unpermuted (afn.c:263-268)
   std::vector<int> hperm(n);
   for (int i = 0; i < n; i++) hperm[i] = i;
   if (k > 0 && k < n) {
      if (perm_opt == 1) {
         std::vector<int> sel(k);
         const int cnt = fps_device(dX, ldim, n, d, k, 0.0, sel.data(), nullptr, s);  // _tol = 0 (afn.c:203)
         if (cnt < 0) return fail("FPS");
         hperm = expand_perm(sel.data(), cnt, n);
         if (cnt != k) fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnSetup: FPS found %d distinct points\n", cnt);
      } else if (perm_opt == 2) {
         hperm.assign(perm, perm + n);
      }
   }
   if (dalloc(&dperm, n) || hipMemcpy(dperm, hperm.data(), sizeof(int) * n, hipMemcpyHostToDevice) != hipSuccess ||
       dalloc(&Xp, (size_t)n * d))
      return fail("allocation");
   hipLaunchKernelGGL(k_gather_points, dim3((n + 255) / 256, d), dim3(256), 0, s, dX, (long long)ldim, n, d, dperm, Xp);
   const size_t kk = (size_t)k * k;
   if (k > 0) {
      // A11 = K(X1) + noise; L11^{-1} (afn.c:425-428: AfnPrecondCholSetupWithKernel)
      if (dalloc(&K11, kk) || dalloc(&G, kk) || dalloc(&Gt, kk) || dalloc(&dinfo, 1)) return fail("allocation");
      hipLaunchKernelGGL(k_kmat, dim3((k + 255) / 256, k), dim3(256), 0, s, Xp, (long long)n, k, Xp, (long long)n, k,
                         d, kernel, f2, inv, f2 * mu, 1, K11, (long long)k);
      const int info = chol_inverse_dev(K11, k, 0.0, G, Gt, dinfo, s);
      if (info > 0) {
         fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnSetup: K11 is not positive definite (column %d)\n", info);
         return fail(nullptr);
      }
      if (info < 0) return fail("Cholesky / triangular inverse of K11");
   }
   if (n2 > 0 && k > 0) {
      // K12 = K(X1, X2) (afn.c:436), W = L11^{-1} K12 (afn.c:443, dtrtrs)
      if (dalloc(&K12, (size_t)k * n2) || dalloc(&W, (size_t)k * n2)) return fail("allocation");
      for (int j0 = 0; j0 < n2; j0 += 65535) {
         const int nb = std::min(65535, n2 - j0);
         hipLaunchKernelGGL(k_kmat, dim3((k + 255) / 256, nb), dim3(256), 0, s, Xp, (long long)n, k, Xp + k + j0,
                            (long long)n, nb, d, kernel, f2, inv, 0.0, 0, K12 + (size_t)j0 * k, (long long)k);
      }
      if (gemm_f64(false, k, n2, k, G, k, K12, k, W, k, s)) return fail("gemm");
   }
   if (n2 > 0) {
      // FSAI of the Schur complement on X2 (afn.c:445-473)
      std::vector<int> ia, ja;
      std::vector<double> aa, da;
      double* X2 = nullptr;
      if (dalloc(&X2, (size_t)n2 * d)) return fail("allocation");
      for (int c = 0; c < d; c++)
         if (hipMemcpyAsync(X2 + (size_t)c * n2, Xp + (size_t)c * n + k, sizeof(double) * n2, hipMemcpyDeviceToDevice,
                            s) != hipSuccess) {
            (void)hipFree(X2);
            return fail("copy");
         }
      const int rc = fsai_kernel_csr(X2, n2, n2, d, schur_lfil, kernel, f, l, mu, W, k > 0 ? k : 0, 0, ia, ja, aa, da,
                                     s);
      (void)hipStreamSynchronize(s);
      (void)hipFree(X2);
      if (rc) return fail("Schur-complement FSAI");
      S = Nfft4GPAmdFsaiCreate(n2, ia.data(), ja.data(), aa.data());
      if (!S) return fail("FSAI upload");
   }
   (void)hipStreamSynchronize(s);
   for (void* p : {(void*)dX, (void*)Xp, (void*)K11, (void*)W, (void*)dinfo}) (void)hipFree(p);
   dX = Xp = K11 = W = nullptr;
   dinfo = nullptr;
   void* A = afn_create_device(n, k, dperm, G, Gt, K12, S);
   if (!A) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnSetup: allocation failed\n");
      return nullptr;  // afn_create_device released the factors and S
   }
   return A;
}

}  // extern "C"
