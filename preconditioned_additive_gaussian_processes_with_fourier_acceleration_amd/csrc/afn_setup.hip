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

#include <chrono>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "callbacks.hpp"
#include "internal.h"
#include "kernel_eval.hpp"

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

// out[i + j*ldo] = K(x_{row0+i}, x_{col0+j}) for i < m, j < gridDim.y over the kernel coordinates X (ld
// ldx); the noise goes on entries where the two are one point when diag_noise (kernel_eval.hpp)
__global__ __launch_bounds__(256) void k_kmat(const double* __restrict__ X, long long ldx, int row0, int m, int col0,
                                              KernelParams P, int diag_noise, double* __restrict__ out, long long ldo)
{
   const int i = blockIdx.x * 256 + threadIdx.x;
   const int j = blockIdx.y;
   if (i >= m) return;
   double K, dK[3];
   kern_pair(P, X, ldx, row0 + i, col0 + j, diag_noise && row0 + i == col0 + j, K, dK);
   out[(size_t)j * ldo + i] = K;
}

// out[i + j*ldo] = dK_g(x_{row0+i}, x_{col0+j}) (kernel_eval.hpp: g = 0 f, 1 l, 2 mu)
__global__ __launch_bounds__(256) void k_kmat_grad(const double* __restrict__ X, long long ldx, int row0, int m,
                                                   int col0, KernelParams P, int diag_noise, int g,
                                                   double* __restrict__ out, long long ldo)
{
   const int i = blockIdx.x * 256 + threadIdx.x;
   const int j = blockIdx.y;
   if (i >= m) return;
   double K, dK[3];
   kern_pair(P, X, ldx, row0 + i, col0 + j, diag_noise && row0 + i == col0 + j, K, dK);
   out[(size_t)j * ldo + i] = dK[g];
}

// Phi(M) of chol_setup.m: the lower triangle with the diagonal halved, in place
__global__ void k_phi(double* M, int k)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
   if (i >= k) return;
   double& v = M[i + (size_t)j * k];
   if (i < j) v = 0.0;
   else if (i == j) v *= 0.5;
}

__global__ void k_diag_of(const double* __restrict__ A, int k, double* __restrict__ out)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < k) out[i] = A[i + (size_t)i * k];
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


// ---- rank estimation (rankest.c) ------------------------------------------------------------------

__global__ void k_scale(double* __restrict__ x, size_t count, double a)
{
   const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
   if (i < count) x[i] *= a;
}

__global__ void k_add_diag_n(double* __restrict__ A, int n, double v)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) A[i + (size_t)i * n] += v;
}

__global__ void k_copy_block(const double* __restrict__ A, long long lda, int m, double* __restrict__ B)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
   if (i < m) B[i + (size_t)j * m] = A[i + (size_t)j * lda];
}

// sum over the lower triangle (off-diagonal entries twice) of (A - B - shift I)^2 (B may be NULL):
// dlansy('F', 'L')^2 of A - B - shift I, one workgroup, fixed order
__global__ __launch_bounds__(1024) void k_sumsq_lower(const double* __restrict__ A, const double* __restrict__ B,
                                                      double shift, int n, double* __restrict__ out)
{
   __shared__ double s[1024];
   double acc = 0.0;
   const size_t nn = (size_t)n * n;
   for (size_t e = threadIdx.x; e < nn; e += 1024) {
      const int i = (int)(e % n), j = (int)(e / n);
      if (i < j) continue;
      double v = A[e];
      if (B) v -= B[e] + (i == j ? shift : 0.0);
      acc += (i == j ? 1.0 : 2.0) * v * v;
   }
   s[threadIdx.x] = acc;
   __syncthreads();
   for (int w = 512; w > 0; w >>= 1) {
      if (threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
      __syncthreads();
   }
   if (threadIdx.x == 0) *out = s[0];
}

// Nfft4GPRandPerm (utils.c:72-105): n draws of libc rand(), the indices of the k smallest (their order
// within the k is the reference's quick-split's; here ascending by (draw, index) -- the sample is used
// as a set)
std::vector<int> rand_perm(int n, int k)
{
   std::vector<std::pair<double, int>> v(n);
   {
      CallerRandBatch caller;
      for (int i = 0; i < n; i++) v[i] = {(double)rand(), i};
   }
   std::partial_sort(v.begin(), v.begin() + k, v.end());
   std::vector<int> out(k);
   for (int i = 0; i < k; i++) out[i] = v[i].second;
   return out;
}

struct RankCtx {
   const double* dX = nullptr;  // device, n x d column-major (ldim)
   long long ldim = 0;
   int n = 0, d = 0;
   KernelSpec ks;  // plain, or the additive kernel of ks.Xk (n x D, ld n) -- kernel_spec_of
   int D = 0;      // kernel coordinates per point
   hipStream_t s = nullptr;
   // the kernel on sample coordinates Xk_sample (additive) with noise `noise`
   KernelParams params(const double* Xk_sample, double noise) const
   {
      KernelSpec K = ks;
      K.Xk = ks.Xk ? Xk_sample : nullptr;
      K.mu = noise;
      return kernel_params_of(K, d);
   }
};

// the subsample rows of Nfft4GPSubData(data, RandPerm(n, n1)) into Xs (n1 x d) and, for an additive
// kernel, of its coordinates into Xks (n1 x D), both scaled by `scale`
int sample_points(const RankCtx& C, int n1, double scale, double* Xs, double* Xks)
{
   std::vector<int> rows = rand_perm(C.n, n1);
   int* drows = nullptr;
   if (dalloc(&drows, n1) || hipMemcpy(drows, rows.data(), sizeof(int) * n1, hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(drows);
      return -1;
   }
   hipLaunchKernelGGL(k_gather_points, dim3((n1 + 255) / 256, C.d), dim3(256), 0, C.s, C.dX, C.ldim, n1, C.d, drows, Xs);
   if (C.ks.Xk)
      hipLaunchKernelGGL(k_gather_points, dim3((n1 + 255) / 256, C.D), dim3(256), 0, C.s, C.ks.Xk, C.ks.ldk, n1, C.D,
                         drows, Xks);
   if (scale != 1.0) {
      hipLaunchKernelGGL(k_scale, dim3((unsigned)(((size_t)n1 * C.d + 255) / 256)), dim3(256), 0, C.s, Xs,
                         (size_t)n1 * C.d, scale);
      if (C.ks.Xk)
         hipLaunchKernelGGL(k_scale, dim3((unsigned)(((size_t)n1 * C.D + 255) / 256)), dim3(256), 0, C.s, Xks,
                            (size_t)n1 * C.D, scale);
   }
   (void)hipStreamSynchronize(C.s);
   (void)hipFree(drows);
   return hipGetLastError() == hipSuccess ? 0 : -1;
}

double device_scalar(const double* d, hipStream_t s)
{
   double h = NAN;
   if (hipMemcpyAsync(&h, d, sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
      return NAN;
   return h;
}

// Nfft4GPRankestNysScaledEstimateRank (rankest.c:248-352)
int nys_scaled_estimate(const RankCtx& C, int max_rank, int nsample)
{
   const int n = C.n, d = C.d;
   const int n1 = std::min(nsample, n);
   double *Xs = nullptr, *Xp = nullptr, *Xks = nullptr, *Xkp = nullptr, *K0 = nullptr, *K11 = nullptr, *G = nullptr,
          *Gt = nullptr, *W = nullptr, *Kn = nullptr, *dsum = nullptr;
   int *dperm = nullptr, *dinfo = nullptr;
   auto done = [&](int rc) {
      (void)hipStreamSynchronize(C.s);
      for (void* p : {(void*)Xs, (void*)Xp, (void*)Xks, (void*)Xkp, (void*)K0, (void*)K11, (void*)G, (void*)Gt,
                      (void*)W, (void*)Kn, (void*)dsum, (void*)dperm, (void*)dinfo})
         (void)hipFree(p);
      return rc;
   };
   const size_t nn = (size_t)n1 * n1;
   if ((C.ks.Xk && (dalloc(&Xks, (size_t)n1 * C.D) || dalloc(&Xkp, (size_t)n1 * C.D))) ||
       dalloc(&Xs, (size_t)n1 * d) || dalloc(&Xp, (size_t)n1 * d) || dalloc(&K0, nn) || dalloc(&K11, nn) ||
       dalloc(&G, nn) || dalloc(&Gt, nn) || dalloc(&W, nn) || dalloc(&Kn, nn) || dalloc(&dsum, 1) ||
       dalloc(&dperm, n1) || dalloc(&dinfo, 1))
      return done(-1);
   // scale so that the sample's spacing resembles the full data's: (n1 / n)^(1/d)
   if (sample_points(C, n1, pow((double)n1 / n, 1.0 / d), Xs, Xks)) return done(-1);
   std::vector<int> perm(n1);
   if (fps_device(Xs, n1, n1, d, n1, 0.0, perm.data(), nullptr, C.s) != n1) return done(-1);
   if (hipMemcpy(dperm, perm.data(), sizeof(int) * n1, hipMemcpyHostToDevice) != hipSuccess) return done(-1);
   hipLaunchKernelGGL(k_gather_points, dim3((n1 + 255) / 256, d), dim3(256), 0, C.s, Xs, (long long)n1, n1, d, dperm, Xp);
   if (C.ks.Xk)
      hipLaunchKernelGGL(k_gather_points, dim3((n1 + 255) / 256, C.D), dim3(256), 0, C.s, Xks, (long long)n1, n1, C.D,
                         dperm, Xkp);
   // K(perm, perm) without noise (rankest.c:307-309)
   hipLaunchKernelGGL(k_kmat, dim3((n1 + 255) / 256, n1), dim3(256), 0, C.s, C.ks.Xk ? Xkp : Xp, (long long)n1, 0, n1,
                      0, C.params(Xkp, 0.0), 1, K0, (long long)n1);
   hipLaunchKernelGGL(k_sumsq_lower, dim3(1), dim3(1024), 0, C.s, K0, nullptr, 0.0, n1, dsum);
   double a_fro = sqrt(device_scalar(dsum, C.s));
   const double nu = sqrt((double)n) * (nextafter(a_fro, a_fro + 1.0) - a_fro);  // rankest.c:318-322
   // A_fro of K + nu I (rankest.c:323-329); K0 itself stays noise-free for K1 = K0(1:k, :)
   hipLaunchKernelGGL(k_copy_block, dim3((n1 + 255) / 256, n1), dim3(256), 0, C.s, K0, (long long)n1, n1, Kn);
   hipLaunchKernelGGL(k_add_diag_n, dim3((n1 + 255) / 256), dim3(256), 0, C.s, Kn, n1, nu);
   hipLaunchKernelGGL(k_sumsq_lower, dim3(1), dim3(1024), 0, C.s, Kn, nullptr, 0.0, n1, dsum);
   a_fro = sqrt(device_scalar(dsum, C.s));
   const double tol = 0.1;
   const int npoints = 50;  // NFFT4GP_RANKEST_NPOINTS
   const int ngap = std::max(n1 / npoints, 1);
   int rank = n1;
   for (int i = 0; i < npoints; i++) {
      // rankest.c:334: for i = 0 the reference's (size_t)(i - 1) * ngap wraps, and the int conversion of
      // the huge double gives INT_MIN on x86, so only i >= 1 can stop here
      if (i * ngap >= n1 || (i >= 1 && (long long)floor(((double)(i - 1) * ngap) * (double)n / n1) > 2LL * max_rank)) {
         rank = (i - 1) * ngap;
         break;
      }
      const int k = i * ngap;
      double err;
      if (k == 0) {
         err = 1.0;
      } else {
         // Nfft4GPRankestNysError (rankest.c:183-240): K1 = K(perm[:k], perm), L = chol(K1(:, :k)),
         // |L^{-1}K1)^T (L^{-1}K1) - (K + nu I)|_F / A_fro
         hipLaunchKernelGGL(k_copy_block, dim3((k + 255) / 256, k), dim3(256), 0, C.s, K0, (long long)n1, k, K11);
         const int info = chol_inverse_dev(K11, k, 0.0, G, Gt, dinfo, C.s);
         if (info < 0) return done(-1);
         if (info > 0) {
            err = INFINITY;  // K11 not positive definite: the reference continues on a partial factor
         } else {
            if (gemm_f64(false, k, n1, k, G, k, K0, n1, W, k, C.s) || gram_tn(n1, n1, k, W, k, W, k, Kn, 0, C.s))
               return done(-1);
            hipLaunchKernelGGL(k_sumsq_lower, dim3(1), dim3(1024), 0, C.s, Kn, K0, nu, n1, dsum);
            err = sqrt(device_scalar(dsum, C.s)) / a_fro;
         }
      }
      if (err < tol) {
         rank = k;
         break;
      }
   }
   return done((int)floor(rank * (double)n / n1));
}

// Nfft4GPRankestDefaultToleranceEstimation (rankest.c:30-130): returns h, *pk = the estimated rank
double default_tolerance(const RankCtx& C, int nsamples, int* pk)
{
   const int n = C.n, d = C.d;
   const int n1 = std::min(nsamples, n);
   double *Xs = nullptr, *Xks = nullptr, *K = nullptr;
   auto done = [&](double v) {
      (void)hipStreamSynchronize(C.s);
      (void)hipFree(Xs);
      (void)hipFree(Xks);
      (void)hipFree(K);
      return v;
   };
   if ((C.ks.Xk && dalloc(&Xks, (size_t)n1 * C.D)) || dalloc(&Xs, (size_t)n1 * d) || dalloc(&K, (size_t)n1 * n1) ||
       sample_points(C, n1, 1.0, Xs, Xks))
      return done(NAN);
   std::vector<int> perm(n1);
   std::vector<double> dist(n1);
   if (fps_device(Xs, n1, n1, d, n1, 0.0, perm.data(), dist.data(), C.s) != n1) return done(NAN);
   // K of the sample with noise (kernels.c:1198) and its eigenvalues (dsyev 'N')
   hipLaunchKernelGGL(k_kmat, dim3((n1 + 255) / 256, n1), dim3(256), 0, C.s, C.ks.Xk ? Xks : Xs, (long long)n1, 0, n1, 0,
                      C.params(Xks, C.ks.mu), 1, K, (long long)n1);
   std::vector<double> eig;
   if (sym_eigvals_dev(K, n1, eig, C.s)) return done(NAN);
   const double tol = 0.41, tol2 = 0.2, tol3 = 1.1 * C.ks.mu;
   int rank = 0;
   for (int i = n1 - 1; i >= 0; i--) {
      if (eig[i] < tol3) break;
      rank++;
   }
   const int rank2 = rank - 1;
   while (rank > 1) {
      rank--;
      if ((dist[rank - 1] - dist[rank]) / dist[rank] > tol || dist[rank] <= (1.0 + tol2) * dist[rank2]) break;
   }
   if (pk) *pk = rank + 1;
   return done(dist[rank]);
}

// Nfft4GPRankestNysScaled (rankest.c:354-391)
int rankest_nys_scaled(const RankCtx& C, int max_rank, int nsample, int nsample_r)
{
   long long total = 0;
   for (int i = 0; i < nsample_r; i++) {
      const int r = nys_scaled_estimate(C, max_rank, nsample);
      if (r < 0) return -1;
      total += r;
   }
   int rank = (int)floor((double)total / nsample_r);
   const int n1 = std::min(nsample, C.n);
   const int ngap = std::max(n1 / 50, 1);
   if (rank <= (int)floor(ngap * (double)C.n / n1)) rank = 0;  // "extra check needed" (rankest.c:380-385)
   return rank;
}

// Nfft4GPRankestDefault (rankest.c:132-181): the rank and the FPS order it selected
int rankest_default(const RankCtx& C, int max_rank, int nsample, int nsample_r, double full_tol, std::vector<int>& perm)
{
   int est = 0, total = 0;
   double tol = default_tolerance(C, nsample, &est);
   if (std::isnan(tol)) return -1;
   total += est;
   for (int i = 1; i < nsample_r; i++) {
      const double t1 = default_tolerance(C, nsample, &est);
      if (std::isnan(t1)) return -1;
      tol += t1;
      total += est;
   }
   tol /= nsample_r;
   const bool full = total / (double)((long long)nsample * nsample_r) > full_tol;
   const int kmax = std::min(max_rank, C.n);
   perm.assign(kmax, 0);
   const int rank = fps_device(C.dX, C.ldim, C.n, C.d, kmax, full ? 0.0 : tol, perm.data(), nullptr, C.s);
   if (rank < 0) return -1;
   perm.resize(rank);
   return rank;
}

int rank_ctx(RankCtx& C, const double* data, int n, int ldim, int d, int kernel, void* params, double** owned,
             double** owned_k)
{
   *owned = *owned_k = nullptr;
   if (!data || !params || n <= 0 || ldim < n || d <= 0 || d > kFpsMaxDims) {
      fprintf(stderr, "nfft4gp_amd: rank estimation needs data (ldim >= n, d <= %d) and kernel parameters\n",
              kFpsMaxDims);
      return -1;
   }
   C.n = n;
   C.d = d;
   C.ldim = ldim;
   C.s = current_stream();
   const int additive = kernel_spec_of(params, nullptr, kernel, n, C.ks, owned_k);
   if (additive < 0) return -1;
   C.D = additive ? (C.ks.nw - 1) * C.ks.dw + C.ks.last_dw : d;
   if (is_device_ptr(data)) {
      C.dX = data;
      return 0;
   }
   if (dalloc(owned, (size_t)ldim * d) ||
       hipMemcpy(*owned, data, sizeof(double) * (size_t)ldim * d, hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(*owned);
      *owned = nullptr;
      return -1;
   }
   C.dX = *owned;
   return 0;
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
   return Nfft4GPAmdAfnSetupSchur(data, n, ldim, d, k, perm_opt, perm, 3, schur_lfil, kernel, fkernel_params);
}

}  // extern "C"

namespace {
// Nfft4GPAmdAfnSetupSchur's body; *breakdown = true when the factors cannot be formed (K11 not positive
// definite, or a row of the Schur complement's FSAI with a non-positive pivot: non-finite values, MATLAB's
// ~isreal(PRE.GS), afn_setup.m:93-98)
void* afn_setup_impl(const double* data, int n, int ldim, int d, int k, int perm_opt, const int* perm, int schur_opt,
                     int schur_lfil, int kernel, void* fkernel_params, bool* breakdown, AfnGrad** gout = nullptr)
{
   *breakdown = false;
   if (gout) *gout = nullptr;
   if (gout && (k <= 0 || k >= n || schur_opt != 3)) {
      fprintf(stderr, "nfft4gp_amd: AFN gradients need 0 < k < n and the Schur FSAI (schur_opt 3)\n");
      return nullptr;
   }
   if (!data || !fkernel_params || n <= 0 || ldim < n || d <= 0 || k < 0 || k > n || perm_opt < 0 || perm_opt > 2 ||
       (perm_opt == 2 && !perm) || (schur_opt != 0 && schur_opt != 3) || (schur_opt == 0 && k == 0)) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnSetup needs data (ldim >= n), kernel parameters, 0 <= k <= n, "
                      "perm_opt 0 (identity), 1 (FPS) or 2 (perm given), schur_opt 0 (k > 0) or 3\n");
      return nullptr;
   }
   // the kernel: plain (data's coordinates) or this library's additive handle (its window buffer)
   KernelSpec K;
   double* dXk = nullptr;
   const int additive = kernel_spec_of(fkernel_params, nullptr, kernel, n, K, &dXk);
   if (additive < 0) return nullptr;
   const int D = additive ? (K.nw - 1) * K.dw + K.last_dw : d;  // kernel coordinates per point
   hipStream_t s = current_stream();
   const int n2 = n - k;
   double *dX = nullptr, *Xp = nullptr, *Xkp = nullptr, *K11 = nullptr, *G = nullptr, *Gt = nullptr, *K12 = nullptr,
          *W = nullptr;
   // gradients: L, dK11 / GdKG (3 k x k each), dL, dK12 (2 panels), B (2) and C (3) panels of the Schur FSAI
   double *Lf = nullptr, *dK11 = nullptr, *GdKG = nullptr, *dLg = nullptr, *dK12 = nullptr, *PB = nullptr,
          *PC = nullptr, *tmp = nullptr;
   AfnGrad* AG = nullptr;
   int *dperm = nullptr, *dinfo = nullptr;
   void* S = nullptr;
   auto fail = [&](const char* what) -> void* {
      if (what) fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnSetup: %s failed\n", what);
      (void)hipStreamSynchronize(s);
      for (void* p : {(void*)dX, (void*)Xp, (void*)Xkp, (void*)dXk, (void*)K11, (void*)G, (void*)Gt, (void*)K12,
                      (void*)W, (void*)dperm, (void*)dinfo, (void*)Lf, (void*)dK11, (void*)GdKG, (void*)dLg,
                      (void*)dK12, (void*)PB, (void*)PC, (void*)tmp})
         (void)hipFree(p);
      if (S) Nfft4GPAmdFsaiFree(S);
      if (AG) afn_grad_free(AG);
      return nullptr;
   };
   // NFFT4GP_AMD_VERBOSE: the setup's phases on stderr (stream synchronised at each stamp)
   const bool verbose = getenv("NFFT4GP_AMD_VERBOSE") != nullptr;
   const auto tv0 = std::chrono::steady_clock::now();
   auto stamp = [&](const char* what) {
      if (!verbose) return;
      (void)hipStreamSynchronize(s);
      fprintf(stderr, "nfft4gp_amd: AFN setup %-28s %8.1f ms\n", what,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tv0).count());
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
   stamp("upload + ordering");
   if (dalloc(&dperm, n) || hipMemcpy(dperm, hperm.data(), sizeof(int) * n, hipMemcpyHostToDevice) != hipSuccess ||
       dalloc(&Xp, (size_t)n * d))
      return fail("allocation");
   hipLaunchKernelGGL(k_gather_points, dim3((n + 255) / 256, d), dim3(256), 0, s, dX, (long long)ldim, n, d, dperm, Xp);
   if (additive) {
      if (dalloc(&Xkp, (size_t)n * D)) return fail("allocation");
      hipLaunchKernelGGL(k_gather_points, dim3((n + 255) / 256, D), dim3(256), 0, s, dXk, (long long)n, n, D, dperm,
                         Xkp);
   }
   const double* Xk = additive ? Xkp : Xp;  // kernel coordinates in the permuted order, ld n
   KernelSpec Kp = K;
   Kp.Xk = additive ? Xkp : nullptr;
   Kp.ldk = n;
   const KernelParams P = kernel_params_of(Kp, d);
   const size_t kk = (size_t)k * k;
   if (k > 0) {
      // A11 = K(X1) + noise; L11^{-1} (afn.c:425-428: AfnPrecondCholSetupWithKernel)
      if (dalloc(&K11, kk) || dalloc(&G, kk) || dalloc(&Gt, kk) || dalloc(&dinfo, 1)) return fail("allocation");
      hipLaunchKernelGGL(k_kmat, dim3((k + 255) / 256, k), dim3(256), 0, s, Xk, (long long)n, 0, k, 0, P, 1, K11,
                         (long long)k);
      if (gout) {  // L itself (afn_dvp.m multiplies by L and L'): a second potrf on a copy
         if (dalloc(&Lf, kk) || hipMemcpyAsync(Lf, K11, sizeof(double) * kk, hipMemcpyDeviceToDevice, s) != hipSuccess)
            return fail("allocation");
      }
      const int info = chol_inverse_dev(K11, k, 0.0, G, Gt, dinfo, s);
      if (info > 0) {
         fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnSetup: K11 is not positive definite (column %d)\n", info);
         *breakdown = true;
         return fail(nullptr);
      }
      if (info < 0) return fail("Cholesky / triangular inverse of K11");
      if (gout && chol_factor_dev(Lf, k, dinfo, s)) return fail("Cholesky of K11");
   }
   stamp("gather + K11 + Cholesky");
   if (n2 > 0 && k > 0) {
      // K12 = K(X1, X2) (afn.c:436), W = L11^{-1} K12 (afn.c:443, dtrtrs; the Schur FSAI's kernel)
      if (dalloc(&K12, (size_t)k * n2) || (schur_opt == 3 && dalloc(&W, (size_t)k * n2))) return fail("allocation");
      for (int j0 = 0; j0 < n2; j0 += 65535) {
         const int nb = std::min(65535, n2 - j0);
         hipLaunchKernelGGL(k_kmat, dim3((k + 255) / 256, nb), dim3(256), 0, s, Xk, (long long)n, 0, k, k + j0, P, 0,
                            K12 + (size_t)j0 * k, (long long)k);
      }
      if (schur_opt == 3 && gemm_f64(false, k, n2, k, G, k, K12, k, W, k, s)) return fail("gemm");
   }
   if (gout) {
      // chol_setup.m with require_grad: GdKG_g = L^{-1} dK11_g L^{-T}, dL_g = L Phi(GdKG_g); the Schur kernel's
      // panels B_g = L^{-1} dK12_g and C_g = GdKG_g L^{-1} K12 (schurCombinedKernel.m); dK12_mu = 0
      const size_t kn2 = (size_t)k * n2;
      if (dalloc(&dK11, 3 * kk) || dalloc(&GdKG, 3 * kk) || dalloc(&dLg, 3 * kk) || dalloc(&tmp, kk) ||
          dalloc(&dK12, 2 * kn2) || dalloc(&PB, 2 * kn2) || dalloc(&PC, 3 * kn2))
         return fail("allocation (gradients)");
      for (int g = 0; g < 3; g++) {
         double* dKg = dK11 + g * kk;
         double* GdKGg = GdKG + g * kk;
         hipLaunchKernelGGL(k_kmat_grad, dim3((k + 255) / 256, k), dim3(256), 0, s, Xk, (long long)n, 0, k, 0, P, 1, g,
                            dKg, (long long)k);
         if (gemm_f64(false, k, k, k, G, k, dKg, k, tmp, k, s) || gemm_f64(false, k, k, k, tmp, k, Gt, k, GdKGg, k, s))
            return fail("gemm (GdKG)");
         if (hipMemcpyAsync(tmp, GdKGg, sizeof(double) * kk, hipMemcpyDeviceToDevice, s) != hipSuccess) return fail("copy");
         hipLaunchKernelGGL(k_phi, dim3((k + 255) / 256, k), dim3(256), 0, s, tmp, k);
         if (gemm_f64(false, k, k, k, Lf, k, tmp, k, dLg + g * kk, k, s)) return fail("gemm (dL)");
         if (gemm_f64(false, k, n2, k, GdKGg, k, W, k, PC + g * kn2, k, s)) return fail("gemm (C)");
      }
      for (int g = 0; g < 2; g++) {
         for (int j0 = 0; j0 < n2; j0 += 65535) {
            const int nb = std::min(65535, n2 - j0);
            hipLaunchKernelGGL(k_kmat_grad, dim3((k + 255) / 256, nb), dim3(256), 0, s, Xk, (long long)n, 0, k, k + j0, P,
                               0, g, dK12 + g * kn2 + (size_t)j0 * k, (long long)k);
         }
         if (gemm_f64(false, k, n2, k, G, k, dK12 + g * kn2, k, PB + g * kn2, k, s)) return fail("gemm (B)");
      }
      if (hipGetLastError() != hipSuccess) return fail("gradient kernels");
   }
   stamp("K12 + W = L11^-1 K12");
   if (n2 > 0 && schur_opt == 3) {
      // FSAI of the Schur complement on X2 (afn.c:445-473): KNN on the points' coordinates, values of the
      // Schur-complement kernel on the kernel coordinates
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
      KernelSpec K2 = Kp;
      K2.Xk = additive ? Xkp + k : nullptr;  // column c of the last n2 points: Xkp + c*n + k + i
      // without gradients the CSR stays in HBM and the handle (L^T included) is formed there
      void* keep[3] = {nullptr, nullptr, nullptr};
      const int rc = fsai_kernel_csr(X2, n2, n2, d, schur_lfil, K2, W, k > 0 ? k : 0, gout ? 1 : 0, ia, ja, aa, da, s,
                                     PB, PC, gout ? nullptr : keep);
      (void)hipStreamSynchronize(s);
      (void)hipFree(X2);
      if (rc) return fail("Schur-complement FSAI");
      if (keep[0]) {
         const long long bad = count_nonfinite((const double*)keep[2], (size_t)ia[n2], s);
         if (bad != 0) {
            for (void* p : keep) (void)hipFree(p);
            if (bad < 0) return fail("Schur-complement FSAI check");
            fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnSetup: the Schur complement's FSAI broke down (non-positive "
                            "pivot)\n");
            *breakdown = true;
            return fail(nullptr);
         }
         stamp("Schur FSAI (KNN, rows)");
         S = fsai_create_from_device(n2, (int*)keep[0], (int*)keep[1], (double*)keep[2], ia, s);
         if (!S) return fail("FSAI handle");
         stamp("FSAI handle (L^T on the device)");
      } else {
         if (gout && !std::all_of(da.begin(), da.end(), [](double v) { return std::isfinite(v); })) {
            fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnSetup: the Schur FSAI's gradients are not finite\n");
            *breakdown = true;
            return fail(nullptr);
         }
         if (!std::all_of(aa.begin(), aa.end(), [](double v) { return std::isfinite(v); })) {
            fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnSetup: the Schur complement's FSAI broke down (non-positive "
                            "pivot)\n");
            *breakdown = true;
            return fail(nullptr);
         }
         stamp("Schur FSAI (KNN, rows)");
         S = Nfft4GPAmdFsaiCreate(n2, ia.data(), ja.data(), aa.data());
         if (!S) return fail("FSAI upload");
         stamp("FSAI handle (L^T, upload)");
         if (gout) {
            AG = new AfnGrad();
            AG->S = fsai_grad_create(n2, ia.data(), ja.data(), aa.data(), da.data());
            if (!AG->S) return fail("FSAI (gradients) upload");
         }
      }
   }
   if (gout) {
      // trace (afn_trace.m) and logdet (afn_logdet.m) from the diagonals; the factors the dvp keeps
      std::vector<double> hL(k), hdL(3 * (size_t)k);
      hipLaunchKernelGGL(k_diag_of, dim3((k + 255) / 256), dim3(256), 0, s, Lf, k, tmp);
      for (int g = 0; g < 3; g++)
         hipLaunchKernelGGL(k_diag_of, dim3((k + 255) / 256), dim3(256), 0, s, dLg + g * kk, k, tmp + (size_t)(g + 1) * k);
      if (hipMemcpyAsync(hL.data(), tmp, sizeof(double) * k, hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipMemcpyAsync(hdL.data(), tmp + k, sizeof(double) * 3 * k, hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
         return fail("copy");
      double ld = 0.0;
      for (int i = 0; i < k; i++) ld += std::log(hL[i]);
      AG->logdet = 2.0 * (ld + fsai_grad_diag(AG->S, -1, s));
      for (int g = 0; g < 3; g++) {
         double t = 0.0;
         for (int i = 0; i < k; i++) t += hdL[(size_t)g * k + i] / hL[i];
         // the Schur part: diagU = 1 / G_ii, diagdU = -dG_ii / G_ii^2, so sum diagdU / diagU = -sum dG_ii / G_ii
         AG->trace[g] = 2.0 * (t - fsai_grad_diag(AG->S, g, s));
      }
      AG->n = n;
      AG->k = k;
      AG->n2 = n2;
      if (dalloc(&AG->perm, n) ||
          hipMemcpyAsync(AG->perm, dperm, sizeof(int) * n, hipMemcpyDeviceToDevice, s) != hipSuccess ||
          dalloc(&AG->Linv, kk) || hipMemcpyAsync(AG->Linv, G, sizeof(double) * kk, hipMemcpyDeviceToDevice, s) != hipSuccess ||
          dalloc(&AG->LinvT, kk) ||
          hipMemcpyAsync(AG->LinvT, Gt, sizeof(double) * kk, hipMemcpyDeviceToDevice, s) != hipSuccess ||
          dalloc(&AG->work, 6 * (size_t)n + 8 * (size_t)k))
         return fail("allocation (gradients)");
      AG->L = Lf;
      AG->dL = dLg;
      AG->dK12 = dK12;
      AG->K12 = K12;
      Lf = dLg = dK12 = nullptr;
   }
   (void)hipStreamSynchronize(s);
   for (void* p : {(void*)dX, (void*)Xp, (void*)Xkp, (void*)dXk, (void*)K11, (void*)W, (void*)dinfo, (void*)dK11,
                   (void*)GdKG, (void*)PB, (void*)PC, (void*)tmp})
      (void)hipFree(p);
   dX = Xp = Xkp = dXk = K11 = W = nullptr;
   dK11 = GdKG = PB = PC = tmp = nullptr;
   dinfo = nullptr;
   // schur_opt 0 (afn.c:451-459): S^{-1} = I / _noise_level
   void* A = afn_create_device(n, k, dperm, G, Gt, K12, S, schur_opt == 0 ? 1.0 / K.mu : 0.0);
   if (!A) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnSetup: allocation failed\n");
      if (AG) afn_grad_free(AG);
      return nullptr;  // afn_create_device released the factors and S
   }
   if (gout) {
      AG->afn = A;
      *gout = AG;
   }
   return A;
}
}  // namespace

namespace {
// the sharded AFN setup (Nfft4GPAmdAfnShardSetup): afn.c:161-489 with the column work split by rows
void* afn_shard_setup_impl(const double* data, int n, int ldim, int d, int k, int perm_opt, const int* perm,
                           int schur_opt, int schur_lfil, int kernel, void* fkernel_params, int rb, int re, Comm* comm)
{
   if (!comm) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnShardSetup needs a communicator\n");
      return nullptr;
   }
   // Every rank reaches the same collectives: a failure on one rank (bad arguments, an allocation, a non-positive
   // pivot of ITS Schur rows, ...) is agreed over the communicator at three points -- before the L11^{-1}
   // broadcast, before the apply object is built, after it is built -- and then every rank returns NULL.
   auto agree = [&](bool ok_here) -> bool {
      double* d_flag = nullptr;
      double flag = ok_here ? 0.0 : 1.0;
      hipStream_t st = current_stream();
      if (hipMalloc((void**)&d_flag, sizeof(double)) != hipSuccess) return false;  // cannot even vote: HIP is gone
      bool ok = hipMemcpyAsync(d_flag, &flag, sizeof(double), hipMemcpyHostToDevice, st) == hipSuccess &&
                comm->allreduce(d_flag, 1, st) == 0 &&
                hipMemcpyAsync(&flag, d_flag, sizeof(double), hipMemcpyDeviceToHost, st) == hipSuccess &&
                hipStreamSynchronize(st) == hipSuccess;
      (void)hipFree(d_flag);
      if (ok && flag != 0.0 && ok_here)
         fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnShardSetup: %d rank(s) failed; every rank returns NULL\n", (int)flag);
      return ok && flag == 0.0;
   };
   const bool args_ok = data && fkernel_params && n > 0 && ldim >= n && d > 0 && k > 0 && k < n && perm_opt >= 0 &&
                        perm_opt <= 2 && (perm_opt != 2 || perm) && (schur_opt == 0 || schur_opt == 3) && rb >= 0 &&
                        re <= n && rb <= re;
   if (!args_ok)
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnShardSetup needs data (ldim >= n), kernel parameters, 0 < k < n, "
                      "perm_opt 0 / 1 / 2 (perm given), schur_opt 0 or 3 and rows within [0, n)\n");
   KernelSpec K;
   double* dXk = nullptr;
   const int additive = args_ok ? kernel_spec_of(fkernel_params, nullptr, kernel, n, K, &dXk) : -1;
   if (!agree(additive >= 0)) {
      (void)hipFree(dXk);
      return nullptr;
   }
   const int D = additive ? (K.nw - 1) * K.dw + K.last_dw : d;
   hipStream_t s = current_stream();
   const int n2 = n - k;
   const size_t kk = (size_t)k * k;
   double *dX = nullptr, *Xp = nullptr, *Xkp = nullptr, *K11 = nullptr, *G = nullptr, *Gt = nullptr, *K12 = nullptr;
   double *X2 = nullptr, *Xc = nullptr, *Ku = nullptr, *Wu = nullptr, *daa = nullptr;
   int *dperm = nullptr, *dinfo = nullptr, *didx = nullptr, *dia = nullptr, *dja = nullptr, *dwcol = nullptr;
   auto release = [&]() {
      (void)hipStreamSynchronize(s);
      for (void* p : {(void*)dX, (void*)Xp, (void*)Xkp, (void*)dXk, (void*)K11, (void*)X2, (void*)Xc, (void*)Ku,
                      (void*)Wu, (void*)daa, (void*)dperm, (void*)dinfo, (void*)didx, (void*)dia, (void*)dja,
                      (void*)dwcol})
         (void)hipFree(p);
   };
   auto fail = [&](const char* what) -> void* {
      if (what) fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnShardSetup: %s failed\n", what);
      release();
      for (void* p : {(void*)G, (void*)Gt, (void*)K12}) (void)hipFree(p);
      return nullptr;
   };
   // phase A (replicated): the ordering, K11 + noise and its Cholesky / inverse
   std::vector<int> hperm;
   auto phase_a = [&]() -> const char* {
   if (dalloc(&dX, (size_t)ldim * d)) return "allocation";
   const hipMemcpyKind kind = is_device_ptr(data) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
   if (hipMemcpy(dX, data, sizeof(double) * (size_t)ldim * d, kind) != hipSuccess) return "upload";
   // the ordering is computed by every rank alike (afn.c:196-256): FPS is deterministic, a given perm is shared
   hperm.resize(n);
   for (int i = 0; i < n; i++) hperm[i] = i;
   if (perm_opt == 1) {
      std::vector<int> sel(k);
      const int cnt = fps_device(dX, ldim, n, d, k, 0.0, sel.data(), nullptr, s);
      if (cnt < 0) return "FPS";
      hperm = expand_perm(sel.data(), cnt, n);
   } else if (perm_opt == 2) {
      hperm.assign(perm, perm + n);
   }
   if (dalloc(&dperm, n) || hipMemcpy(dperm, hperm.data(), sizeof(int) * n, hipMemcpyHostToDevice) != hipSuccess ||
       dalloc(&Xp, (size_t)n * d))
      return "allocation";
   hipLaunchKernelGGL(k_gather_points, dim3((n + 255) / 256, d), dim3(256), 0, s, dX, (long long)ldim, n, d, dperm, Xp);
   if (additive) {
      if (dalloc(&Xkp, (size_t)n * D)) return "allocation";
      hipLaunchKernelGGL(k_gather_points, dim3((n + 255) / 256, D), dim3(256), 0, s, dXk, (long long)n, n, D, dperm,
                         Xkp);
   }
   return (const char*)nullptr;
   };
   const char* err = phase_a();
   const double* Xk = additive ? Xkp : Xp;  // kernel coordinates in the permuted order, ld n
   KernelSpec Kp = K;
   Kp.Xk = additive ? Xkp : nullptr;
   Kp.ldk = n;
   const KernelParams P = kernel_params_of(Kp, d);
   // A11 = K(X1) + noise, L11^{-1}: replicated; every rank keeps rank 0's factors (afn.c:425-428)
   if (!err && (dalloc(&K11, kk) || dalloc(&G, kk) || dalloc(&Gt, kk) || dalloc(&dinfo, 1))) err = "allocation";
   int info = 0;
   if (!err) {
      hipLaunchKernelGGL(k_kmat, dim3((k + 255) / 256, k), dim3(256), 0, s, Xk, (long long)n, 0, k, 0, P, 1, K11,
                         (long long)k);
      info = chol_inverse_dev(K11, k, 0.0, G, Gt, dinfo, s);
      if (info > 0) {
         fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnShardSetup: K11 is not positive definite (column %d)\n", info);
         err = "";
      } else if (info < 0) {
         err = "Cholesky / triangular inverse of K11";
      }
   }
   if (err && *err) fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnShardSetup: %s failed\n", err);
   if (!agree(err == nullptr)) return fail(nullptr);
   if (comm->rank != 0 &&
       (hipMemsetAsync(G, 0, sizeof(double) * kk, s) != hipSuccess || hipMemsetAsync(Gt, 0, sizeof(double) * kk, s) != hipSuccess))
      return fail("broadcast");
   if (comm->allreduce(G, kk, s) || comm->allreduce(Gt, kk, s)) return fail("broadcast of L11^{-1}");
   // phase B (this rank's rows): its landmarks and Schur points, K12 at those points, the Schur FSAI's rows
   std::vector<int> lm_idx, lm_row, nl_pos, nl_row;
   std::vector<int> gia, gja;
   std::vector<double> gaa;
   auto phase_b = [&]() -> const char* {
   // fault injection for the tests (tests/test_gpu_dist.py): this rank's rows fail as a local breakdown would
   if (const char* e = getenv("NFFT4GP_AMD_FAULT_AFN_SHARD"))
      if (atoi(e) != 0) return "the fault injected by NFFT4GP_AMD_FAULT_AFN_SHARD";
   for (int p = 0; p < n; p++) {
      const int row = hperm[p];
      if (row < rb || row >= re) continue;
      if (p < k) {
         lm_idx.push_back(p);
         lm_row.push_back(row - rb);
      } else {
         nl_pos.push_back(p - k);
         nl_row.push_back(row - rb);
      }
   }
   const int m2 = (int)nl_pos.size();
   // kernel coordinates of [X1; the listed X2 points] (ld k + m), then K(X1, those points): k x m
   auto panel = [&](const std::vector<int>& pos, double* out) -> int {
      const int m = (int)pos.size();
      std::vector<int> idx(k + m);
      for (int a = 0; a < k; a++) idx[a] = a;
      for (int j = 0; j < m; j++) idx[k + j] = k + pos[j];
      (void)hipFree(Xc);
      (void)hipFree(didx);
      Xc = nullptr;
      didx = nullptr;
      if (dalloc(&Xc, (size_t)(k + m) * D) || dalloc(&didx, idx.size()) ||
          hipMemcpy(didx, idx.data(), sizeof(int) * idx.size(), hipMemcpyHostToDevice) != hipSuccess)
         return -1;
      hipLaunchKernelGGL(k_gather_points, dim3((k + m + 255) / 256, D), dim3(256), 0, s, Xk, (long long)n, k + m, D,
                         (const int*)didx, Xc);
      for (int j0 = 0; j0 < m; j0 += 65535) {
         const int nb = std::min(65535, m - j0);
         hipLaunchKernelGGL(k_kmat, dim3((k + 255) / 256, nb), dim3(256), 0, s, (const double*)Xc, (long long)(k + m), 0,
                            k, k + j0, P, 0, out + (size_t)j0 * k, (long long)k);
      }
      return hipGetLastError() == hipSuccess ? 0 : -1;
   };
   // K12 at this rank's Schur points only (afn.c:436): k x m2 instead of k x (n - k)
   if (dalloc(&K12, (size_t)k * std::max(1, m2)) || (m2 > 0 && panel(nl_pos, K12))) return "K12 panel";
   if (schur_opt == 3) {
      // FSAI of the Schur complement (afn.c:445-473) at this rank's rows: the KNN over their earlier points,
      // then the values in chunks of rows, each with W = L11^{-1} K12 formed for the columns it touches only
      if (dalloc(&X2, (size_t)n2 * d)) return "allocation";
      for (int c = 0; c < d; c++)
         if (hipMemcpyAsync(X2 + (size_t)c * n2, Xp + (size_t)c * n + k, sizeof(double) * n2, hipMemcpyDeviceToDevice,
                            s) != hipSuccess)
            return "copy";
      if (fsai_pattern_rows(X2, n2, n2, d, schur_lfil, nl_pos, gia, gja, s)) return "Schur FSAI pattern";
      const size_t nnz = gja.size();
      gaa.assign(nnz, 0.0);
      if (nnz > 0) {
         if (dalloc(&dia, gia.size()) || dalloc(&dja, nnz) || dalloc(&daa, nnz) || dalloc(&dwcol, nnz) ||
             hipMemcpy(dia, gia.data(), sizeof(int) * gia.size(), hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(dja, gja.data(), sizeof(int) * nnz, hipMemcpyHostToDevice) != hipSuccess)
            return "allocation";
         KernelSpec K2 = Kp;
         K2.Xk = additive ? Xkp + k : nullptr;  // column c of the Schur points: Xkp + c n + k + i
         constexpr int kMaxCols = 65536;        // W columns per chunk (k x 64 Ki doubles: 256 MB at k = 512)
         std::vector<int> U, wcol;
         std::vector<int> mark(n2, -1);
         int r0 = 0;
         while (r0 < m2) {
            // the chunk: rows while the union of their columns stays below kMaxCols
            U.clear();
            int r1 = r0;
            while (r1 < m2) {
               int add = 0;
               for (int e = gia[r1]; e < gia[r1 + 1]; e++) add += mark[gja[e]] < 0 ? 1 : 0;
               if (r1 > r0 && (int)U.size() + add > kMaxCols) break;
               for (int e = gia[r1]; e < gia[r1 + 1]; e++)
                  if (mark[gja[e]] < 0) {
                     mark[gja[e]] = (int)U.size();
                     U.push_back(gja[e]);
                  }
               r1++;
            }
            wcol.resize(gia[r1] - gia[r0]);
            for (int e = gia[r0]; e < gia[r1]; e++) wcol[e - gia[r0]] = mark[gja[e]];
            for (int j : U) mark[j] = -1;
            const size_t ku = (size_t)k * U.size();
            (void)hipFree(Ku);
            (void)hipFree(Wu);
            Ku = Wu = nullptr;
            if (dalloc(&Ku, ku) || dalloc(&Wu, ku) ||
                hipMemcpy(dwcol + gia[r0], wcol.data(), sizeof(int) * wcol.size(), hipMemcpyHostToDevice) != hipSuccess ||
                panel(U, Ku) || gemm_f64(false, k, (int)U.size(), k, G, k, Ku, k, Wu, k, s) ||
                fsai_values_rows(K2, X2, n2, d, schur_lfil, dia + r0, dja, r1 - r0, Wu, k, dwcol, daa, s))
               return "Schur FSAI values";
            r0 = r1;
         }
         if (hipMemcpyAsync(gaa.data(), daa, sizeof(double) * nnz, hipMemcpyDeviceToHost, s) != hipSuccess ||
             hipStreamSynchronize(s) != hipSuccess)
            return "copy";
         if (!std::all_of(gaa.begin(), gaa.end(), [](double v) { return std::isfinite(v); })) {
            return "the Schur complement's FSAI (a non-positive pivot)";
         }
      }
   } else {
      gia.assign(m2 + 1, 0);
   }
   return (const char*)nullptr;
   };
   err = phase_b();
   if (err) fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnShardSetup: %s failed\n", err);
   if (!agree(err == nullptr)) return fail(nullptr);
   release();
   // the apply object takes G, Gt and K12 (and frees them if it fails)
   void* S = afn_shard_from_parts(re - rb, k, n2, comm, lm_idx, lm_row, nl_pos, nl_row, G, Gt, K12, schur_opt == 3,
                                  schur_opt == 0 ? 1.0 / K.mu : 0.0, gia, gja, gaa);
   if (!agree(S != nullptr)) {
      if (S) Nfft4GPAmdDistAfnFree(S);
      return nullptr;
   }
   return S;
}
}  // namespace

extern "C" {

void* Nfft4GPAmdAfnSetupSchur(const double* data, int n, int ldim, int d, int k, int perm_opt, const int* perm,
                              int schur_opt, int schur_lfil, int kernel, void* fkernel_params)
{
   if (!need_device("Nfft4GPAmdAfnSetup")) return nullptr;
   bool breakdown = false;
   return afn_setup_impl(data, n, ldim, d, k, perm_opt, perm, schur_opt, schur_lfil, kernel, fkernel_params,
                         &breakdown);
}


// afn.c:161-489 split over row shards (the AFN apply of Nfft4GPAmdAfnShard, set up without a full AFN on any rank)
void* Nfft4GPAmdAfnShardSetup(const double* data, int n, int ldim, int d, int k, int perm_opt, const int* perm,
                              int schur_opt, int schur_lfil, int kernel, void* fkernel_params, int row_begin,
                              int row_end, void* comm)
{
   if (!need_device("Nfft4GPAmdAfnShardSetup")) return nullptr;
   return afn_shard_setup_impl(data, n, ldim, d, k, perm_opt, perm, schur_opt, schur_lfil, kernel, fkernel_params,
                               row_begin, row_end, (Comm*)comm);
}

int Nfft4GPAmdRankestNysScaled(const double* data, int n, int ldim, int d, int kernel, void* fkernel_params,
                               int max_rank, int nsample, int nsample_r)
{
   RandScope rand_scope;  // libc rand() as the reference draws it (internal.h)
   if (!need_device("Nfft4GPAmdRankestNysScaled")) return -1;
   RankCtx C;
   double *owned = nullptr, *owned_k = nullptr;
   if (rank_ctx(C, data, n, ldim, d, kernel, fkernel_params, &owned, &owned_k)) return -1;
   const int r = rankest_nys_scaled(C, max_rank, nsample, nsample_r);
   (void)hipFree(owned);
   (void)hipFree(owned_k);
   return r;
}

int Nfft4GPAmdRankestDefault(const double* data, int n, int ldim, int d, int kernel, void* fkernel_params,
                             int max_rank, int nsample, int nsample_r, double full_tol, int* perm)
{
   RandScope rand_scope;  // libc rand() as the reference draws it (internal.h)
   if (!need_device("Nfft4GPAmdRankestDefault")) return -1;
   RankCtx C;
   double *owned = nullptr, *owned_k = nullptr;
   if (rank_ctx(C, data, n, ldim, d, kernel, fkernel_params, &owned, &owned_k)) return -1;
   std::vector<int> p;
   const int r = rankest_default(C, max_rank, nsample, nsample_r, full_tol, p);
   (void)hipFree(owned);
   (void)hipFree(owned_k);
   if (r > 0 && perm) std::copy(p.begin(), p.end(), perm);
   return r;
}

int Nfft4GPAmdAfnRankEstimate(const double* data, int n, int ldim, int d, int max_k, int perm_opt, int nsamples,
                              int kernel, void* fkernel_params, int* perm)
{
   RandScope rand_scope;  // libc rand() as the reference draws it (internal.h)
   if (!need_device("Nfft4GPAmdAfnRankEstimate")) return -1;
   if (!perm) return -1;
   max_k = std::min(max_k, n);  // afn.c:167
   if (max_k <= 0) {            // afn.c:245-256: the predefined rank -max_k, natural order
      for (int i = 0; i < n; i++) perm[i] = i;
      return std::min(-max_k, n);
   }
   RankCtx C;
   double *owned = nullptr, *owned_k = nullptr;
   if (rank_ctx(C, data, n, ldim, d, kernel, fkernel_params, &owned, &owned_k)) return -1;
   int k = -1;
   std::vector<int> sel;
   const int rank = rankest_nys_scaled(C, max_k, nsamples, 5);  // _nsample_r = 5 (rankest.c:11)
   if (rank >= 0) {
      if (rank >= max_k) {  // afn.c:193-219: not low rank
         k = max_k;
         if (perm_opt == 1) {
            sel.assign(k, 0);
            k = fps_device(C.dX, C.ldim, n, d, k, 0.0, sel.data(), nullptr, C.s);
            if (k >= 0) sel.resize(k);
         } else {
            sel = rand_perm(n, k);
         }
      } else {  // afn.c:220-242
         k = rankest_default(C, max_k, nsamples, 5, 0.9, sel);
         if (k == max_k && perm_opt == 0) sel = rand_perm(n, k);
      }
   }
   (void)hipFree(owned);
   (void)hipFree(owned_k);
   if (k < 0) return -1;
   const std::vector<int> full = expand_perm(sel.data(), (int)sel.size(), n);
   std::copy(full.begin(), full.end(), perm);
   return k;
}


/* Nfft4GPPrecondAFNSetup (afn.c:161-489): the rank estimation and ordering (Nfft4GPAmdAfnRankEstimate), then
 *   k == 0 or k == n, or k == max_k: the AFN (Nfft4GPAmdAfnSetupSchur with that k and order);
 *   0 < k < max_k: the rank-k Nystrom on those landmarks instead (afn.c:294-304, afn_setup.m:80-83);
 *   the AFN's factors break down (K11 not positive definite, or the Schur FSAI meets a non-positive pivot):
 *   the Nystrom on the same order, MATLAB's RAN fallback (afn_setup.m:93-98).
 * With require_grad the AFN keeps its gradient pieces (afn_grad.hip) and the Nystrom branches are the
 * Nystrom-with-gradients of nys_grad.hip (an additive handle of this library as kernel data). */
struct AfnFlow {
   // parameters (Nfft4GPAmdPrecondAFNCreate)
   int max_k = 0, perm_opt = 0, schur_opt = 3, schur_lfil = 20, nsamples = 500;
   // what the last setup built
   // 0 AFN, 1 Nystrom (rank below max_k), 2 Nystrom after an AFN breakdown (RAN); with gradients the AFN's
   // k = 0 / k = n branches (afn.c:263-284) as their exact equivalents: 3 the FSAI of the whole kernel
   // (k = 0), 4 the rank-n Nystrom, which is K + mu f^2 I itself (k = n)
   int kind = 0;
   int k = 0;
   int n = 0;
   void* afn = nullptr;
   NysDev* nys = nullptr;     // Nystrom branches without gradients
   void* nysg = nullptr;      // Nystrom branches with gradients (Nfft4GPAmdPrecondNys* handle)
   AfnGrad* grad = nullptr;   // the AFN's gradient pieces
   void* fsaig = nullptr;     // kind 3 (Nfft4GPAmdPrecondFsai* handle with gradients)
   void reset()
   {
      if (grad) afn_grad_free(grad);
      if (fsaig) Nfft4GPAmdPrecondFsaiFree(fsaig);
      fsaig = nullptr;
      if (afn) Nfft4GPAmdAfnFree(afn);
      if (nys) Nfft4GPAmdNysFree(nys);
      if (nysg) Nfft4GPAmdPrecondNysFree(nysg);
      grad = nullptr;
      afn = nullptr;
      nys = nullptr;
      nysg = nullptr;
      kind = k = n = 0;
   }
};

static NysDev* flow_nystrom(const double* data, int n, int ldim, int d, int kernel, void* fkernel_params,
                            const int* perm, int k)
{
   KernelSpec K;
   double* owned = nullptr;
   const int additive = kernel_spec_of(fkernel_params, nullptr, kernel, n, K, &owned);
   (void)hipFree(owned);
   if (additive < 0) return nullptr;
   if (additive) return (NysDev*)Nfft4GPAmdNysSetupAdditive(fkernel_params, perm, k, 1);
   // the plain kernel of all d features is the additive kernel of one d-feature window (weight 1)
   std::vector<double> xw((size_t)n * d);
   for (int c = 0; c < d; c++) {
      const hipMemcpyKind kind = is_device_ptr(data) ? hipMemcpyDeviceToHost : hipMemcpyHostToHost;
      if (hipMemcpy(xw.data() + (size_t)c * n, data + (size_t)c * ldim, sizeof(double) * n, kind) != hipSuccess)
         return nullptr;
   }
   return nys_setup_additive(xw.data(), n, 1, d, 0, kernel, K.f, K.l, K.mu, perm, k, 1);
}

// the Nystrom with gradients on the landmarks perm[:k] (nys.c:518-660 restated, K11 on the landmarks)
static void* flow_nystrom_grad(double* data, int n, int ldim, int d, int kernel, void* fkernel_params, int* perm,
                               int k)
{
   KernelSpec K;
   double* owned = nullptr;
   const int additive = kernel_spec_of(fkernel_params, nullptr, kernel, n, K, &owned);
   (void)hipFree(owned);
   if (additive != 1) {
      fprintf(stderr, "nfft4gp_amd: the AFN's Nystrom branch with gradients needs this library's additive handle as "
                      "kernel data\n");
      return nullptr;
   }
   void* N = Nfft4GPAmdPrecondNysCreate();
   Nfft4GPAmdPrecondNysSetRank(N, k);
   Nfft4GPAmdPrecondNysSetPerm(N, perm, 0);
   Nfft4GPAmdPrecondNysSetK11Mode(N, 1);
   func_kernel fk = K.kernel ? &Nfft4GPNFFTAdditiveKernelMatern12Kernel : &Nfft4GPNFFTAdditiveKernelGaussianKernel;
   if (Nfft4GPAmdPrecondNysSetupWithKernel(data, n, ldim, d, fk, fkernel_params, 1, N)) {
      Nfft4GPAmdPrecondNysFree(N);
      return nullptr;
   }
   return N;
}

// the FSAI with gradients of the whole kernel (the AFN at k = 0 with its Schur FSAI, schur_opt 3)
static void* flow_fsai_grad(double* data, int n, int ldim, int d, int kernel, void* fkernel_params, int lfil)
{
   void* S = Nfft4GPAmdPrecondFsaiCreate();
   Nfft4GPAmdPrecondFsaiSetLfil(S, lfil);
   Nfft4GPAmdPrecondFsaiSetKernel(S, kernel);
   func_kernel fk = kernel ? &Nfft4GPNFFTAdditiveKernelMatern12Kernel : &Nfft4GPNFFTAdditiveKernelGaussianKernel;
   if (Nfft4GPAmdPrecondFsaiSetupWithKernel(data, n, ldim, d, fk, fkernel_params, 1, S)) {
      Nfft4GPAmdPrecondFsaiFree(S);
      return nullptr;
   }
   return S;
}

static int flow_setup(AfnFlow* F, double* data, int n, int ldim, int d, int kernel, void* fkernel_params, int grad)
{
   F->reset();
   std::vector<int> perm(n);
   const int max_kk = std::min(F->max_k, n);
   const int k = Nfft4GPAmdAfnRankEstimate(data, n, ldim, d, F->max_k, F->perm_opt, F->nsamples, kernel,
                                           fkernel_params, perm.data());
   if (k < 0) return -1;
   F->n = n;
   F->k = k;
   auto nystrom = [&](int kind) {
      F->kind = kind;
      if (grad)
         F->nysg = flow_nystrom_grad(data, n, ldim, d, kernel, fkernel_params, perm.data(), k);
      else
         F->nys = flow_nystrom(data, n, ldim, d, kernel, fkernel_params, perm.data(), k);
   };
   if (max_kk > 0 && k > 0 && k < n && k < max_kk) {
      printf("The estimated rank %d is below max_k = %d: rank-%d Nystrom (afn.c:294-304)\n", k, max_kk, k);
      nystrom(1);
   } else if (grad && k >= n) {
      // M = K11 + mu f^2 I = K + mu f^2 I (afn.c:263-272); the rank-n Nystrom is the same matrix and has
      // gradients (nys_grad.hip)
      nystrom(4);
   } else if (grad && k == 0 && F->schur_opt == 3) {
      // M^{-1} = G^T G, the FSAI of the whole kernel (afn.c:274-284); fsai_setup.hip has its gradients
      F->kind = 3;
      F->fsaig = flow_fsai_grad(data, n, ldim, d, kernel, fkernel_params, F->schur_lfil);
   } else {
      bool breakdown = false;
      F->afn = afn_setup_impl(data, n, ldim, d, k, 2, perm.data(), F->schur_opt, F->schur_lfil, kernel,
                              fkernel_params, &breakdown, grad ? &F->grad : nullptr);
      if (!F->afn && breakdown && k > 0 && k < n) {
         printf("AFN factors broke down: rank-%d Nystrom on the same order (afn_setup.m:93-98)\n", k);
         nystrom(2);
      }
   }
   if (!F->afn && !F->nys && !F->nysg && !F->fsaig) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdPrecondAFNSetup failed\n");
      return -1;
   }
   return 0;
}

void* Nfft4GPAmdPrecondAFNCreate(int max_k, int perm_opt, int schur_opt, int schur_lfil, int nsamples)
{
   if ((perm_opt != 0 && perm_opt != 1) || (schur_opt != 0 && schur_opt != 3)) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdPrecondAFNCreate: perm_opt 0 (random) or 1 (FPS), schur_opt 0 or 3\n");
      return nullptr;
   }
   AfnFlow* F = new AfnFlow();
   F->max_k = max_k;
   F->perm_opt = perm_opt;
   F->schur_opt = schur_opt;
   F->schur_lfil = schur_lfil;
   F->nsamples = nsamples;
   return F;
}

int Nfft4GPAmdPrecondAFNSetupWithKernel(double* data, int n, int ldim, int d, func_kernel fkernel,
                                        void* fkernel_params, int require_grad, void* pre)
{
   RandScope rand_scope;  // libc rand() as the reference draws it (internal.h)
   if (!need_device("Nfft4GPAmdPrecondAFNSetupWithKernel")) return -1;
   AfnFlow* F = (AfnFlow*)pre;
   if (!F || !data || !fkernel_params || n <= 0 || ldim < n) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdPrecondAFNSetupWithKernel needs a handle, data (ldim >= n) and kernel "
                      "parameters\n");
      return -1;
   }
   const int kernel = fkernel == &Nfft4GPNFFTAdditiveKernelMatern12Kernel ? 1 : 0;
   return flow_setup(F, data, n, ldim, d, kernel, fkernel_params, require_grad ? 1 : 0);
}

void* Nfft4GPAmdPrecondAFNSetup(const double* data, int n, int ldim, int d, int max_k, int perm_opt, int schur_opt,
                                int schur_lfil, int nsamples, int kernel, void* fkernel_params, int require_grad)
{
   RandScope rand_scope;  // libc rand() as the reference draws it (internal.h)
   if (!need_device("Nfft4GPAmdPrecondAFNSetup")) return nullptr;
   if (!data || !fkernel_params || n <= 0 || ldim < n) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdPrecondAFNSetup needs data (ldim >= n) and kernel parameters\n");
      return nullptr;
   }
   AfnFlow* F = (AfnFlow*)Nfft4GPAmdPrecondAFNCreate(max_k, perm_opt, schur_opt, schur_lfil, nsamples);
   if (!F) return nullptr;
   if (flow_setup(F, const_cast<double*>(data), n, ldim, d, kernel, fkernel_params, require_grad ? 1 : 0)) {
      delete F;
      return nullptr;
   }
   return F;
}

int Nfft4GPAmdPrecondAFNSolve(void* pre, int n, double* x, double* rhs)
{
   AfnFlow* F = (AfnFlow*)pre;
   if (!F || n != F->n) return -1;
   if (F->afn) return Nfft4GPAmdAfnSolve(F->afn, n, x, rhs);
   if (F->nysg) return Nfft4GPAmdPrecondNysSolve(F->nysg, n, x, rhs);
   if (F->fsaig) return Nfft4GPAmdPrecondFsaiSolve(F->fsaig, n, x, rhs);
   return Nfft4GPAmdNysSolve(F->nys, n, x, rhs);
}

int Nfft4GPAmdPrecondAFNSetStorage(void* pre, int bits)
{
   AfnFlow* F = (AfnFlow*)pre;
   if (!F || (bits != 32 && bits != 64)) return -1;
   // with gradients the fp64 factors serve Dvp, Trace and Logdet: an fp32 solve would no longer be the
   // preconditioner those terms describe, so the storage stays fp64
   if (F->grad) return 0;
   if (F->afn) return Nfft4GPAmdAfnSetStorage(F->afn, bits);
   if (F->nys) return Nfft4GPAmdNysSetStorage(F->nys, bits);
   return 0;  // the gradient-capable branches keep their fp64 factors
}

int Nfft4GPAmdPrecondAFNDvp(void* pre, int n, int* mask, double* x, double** yp)
{
   AfnFlow* F = (AfnFlow*)pre;
   if (!F || n != F->n || !yp) return -1;
   if (F->nysg) return Nfft4GPAmdPrecondNysDvp(F->nysg, n, mask, x, yp);
   if (F->fsaig) return Nfft4GPAmdPrecondFsaiDvp(F->fsaig, n, mask, x, yp);
   if (!F->grad) {
      printf("Setup AFN without gradient, dvp not supported.\n");
      return -1;
   }
   // host or device x; *yp allocated on x's side when NULL (the reference's convention)
   hipStream_t s = current_stream();
   const bool xd = is_device_ptr(x);
   if (!*yp) {
      if (xd)
         NFFT4GP_HIP_CHECK(hipMalloc((void**)yp, sizeof(double) * 3 * (size_t)n));
      else
         *yp = (double*)calloc(3 * (size_t)n, sizeof(double));
   }
   const bool yd = is_device_ptr(*yp);
   double *dx = x, *dy = *yp;
   if (!xd) {
      NFFT4GP_HIP_CHECK(hipMalloc((void**)&dx, sizeof(double) * n));
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(dx, x, sizeof(double) * n, hipMemcpyHostToDevice, s));
   }
   if (!yd) NFFT4GP_HIP_CHECK(hipMalloc((void**)&dy, sizeof(double) * 3 * (size_t)n));
   int rc = afn_grad_dvp(F->grad, mask, dx, dy, s);
   if (!yd) {
      if (!rc && hipMemcpyAsync(*yp, dy, sizeof(double) * 3 * (size_t)n, hipMemcpyDeviceToHost, s) != hipSuccess) rc = -1;
      (void)hipStreamSynchronize(s);
      (void)hipFree(dy);
   }
   if (!xd) {
      (void)hipStreamSynchronize(s);
      (void)hipFree(dx);
   }
   return rc;
}

int Nfft4GPAmdPrecondAFNTrace(void* pre, double** tracesp)
{
   AfnFlow* F = (AfnFlow*)pre;
   if (!F || !tracesp) return -1;
   if (F->nysg) return Nfft4GPAmdPrecondNysTrace(F->nysg, tracesp);
   if (F->fsaig) return Nfft4GPAmdPrecondFsaiTrace(F->fsaig, tracesp);
   if (!F->grad) {
      printf("Setup AFN without gradient, trace not supported.\n");
      return -1;
   }
   if (!*tracesp) *tracesp = (double*)calloc(3, sizeof(double));
   for (int g = 0; g < 3; g++) (*tracesp)[g] = F->grad->trace[g];
   return 0;
}

double Nfft4GPAmdPrecondAFNLogdet(void* pre)
{
   AfnFlow* F = (AfnFlow*)pre;
   if (!F) return NAN;
   if (F->nysg) return Nfft4GPAmdPrecondNysLogdet(F->nysg);
   if (F->fsaig) return Nfft4GPAmdPrecondFsaiLogdet(F->fsaig);
   return F->grad ? F->grad->logdet : NAN;
}

void Nfft4GPAmdPrecondAFNReset(void* pre)
{
   if (pre) ((AfnFlow*)pre)->reset();
}

int Nfft4GPAmdPrecondAFNInfo(void* pre, int* kind, int* k, void** afn, void** nys)
{
   AfnFlow* F = (AfnFlow*)pre;
   if (!F) return -1;
   if (kind) *kind = F->kind;
   if (k) *k = F->k;
   if (afn) *afn = F->afn;
   if (nys) *nys = F->nys ? (void*)F->nys : F->nysg;
   return 0;
}

void Nfft4GPAmdPrecondAFNFree(void* pre)
{
   AfnFlow* F = (AfnFlow*)pre;
   if (!F) return;
   F->reset();
   delete F;
}

}  // extern "C"
