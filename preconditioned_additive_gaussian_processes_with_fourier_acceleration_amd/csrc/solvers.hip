// solvers.hip -- device-resident BLAS-1 vector ops, PCG and the Nystrom preconditioner apply.
//
//   Nfft4GPVec*          SRC/linearalg/vecops.c:3-155   (host or device pointers; GPU compute)
//   Nfft4GPSolverPcg     SRC/solvers/pcg.c:3-206        (same control flow, breakdown tests,
//                                                       true-residual recheck and reporting quirks)
//   Nfft4GPAmdNys*       SRC/preconds/nys.c:115-173     (x = M^{-1} rhs, M = U S U^T + eta I)
//
// Reductions are two-stage and fixed-order (bitwise reproducible run to run).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "internal.h"

using namespace nfft4gp_amd;

namespace {

constexpr int kVecThreads = 256;
constexpr int kMaxRedBlocks = 1024;

__global__ __launch_bounds__(kVecThreads) void k_dot_partial(const double* __restrict__ x,
                                                             const double* __restrict__ y, size_t n,
                                                             double* __restrict__ part)
{
   __shared__ double s[kVecThreads / 64];
   double acc = 0.0;
   for (size_t i = (size_t)blockIdx.x * kVecThreads + threadIdx.x; i < n; i += (size_t)gridDim.x * kVecThreads)
      acc = fma(x[i], y[i], acc);
   for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
   if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
   __syncthreads();
   if (threadIdx.x == 0) {
      double v = 0.0;
      for (int w = 0; w < kVecThreads / 64; w++) v += s[w];
      part[blockIdx.x] = v;
   }
}

__global__ __launch_bounds__(kVecThreads) void k_sum_final(const double* __restrict__ part, int np,
                                                           double* __restrict__ out)
{
   __shared__ double s[kVecThreads / 64];
   double acc = 0.0;
   for (int i = threadIdx.x; i < np; i += kVecThreads) acc += part[i];
   for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
   if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
   __syncthreads();
   if (threadIdx.x == 0) {
      double v = 0.0;
      for (int w = 0; w < kVecThreads / 64; w++) v += s[w];
      *out = v;
   }
}

__global__ void k_fill(double* __restrict__ x, size_t n, double v)
{
   for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
      x[i] = v;
}

__global__ void k_scale(double* __restrict__ x, size_t n, double a)
{
   for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
      x[i] *= a;
}

__global__ void k_axpy(double a, const double* __restrict__ x, size_t n, double* __restrict__ y)
{
   for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
      y[i] += a * x[i];
}

// p = beta*p + z  (pcg.c:145-146: Scale then Axpy)
__global__ void k_pupdate(double* __restrict__ p, const double* __restrict__ z, size_t n, double beta)
{
   for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
      const double t = beta * p[i];
      p[i] = t + z[i];
   }
}

// x += a p ; r -= a q ; partial ||r||^2   (pcg.c:168-172 fused into one pass)
__global__ __launch_bounds__(kVecThreads) void k_xr_update(double* __restrict__ x, double* __restrict__ r,
                                                           const double* __restrict__ p,
                                                           const double* __restrict__ q, size_t n, double a,
                                                           double* __restrict__ part)
{
   __shared__ double s[kVecThreads / 64];
   double acc = 0.0;
   for (size_t i = (size_t)blockIdx.x * kVecThreads + threadIdx.x; i < n; i += (size_t)gridDim.x * kVecThreads) {
      x[i] += a * p[i];
      const double ri = r[i] + (-a) * q[i];
      r[i] = ri;
      acc = fma(ri, ri, acc);
   }
   for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
   if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
   __syncthreads();
   if (threadIdx.x == 0) {
      double v = 0.0;
      for (int w = 0; w < kVecThreads / 64; w++) v += s[w];
      part[blockIdx.x] = v;
   }
}

int grid_for(size_t n)
{
   size_t g = (n + kVecThreads - 1) / kVecThreads;
   if (g > (size_t)kMaxRedBlocks) g = kMaxRedBlocks;
   return (int)(g == 0 ? 1 : g);
}

// scratch for reductions (per process; the library is single-threaded per stream like the
// reference, whose handles are not re-entrant)
struct RedScratch {
   double* part = nullptr;
   double* res = nullptr;
   double* host = nullptr;
   int ensure()
   {
      if (!part) {
         NFFT4GP_HIP_CHECK(hipMalloc((void**)&part, sizeof(double) * kMaxRedBlocks));
         NFFT4GP_HIP_CHECK(hipMalloc((void**)&res, sizeof(double) * 4));
         NFFT4GP_HIP_CHECK(hipHostMalloc((void**)&host, sizeof(double) * 4));
      }
      return 0;
   }
};
RedScratch g_red;

int dev_dot(const double* x, const double* y, size_t n, double* out)
{
   if (g_red.ensure()) return -1;
   hipStream_t s = current_stream();
   const int g = grid_for(n);
   hipLaunchKernelGGL(k_dot_partial, dim3(g), dim3(kVecThreads), 0, s, x, y, n, g_red.part);
   hipLaunchKernelGGL(k_sum_final, dim3(1), dim3(kVecThreads), 0, s, g_red.part, g, g_red.res);
   NFFT4GP_HIP_CHECK(hipMemcpyAsync(g_red.host, g_red.res, sizeof(double), hipMemcpyDeviceToHost, s));
   NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
   *out = g_red.host[0];
   return 0;
}

int elem_grid(size_t n)
{
   size_t g = (n + 255) / 256;
   if (g > 4096) g = 4096;
   return (int)(g == 0 ? 1 : g);
}

// host-or-device view of a vector: host pointers are staged through device memory
struct Vec {
   double* d = nullptr;
   double* h = nullptr;
   size_t n = 0;
   bool staged = false;
   int open(double* p, size_t nn, bool copy_in)
   {
      n = nn;
      if (is_device_ptr(p)) {
         d = p;
         return 0;
      }
      h = p;
      staged = true;
      NFFT4GP_HIP_CHECK(hipMalloc((void**)&d, sizeof(double) * (n ? n : 1)));
      if (copy_in && n) NFFT4GP_HIP_CHECK(hipMemcpy(d, h, sizeof(double) * n, hipMemcpyHostToDevice));
      return 0;
   }
   int close(bool copy_out)
   {
      if (staged) {
         hipStream_t s = current_stream();
         NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
         if (copy_out && n) NFFT4GP_HIP_CHECK(hipMemcpy(h, d, sizeof(double) * n, hipMemcpyDeviceToHost));
         NFFT4GP_HIP_CHECK(hipFree(d));
         d = nullptr;
      }
      return 0;
   }
};

bool need_device(const char* who)
{
   if (!device_ok()) {
      fprintf(stderr, "nfft4gp_amd: %s: no HIP device visible (no CPU fallback).\n", who);
      return false;
   }
   return true;
}

// ---------------------------------------------------------------------------------------------
// Nystrom apply kernels
// ---------------------------------------------------------------------------------------------
constexpr int kNysRows = 2048;   // rows per workgroup in U^T r
constexpr int kNysThreads = 256;

// partial[blk][j] = sum_{i in blk rows} U[i, j] r[i]; one wave per column at a time, the block's
// r segment kept in registers (kNysRows/64 = 32 values per lane)
__global__ __launch_bounds__(kNysThreads) void k_nys_ut(const double* __restrict__ U, size_t ldu, int n, int k,
                                                       const double* __restrict__ r, double* __restrict__ part)
{
   constexpr int kPer = kNysRows / 64;
   const int lane = threadIdx.x & 63;
   const int wave = threadIdx.x >> 6;
   const int nw = kNysThreads / 64;
   const size_t r0 = (size_t)blockIdx.x * kNysRows;
   double rv[kPer];
#pragma unroll
   for (int t = 0; t < kPer; t++) {
      const size_t i = r0 + (size_t)t * 64 + lane;
      rv[t] = (i < (size_t)n) ? r[i] : 0.0;
   }
   for (int j = wave; j < k; j += nw) {
      const double* col = U + (size_t)j * ldu;
      double acc = 0.0;
#pragma unroll
      for (int t = 0; t < kPer; t++) {
         const size_t i = r0 + (size_t)t * 64 + lane;
         if (i < (size_t)n) acc = fma(col[i], rv[t], acc);
      }
      for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
      if (lane == 0) part[(size_t)blockIdx.x * k + j] = acc;
   }
}

// w[j] = (s[j] - 1/eta) * sum_blk part[blk][j]
__global__ void k_nys_w(const double* __restrict__ part, int nblk, int k, const double* __restrict__ s, double eta,
                        double* __restrict__ w)
{
   const int j = blockIdx.x * blockDim.x + threadIdx.x;
   if (j >= k) return;
   double z = 0.0;
   for (int b = 0; b < nblk; b++) z += part[(size_t)b * k + j];
   w[j] = s[j] * z - z / eta;
}

// x[i] = r[i]/eta + sum_j U[i, j] w[j]
__global__ __launch_bounds__(kNysThreads) void k_nys_u(const double* __restrict__ U, size_t ldu, int n, int k,
                                                      const double* __restrict__ w, const double* __restrict__ r,
                                                      double eta, double* __restrict__ x)
{
   extern __shared__ double s_w[];
   for (int j = threadIdx.x; j < k; j += blockDim.x) s_w[j] = w[j];
   __syncthreads();
   const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
   if (i >= (size_t)n) return;
   double acc = 0.0;
   for (int j = 0; j < k; j++) acc = fma(U[(size_t)j * ldu + i], s_w[j], acc);
   x[i] = r[i] / eta + acc;
}

struct NysDev {
   int n = 0, k = 0;
   double eta = 0.0;
   double* U = nullptr;  // natural row order
   double* s = nullptr;
   double* w = nullptr;
   double* part = nullptr;
   int nblk = 0;
};

int g_last_hist_len = 0;

}  // namespace

extern "C" {

int Nfft4GPAmdPcgHistoryLength(void) { return g_last_hist_len; }

double Nfft4GPVecDdot(double* x, int n, double* y)
{
   if (!need_device("Nfft4GPVecDdot")) return NAN;
   Vec vx, vy;
   double out = NAN;
   if (vx.open(x, n, true) || vy.open(y, n, true)) return NAN;
   if (dev_dot(vx.d, vy.d, (size_t)n, &out)) out = NAN;
   vx.close(false);
   vy.close(false);
   return out;
}

double Nfft4GPVecNorm2(double* x, int n)
{
   return std::sqrt(Nfft4GPVecDdot(x, n, x));
}

void Nfft4GPVecFill(double* x, size_t n, double val)
{
   if (!need_device("Nfft4GPVecFill")) return;
   Vec v;
   if (v.open(x, n, false)) return;
   hipLaunchKernelGGL(k_fill, dim3(elem_grid(n)), dim3(256), 0, current_stream(), v.d, n, val);
   v.close(true);
}

void Nfft4GPVecScale(double* x, size_t n, double scale)
{
   if (scale == 0.0) {  // vecops.c:74-77
      Nfft4GPVecFill(x, n, 0.0);
      return;
   }
   if (!need_device("Nfft4GPVecScale")) return;
   Vec v;
   if (v.open(x, n, true)) return;
   hipLaunchKernelGGL(k_scale, dim3(elem_grid(n)), dim3(256), 0, current_stream(), v.d, n, scale);
   v.close(true);
}

void Nfft4GPVecAxpy(double alpha, double* x, size_t n, double* y)
{
   if (alpha == 0.0) return;  // vecops.c:107-110
   if (!need_device("Nfft4GPVecAxpy")) return;
   Vec vx, vy;
   if (vx.open(x, n, true) || vy.open(y, n, true)) return;
   hipLaunchKernelGGL(k_axpy, dim3(elem_grid(n)), dim3(256), 0, current_stream(), alpha, vx.d, n, vy.d);
   vx.close(false);
   vy.close(true);
}

int Nfft4GPSolverPcg(void* mat_data, int n, func_symmatvec matvec, void* prec_data, func_solve precondfunc,
                     double* x, double* rhs, int maxits, int atol, double tol, double* prel_res, double** prel_res_v,
                     int* piter, int print_level)
{
   if (!need_device("Nfft4GPSolverPcg")) return -1;
   hipStream_t s = current_stream();
   const size_t N = (size_t)n;
   Vec vx, vb;
   if (vx.open(x, N, true) || vb.open(rhs, N, true)) return -1;
   double *r = nullptr, *z = nullptr, *p = nullptr, *q = nullptr;
   int iter = 0, ii;
   double rho = 1.0, alpha, beta, normb, normr, normr2, tolb;
   double* rel_res_v = nullptr;
   const double EPSILON = DBL_EPSILON;
   if (g_red.ensure()) return -1;

   auto cleanup = [&](bool copy_x) {
      if (r) (void)hipFree(r);
      if (z) (void)hipFree(z);
      if (p) (void)hipFree(p);
      if (q) (void)hipFree(q);
      vx.close(copy_x);
      vb.close(false);
   };

   if (dev_dot(vb.d, vb.d, N, &normb)) return -1;
   normb = std::sqrt(normb);
   if (normb < EPSILON) {  // pcg.c:32-41
      hipLaunchKernelGGL(k_fill, dim3(elem_grid(N)), dim3(256), 0, s, vx.d, N, 0.0);
      *prel_res = 0.0;
      *piter = 0;
      rel_res_v = (double*)calloc(1, sizeof(double));
      *prel_res_v = rel_res_v;
      g_last_hist_len = 1;
      cleanup(true);
      return 0;
   }
   tolb = atol ? tol : tol * normb;
   if (maxits > n) maxits = n;

   NFFT4GP_HIP_CHECK(hipMalloc((void**)&r, sizeof(double) * N));
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&z, sizeof(double) * N));
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&p, sizeof(double) * N));
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&q, sizeof(double) * N));

   NFFT4GP_HIP_CHECK(hipMemcpyAsync(r, vb.d, sizeof(double) * N, hipMemcpyDeviceToDevice, s));
   if (matvec(mat_data, n, -1.0, vx.d, 1.0, r)) {
      cleanup(false);
      return -1;
   }
   if (dev_dot(r, r, N, &normr)) return -1;
   normr = std::sqrt(normr);
   if (normr < tolb) {  // pcg.c:70-84
      *prel_res = normr / normb;
      *piter = 0;
      rel_res_v = (double*)malloc(sizeof(double));
      rel_res_v[0] = *prel_res;
      *prel_res_v = rel_res_v;
      g_last_hist_len = 1;
      cleanup(true);
      return 0;
   }
   normr2 = normr;
   rel_res_v = (double*)calloc((size_t)maxits + 1, sizeof(double));
   g_last_hist_len = maxits + 1;
   rel_res_v[0] = normr / normb;
   if (print_level > 0) {
      printf("--------------------------------------------------------------------------------\n");
      printf("Start PCG\n");
      printf("Residual Tol: %e\nMax number of iterations: %d\n", tolb, maxits);
      printf("--------------------------------------------------------------------------------\n");
      printf("Step    Residual norm  Relative res.  Convergence Rate\n");
      printf("%5d   %8e   %8e   N/A\n", 0, normr, rel_res_v[0]);
   }
   const int g = grid_for(N);
   for (ii = 1; ii <= maxits; ii++) {
      if (prec_data) {
         if (precondfunc(prec_data, n, z, r)) break;
      } else {
         NFFT4GP_HIP_CHECK(hipMemcpyAsync(z, r, sizeof(double) * N, hipMemcpyDeviceToDevice, s));
      }
      const double rho1 = rho;
      if (dev_dot(z, r, N, &rho)) break;
      if (rho == 0.0) {
         if (print_level > 1) printf("rho = %.16e\n", rho);
         break;
      }
      if (ii == 1) {
         NFFT4GP_HIP_CHECK(hipMemcpyAsync(p, z, sizeof(double) * N, hipMemcpyDeviceToDevice, s));
      } else {
         beta = rho / rho1;
         if (beta == 0.0) {
            if (print_level > 1) printf("beta = %.16e\n", beta);
            break;
         }
         hipLaunchKernelGGL(k_pupdate, dim3(elem_grid(N)), dim3(256), 0, s, p, z, N, beta);
      }
      if (matvec(mat_data, n, 1.0, p, 0.0, q)) break;
      double pq;
      if (dev_dot(q, p, N, &pq)) break;
      if (pq <= 0) {
         if (print_level > 1) printf("pq = %.16e\n", pq);
         break;
      }
      alpha = rho / pq;
      hipLaunchKernelGGL(k_xr_update, dim3(g), dim3(kVecThreads), 0, s, vx.d, r, p, q, N, alpha, g_red.part);
      hipLaunchKernelGGL(k_sum_final, dim3(1), dim3(kVecThreads), 0, s, g_red.part, g, g_red.res);
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(g_red.host, g_red.res, sizeof(double), hipMemcpyDeviceToHost, s));
      NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
      normr = std::sqrt(g_red.host[0]);
      normr2 = normr;
      rel_res_v[ii] = normr / normb;
      if (print_level > 0)
         printf("%5d   %8e   %8e   %8.6f\n", ii, normr, rel_res_v[ii], rel_res_v[ii] / rel_res_v[ii - 1]);
      if (normr <= tolb) {  // pcg.c:181-193: true residual recheck
         NFFT4GP_HIP_CHECK(hipMemcpyAsync(r, vb.d, sizeof(double) * N, hipMemcpyDeviceToDevice, s));
         if (matvec(mat_data, n, -1.0, vx.d, 1.0, r)) break;
         if (dev_dot(r, r, N, &normr2)) break;
         normr2 = std::sqrt(normr2);
         rel_res_v[ii] = normr2;
         if (normr2 <= tolb) {
            iter = ii;
            break;
         }
      }
   }
   *prel_res = normr2 / normb;
   *piter = iter;
   *prel_res_v = rel_res_v;
   cleanup(true);
   return 0;
}

void* Nfft4GPAmdNysCreate(int n, int k, const double* U, const double* s, double eta, const int* perm)
{
   if (!need_device("Nfft4GPAmdNysCreate")) return nullptr;
   NysDev* N = new NysDev();
   N->n = n;
   N->k = k;
   N->eta = eta;
   // rows of the reference's U are in permuted order (nys.c:127-133); store U in natural order
   std::vector<double> hU((size_t)n * k);
   const bool dU = is_device_ptr(U);
   std::vector<double> src;
   const double* Uh = U;
   if (dU) {
      src.resize((size_t)n * k);
      if (hipMemcpy(src.data(), U, sizeof(double) * src.size(), hipMemcpyDeviceToHost) != hipSuccess) return nullptr;
      Uh = src.data();
   }
   for (int j = 0; j < k; j++)
      for (int i = 0; i < n; i++) {
         const int dst = perm ? perm[i] : i;
         hU[(size_t)j * n + dst] = Uh[(size_t)j * n + i];
      }
   std::vector<double> hs(k);
   if (is_device_ptr(s)) {
      if (hipMemcpy(hs.data(), s, sizeof(double) * k, hipMemcpyDeviceToHost) != hipSuccess) return nullptr;
   } else {
      memcpy(hs.data(), s, sizeof(double) * k);
   }
   N->nblk = (n + kNysRows - 1) / kNysRows;
   if (hipMalloc((void**)&N->U, sizeof(double) * hU.size()) != hipSuccess ||
       hipMalloc((void**)&N->s, sizeof(double) * k) != hipSuccess ||
       hipMalloc((void**)&N->w, sizeof(double) * k) != hipSuccess ||
       hipMalloc((void**)&N->part, sizeof(double) * (size_t)N->nblk * k) != hipSuccess) {
      fprintf(stderr, "nfft4gp_amd: Nystrom allocation failed\n");
      return nullptr;
   }
   (void)hipMemcpy(N->U, hU.data(), sizeof(double) * hU.size(), hipMemcpyHostToDevice);
   (void)hipMemcpy(N->s, hs.data(), sizeof(double) * k, hipMemcpyHostToDevice);
   return N;
}

int Nfft4GPAmdNysSolve(void* nys, int n, double* x, double* rhs)
{
   NysDev* N = (NysDev*)nys;
   if (!N || n != N->n) return -1;
   hipStream_t s = current_stream();
   Vec vx, vr;
   if (vx.open(x, n, false) || vr.open(rhs, n, true)) return -1;
   hipLaunchKernelGGL(k_nys_ut, dim3(N->nblk), dim3(kNysThreads), 0, s, N->U, (size_t)n, n, N->k, vr.d, N->part);
   hipLaunchKernelGGL(k_nys_w, dim3((N->k + 255) / 256), dim3(256), 0, s, N->part, N->nblk, N->k, N->s, N->eta, N->w);
   hipLaunchKernelGGL(k_nys_u, dim3((n + kNysThreads - 1) / kNysThreads), dim3(kNysThreads),
                      sizeof(double) * N->k, s, N->U, (size_t)n, n, N->k, N->w, vr.d, N->eta, vx.d);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   vr.close(false);
   vx.close(true);
   return 0;
}

void Nfft4GPAmdNysFree(void* nys)
{
   NysDev* N = (NysDev*)nys;
   if (!N) return;
   (void)hipFree(N->U);
   (void)hipFree(N->s);
   (void)hipFree(N->w);
   (void)hipFree(N->part);
   delete N;
}

}  // extern "C"
