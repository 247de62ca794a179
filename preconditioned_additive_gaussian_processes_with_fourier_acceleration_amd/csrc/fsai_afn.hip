// fsai_afn.hip -- FSAI and AFN preconditioner applies in HBM.
//
//   Nfft4GPAmdFsai*  SRC/preconds/fsai.c:106-123  x = L^T (L rhs), L lower CSR (diagonal
//                    last), both products through Nfft4GPCsrMv (matops.c:139-272).  L^T is kept as its
//                    own CSR (built at create, entries in ascending row order) so both products are
//                    row-parallel gathers; each row sums in the reference's order with unfused multiply
//                    and add, so the result is bitwise the reference's.
//   Nfft4GPAmdAfn*   SRC/preconds/afn.c:82-143 (not part of the reference build): with [rp; rp2] =
//                    rhs(perm), y = A11 \ rp, rp2 -= A12^T y, y2 = FSAI(rp2), rp -= A12 y2, y = A11 \ rp,
//                    x(perm) = [y; y2].  A11 \ . uses L11^{-1} (two triangular products) instead of the
//                    reference's Cholesky solves.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "csr.hpp"
#include "internal.h"

namespace nfft4gp_amd {

namespace {

struct FsaiDev {
   int n = 0;
   int *ia = nullptr, *ja = nullptr;  // L
   double* aa = nullptr;
   int *tia = nullptr, *tja = nullptr;  // L^T
   double* taa = nullptr;
   double* work = nullptr;
   int *part = nullptr, *tpart = nullptr;  // row spans of the workgroups of L and L^T (csr_partition)
   int nparts = 0, ntparts = 0;
};

struct AfnDev {
   int n = 0, k = 0, n2 = 0;
   int* perm = nullptr;
   double* Linv = nullptr;   // k x k, inverse of the lower Cholesky factor of A11 (column j: rows >= j)
   double* LinvT = nullptr;  // its transpose (column i = row i of Linv)
   double* K12 = nullptr;   // k x n2 column-major
   float* K12f = nullptr;   // optional fp32 copy the two K12 passes read instead (Nfft4GPAmdAfnSetStorage)
   FsaiDev* S = nullptr;    // FSAI of the Schur complement (n2)
   double schur_scale = 0.0;  // S == NULL, n2 > 0: S^{-1} = schur_scale I (schur_opt 0, afn.c:451-459)
   bool own_S = false;
   double *rp = nullptr, *y = nullptr, *t = nullptr, *part = nullptr;
   int nblk = 0, cols = 1;  // A12 y2: workgroups, columns per workgroup
   // Nfft4GPAmdAfnSetOperator: K12^T y and K12 y2 as matvecs of this library's additive handle (whole rows, the
   // AFN's points and kernel) instead of passes over the stored K12; u, w: its input and output (n each)
   void* op = nullptr;
   double *u = nullptr, *w = nullptr;
};

// u[perm[i]] = y[i] for the landmark part (which 0: i < k) or the Schur part (which 1: i >= k) of the permuted y,
// 0 at every other point: the additive operator's input for K12^T y1 (which 0) or K12 y2 (which 1)
__global__ void k_afn_place(const double* __restrict__ y, const int* __restrict__ perm, int n, int k, int which,
                            double* __restrict__ u)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) u[perm[i]] = (which ? i >= k : i < k) ? y[i] : 0.0;
}

// rp[i] -= w[perm[i]], i in [i0, i1): the operator's output read back at the other part's points
__global__ void k_afn_sub(const double* __restrict__ w, const int* __restrict__ perm, int i0, int i1,
                          double* __restrict__ rp)
{
   const int i = i0 + blockIdx.x * blockDim.x + threadIdx.x;
   if (i < i1) rp[i] -= w[perm[i]];
}

// y = A x, a thread per CSR row summing in the row's stored order, unfused (matops.c:239-248); the
// entries and their gathers go through LDS a workgroup-wide chunk at a time (csr.hpp)
constexpr int kCsrT = 256;
constexpr int kCsrCH = 2048;
constexpr int kCsrBudget = 3 * kCsrCH;  // entries per workgroup span (a longer row gets a span of its own)
__global__ __launch_bounds__(kCsrT) void k_csr_staged(const int* __restrict__ ia, const int* __restrict__ ja,
                                                      const double* __restrict__ a, const double* __restrict__ x,
                                                      double* __restrict__ y, const int* __restrict__ part)
{
   csr_rows_staged<kCsrT, kCsrCH>(ia, ja, a, x, y, part[blockIdx.x], part[blockIdx.x + 1], false);
}

// workgroup row spans: at most kCsrT rows and kCsrBudget entries each, so that the workgroups holding a
// transposed KNN pattern's long rows do not run many more chunks than the rest
std::vector<int> csr_partition(int n, const int* ia)
{
   std::vector<int> p{0};
   int r0 = 0;
   for (int i = 0; i < n; i++) {
      if (i > r0 && (i - r0 == kCsrT || ia[i + 1] - ia[r0] > kCsrBudget)) {
         p.push_back(i);
         r0 = i;
      }
   }
   p.push_back(n);
   return p;
}

__global__ void k_scale_into(const double* __restrict__ src, int n, double a, double* __restrict__ dst)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) dst[i] = a * src[i];
}

__global__ void k_gather(const double* __restrict__ src, const int* __restrict__ perm, int n, double* __restrict__ dst)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) dst[i] = src[perm[i]];
}

__global__ void k_scatter(const double* __restrict__ src, const int* __restrict__ perm, int n, double* __restrict__ dst)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) dst[perm[i]] = src[i];
}

// out[i] = sum_j M[j + i*k] v[j]: one wave per output over a contiguous column of M.  M = LinvT gives
// Linv v, M = Linv gives Linv^T v (the other triangle holds zeros)
__global__ __launch_bounds__(256) void k_trmv(const double* __restrict__ M, int k, const double* __restrict__ v,
                                              double* __restrict__ out)
{
   const int lane = threadIdx.x & 63;
   const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
   if (i >= k) return;
   const double* col = M + (size_t)i * k;
   double r = 0.0;
   for (int j = lane; j < k; j += 64) r = fma(col[j], v[j], r);
   for (int off = 32; off > 0; off >>= 1) r += __shfl_down(r, off, 64);
   if (lane == 0) out[i] = r;
}

// rp2[j] -= sum_i K12[i + j*k] y[i]: one wave per kA12tCols consecutive columns (their loads in flight
// together), y staged in LDS (k <= kA12tLdsMax; beyond, read from HBM through the caches).  Each column's
// sum is the same lane-strided sum and shuffle tree as with a wave per column.
constexpr int kA12tCols = 4;
constexpr int kA12tLdsMax = 8192;
template <bool LDS, typename TK = double>
__global__ __launch_bounds__(256) void k_a12t(const TK* __restrict__ K12, int k, int n2, const double* __restrict__ y,
                                              double* __restrict__ rp2)
{
   extern __shared__ double s_y_[];
   const double* s_y = LDS ? s_y_ : y;
   if (LDS) {
      for (int i = threadIdx.x; i < k; i += 256) s_y_[i] = y[i];
      __syncthreads();
   }
   const int lane = threadIdx.x & 63;
   const long long j0 = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * kA12tCols;
   if (j0 >= n2) return;
   const int nc = (int)std::min<long long>(kA12tCols, n2 - j0);
   const TK* col = K12 + j0 * k;
   double r[kA12tCols];
#pragma unroll
   for (int c = 0; c < kA12tCols; c++) r[c] = 0.0;
   if (nc == kA12tCols) {
      for (int i = lane; i < k; i += 64) {
         const double yi = s_y[i];
#pragma unroll
         for (int c = 0; c < kA12tCols; c++) r[c] = fma((double)col[(size_t)c * k + i], yi, r[c]);
      }
   } else {
      for (int i = lane; i < k; i += 64) {
         const double yi = s_y[i];
         for (int c = 0; c < nc; c++) r[c] = fma((double)col[(size_t)c * k + i], yi, r[c]);
      }
   }
#pragma unroll
   for (int c = 0; c < kA12tCols; c++) {
      double v = r[c];
      for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
      if (lane == 0 && c < nc) rp2[j0 + c] -= v;
   }
}

// part[blk][i] = sum_{j in blk} K12[i + j*k] y2[j]; `cols` columns per workgroup, sized at create so
// that ~2048 workgroups stream K12 (one HBM pass over k x n2)
constexpr int kA12Blocks = 2048;
template <typename TK = double>
__global__ __launch_bounds__(256) void k_a12_part(const TK* __restrict__ K12, int k, int n2, int cols,
                                                  const double* __restrict__ y2, double* __restrict__ part)
{
   const int j0 = blockIdx.x * cols, j1 = min(n2, j0 + cols);
   for (int i = threadIdx.x; i < k; i += blockDim.x) {
      double r0 = 0.0, r1 = 0.0;
      int j = j0;
      for (; j + 1 < j1; j += 2) {
         r0 = fma((double)K12[i + (size_t)j * k], y2[j], r0);
         r1 = fma((double)K12[i + (size_t)(j + 1) * k], y2[j + 1], r1);
      }
      if (j < j1) r0 = fma((double)K12[i + (size_t)j * k], y2[j], r0);
      part[(size_t)blockIdx.x * k + i] = r0 + r1;
   }
}

// The two K12 passes in one when S^{-1} = schur_scale I (schur_opt 0): y2[j] = schur_scale (rp2[j] - K12[:, j]^T y)
// needs only column j, and the second pass adds K12[:, j] y2[j], so each column is read from HBM once and used
// twice from registers.  A wave takes 4 columns at a time (k_a12t's dot: the same lane-strided sum and shuffle tree,
// so y2 has k_a12t + k_scale_into's bits), then adds the 4 columns times their y2 into its lanes' row sums (rows
// lane + 64 m); the workgroup's part[blk] adds its 4 waves' sums in wave order.  Fixed order: the same bits every
// run (the K12 y2 sum in another order than k_a12_part's).  MI rows per lane (k <= 64 MI; EXACT: k = 64 MI).
template <typename TK, int MI, bool EXACT>
__device__ __forceinline__ void a12_fused_body(const TK* __restrict__ K12, int k, int n2, int cols,
                                               const double* __restrict__ y, const double* __restrict__ rp2,
                                               double scale, double* __restrict__ y2, double* __restrict__ part)
{
   extern __shared__ double s_y[];  // [k] y, then [4][k] the waves' row sums
   double* s_acc = s_y + k;
   for (int i = threadIdx.x; i < k; i += 256) s_y[i] = y[i];
   __syncthreads();
   const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
   const int j0 = blockIdx.x * cols, j1 = min(n2, j0 + cols);
   double yl[MI], acc[MI];
#pragma unroll
   for (int m = 0; m < MI; m++) {
      const int i = lane + 64 * m;
      yl[m] = i < k ? s_y[i] : 0.0;
      acc[m] = 0.0;
   }
   for (int jw = j0 + wave * kA12tCols; jw < j1; jw += 4 * kA12tCols) {
      const int nc = min(kA12tCols, j1 - jw);
      const TK* col = K12 + (size_t)jw * k;
      // every load unconditional, so all 4 MI of them are in flight together: an element past the column's k rows
      // or past the workgroup's columns reads a valid entry instead and is never used (its row's sum is not
      // stored; such a column's y2 is 0)
      TK v[kA12tCols][MI];
#pragma unroll
      for (int c = 0; c < kA12tCols; c++) {
         const TK* cc = col + (size_t)min(c, nc - 1) * k;  // a column past the workgroup's re-reads its last one
         if (EXACT) {  // k = 64 MI: one base per column, immediate row offsets
#pragma unroll
            for (int m = 0; m < MI; m++) v[c][m] = cc[lane + 64 * m];
         } else {
#pragma unroll
            for (int m = 0; m < MI; m++) v[c][m] = cc[min(lane + 64 * m, k - 1)];
         }
      }
      double r[kA12tCols];
#pragma unroll
      for (int c = 0; c < kA12tCols; c++) {
         r[c] = 0.0;
#pragma unroll
         for (int m = 0; m < MI; m++)
            if (lane + 64 * m < k) r[c] = fma((double)v[c][m], yl[m], r[c]);
      }
#pragma unroll
      for (int c = 0; c < kA12tCols; c++) {
         double t = r[c];
         for (int off = 32; off > 0; off >>= 1) t += __shfl_down(t, off, 64);
         double yv = 0.0;
         if (lane == 0 && c < nc) {
            yv = scale * (rp2[jw + c] - t);
            y2[jw + c] = yv;
         }
         yv = __shfl(yv, 0, 64);
#pragma unroll
         for (int m = 0; m < MI; m++) acc[m] = fma((double)v[c][m], yv, acc[m]);
      }
   }
#pragma unroll
   for (int m = 0; m < MI; m++) {
      const int i = lane + 64 * m;
      if (i < k) s_acc[(size_t)wave * k + i] = acc[m];
   }
   __syncthreads();
   for (int i = threadIdx.x; i < k; i += 256)
      part[(size_t)blockIdx.x * k + i] = ((s_acc[i] + s_acc[(size_t)k + i]) + s_acc[2 * (size_t)k + i]) +
                                         s_acc[3 * (size_t)k + i];
}

// fp64 storage: 133 VGPRs, 3 waves per SIMD; fp32 storage held to 128 VGPRs (4 waves per SIMD: 0.505 -> 0.472 ms per
// apply at k = 512, n = 1e6, where the same bound costs fp64 0.797 -> 0.821; profiles/r06_afn_fused.txt)
template <int MI, bool EXACT>
__global__ __launch_bounds__(256) void k_a12_fused_f64(const double* __restrict__ K12, int k, int n2, int cols,
                                                       const double* __restrict__ y, const double* __restrict__ rp2,
                                                       double scale, double* __restrict__ y2, double* __restrict__ part)
{
   a12_fused_body<double, MI, EXACT>(K12, k, n2, cols, y, rp2, scale, y2, part);
}
template <int MI, bool EXACT>
__global__ __launch_bounds__(256, 4) void k_a12_fused_f32(const float* __restrict__ K12, int k, int n2, int cols,
                                                          const double* __restrict__ y, const double* __restrict__ rp2,
                                                          double scale, double* __restrict__ y2, double* __restrict__ part)
{
   a12_fused_body<float, MI, EXACT>(K12, k, n2, cols, y, rp2, scale, y2, part);
}

// the fused pass for k <= 1024 (K12f: the fp32 copy, else K12); false when k is larger or NFFT4GP_AMD_AFN_FUSED=0
bool a12_fused(const double* K12, const float* K12f, int k, int n2, int cols, int nblk, const double* y,
               const double* rp2, double scale, double* y2, double* part, hipStream_t s)
{
   const char* fe = getenv("NFFT4GP_AMD_AFN_FUSED");
   if (k > 1024 || (fe && atoi(fe) == 0)) return false;
   const size_t lds = sizeof(double) * 5 * (size_t)k;
#define NFFT4GP_A12F(KER, MIv, M)                                                                                    \
   if (k == 64 * MIv)                                                                                                 \
      hipLaunchKernelGGL((KER<MIv, true>), dim3(nblk), dim3(256), lds, s, M, k, n2, cols, y, rp2, scale, y2, part);   \
   else                                                                                                               \
      hipLaunchKernelGGL((KER<MIv, false>), dim3(nblk), dim3(256), lds, s, M, k, n2, cols, y, rp2, scale, y2, part)
#define NFFT4GP_A12F_MI(KER, M)                                                                                      \
   if (k <= 128) NFFT4GP_A12F(KER, 2, M);                                                                             \
   else if (k <= 256) NFFT4GP_A12F(KER, 4, M);                                                                        \
   else if (k <= 512) NFFT4GP_A12F(KER, 8, M);                                                                        \
   else NFFT4GP_A12F(KER, 16, M)
   if (K12f) {
      NFFT4GP_A12F_MI(k_a12_fused_f32, K12f);
   } else {
      NFFT4GP_A12F_MI(k_a12_fused_f64, K12);
   }
#undef NFFT4GP_A12F_MI
#undef NFFT4GP_A12F
   return true;
}

// rp[i] -= sum_blk part[blk][i]: a workgroup per 16 outputs, 64 strands over the partials (strand s takes
// blk = s mod 64, four rotating accumulators, all its loads independent), strands added in order in LDS.
// Fixed order, so the same bits every run.
__global__ __launch_bounds__(1024) void k_a12_reduce(const double* __restrict__ part, int nblk, int k,
                                                     double* __restrict__ rp)
{
   __shared__ double s[64][17];
   const int c = threadIdx.x & 15, strand = threadIdx.x >> 4;
   const int i = blockIdx.x * 16 + c;
   double z[4] = {0.0, 0.0, 0.0, 0.0};
   if (i < k) {
      int u = 0;
      for (int b = strand; b < nblk; b += 64, u = (u + 1) & 3) z[u] += part[(size_t)b * k + i];
   }
   s[strand][c] = (z[0] + z[1]) + (z[2] + z[3]);
   __syncthreads();
   if (threadIdx.x < 16 && i < k) {
      double t = 0.0;
      for (int q = 0; q < 64; q++) t += s[q][threadIdx.x];
      rp[i] -= t;
   }
}

void a12_shape(int n2, int& cols, int& nblk)
{
   cols = std::max(16, std::min(1024, (n2 + kA12Blocks - 1) / kA12Blocks));
   nblk = (n2 + cols - 1) / cols;
}

template <class T>
int up(T** d, const T* h, size_t count)
{
   NFFT4GP_HIP_CHECK(hipMalloc((void**)d, sizeof(T) * std::max<size_t>(1, count)));
   if (count) NFFT4GP_HIP_CHECK(hipMemcpy(*d, h, sizeof(T) * count, hipMemcpyHostToDevice));
   return 0;
}

void fsai_free(FsaiDev* F)
{
   if (!F) return;
   for (void* p : {(void*)F->ia, (void*)F->ja, (void*)F->aa, (void*)F->tia, (void*)F->tja, (void*)F->taa,
                   (void*)F->work, (void*)F->part, (void*)F->tpart})
      (void)hipFree(p);
   delete F;
}

FsaiDev* fsai_create(int n, const int* ia, const int* ja, const double* aa)
{
   if (n <= 0 || !ia || !ja || !aa) return nullptr;
   const int nnz = ia[n];
   // L^T as CSR: column c's entries in ascending row order, i.e. Nfft4GPCsrMv('T')'s accumulation order
   std::vector<int> tia(n + 1, 0), tja(nnz);
   std::vector<double> taa(nnz);
   for (int j = 0; j < nnz; j++) tia[ja[j] + 1]++;
   for (int c = 0; c < n; c++) tia[c + 1] += tia[c];
   std::vector<int> pos(tia.begin(), tia.end() - 1);
   for (int i = 0; i < n; i++)
      for (int j = ia[i]; j < ia[i + 1]; j++) {
         const int p = pos[ja[j]]++;
         tja[p] = i;
         taa[p] = aa[j];
      }
   FsaiDev* F = new FsaiDev();
   F->n = n;
   if (up(&F->ia, ia, (size_t)n + 1) || up(&F->ja, ja, (size_t)nnz) || up(&F->aa, aa, (size_t)nnz) ||
       up(&F->tia, tia.data(), (size_t)n + 1) || up(&F->tja, tja.data(), (size_t)nnz) ||
       up(&F->taa, taa.data(), (size_t)nnz) || hipMalloc((void**)&F->work, sizeof(double) * n) != hipSuccess) {
      fsai_free(F);
      return nullptr;
   }
   const std::vector<int> p = csr_partition(n, ia), tp = csr_partition(n, tia.data());
   F->nparts = (int)p.size() - 1;
   F->ntparts = (int)tp.size() - 1;
   if (up(&F->part, p.data(), p.size()) || up(&F->tpart, tp.data(), tp.size())) {
      fsai_free(F);
      return nullptr;
   }
   return F;
}

int fsai_apply_dev(FsaiDev* F, double* dx, const double* drhs, hipStream_t s)
{
   hipLaunchKernelGGL(k_csr_staged, dim3(F->nparts), dim3(kCsrT), 0, s, F->ia, F->ja, F->aa, drhs, F->work,
                      F->part);
   hipLaunchKernelGGL(k_csr_staged, dim3(F->ntparts), dim3(kCsrT), 0, s, F->tia, F->tja, F->taa, F->work, dx,
                      F->tpart);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

// host or device vectors, like the library's other applies
int with_device_vectors(int n, double* x, double* rhs, int (*fn)(void*, double*, const double*, hipStream_t),
                        void* obj)
{
   hipStream_t s = current_stream();
   const bool dx = is_device_ptr(x), dr = is_device_ptr(rhs);
   double *xd = x, *rd = rhs;
   if (!dx) NFFT4GP_HIP_CHECK(hipMalloc((void**)&xd, sizeof(double) * std::max(1, n)));
   if (!dr) {
      NFFT4GP_HIP_CHECK(hipMalloc((void**)&rd, sizeof(double) * std::max(1, n)));
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(rd, rhs, sizeof(double) * n, hipMemcpyHostToDevice, s));
   }
   int rc = fn(obj, xd, rd, s);
   if (!dx) {
      if (!rc) NFFT4GP_HIP_CHECK(hipMemcpyAsync(x, xd, sizeof(double) * n, hipMemcpyDeviceToHost, s));
      NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
      (void)hipFree(xd);
   }
   if (!dr) {
      NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
      (void)hipFree(rd);
   }
   return rc;
}

int fsai_apply_obj(void* obj, double* dx, const double* drhs, hipStream_t s)
{
   return fsai_apply_dev((FsaiDev*)obj, dx, drhs, s);
}

int afn_apply_obj(void* obj, double* dx, const double* drhs, hipStream_t s)
{
   AfnDev* A = (AfnDev*)obj;
   const int n = A->n, k = A->k, n2 = A->n2;
   const int g = (n + 255) / 256, gk = (k + 3) / 4;
   double* rp2 = A->rp + k;
   double* y2 = A->y + k;
   if (k == 0) return fsai_apply_dev(A->S, dx, drhs, s);  // afn.c:106-110
   if (n2 == 0) {                                          // afn.c:101-105: A11 solve on the unpermuted rhs
      hipLaunchKernelGGL(k_trmv, dim3(gk), dim3(256), 0, s, A->LinvT, k, drhs, A->t);
      hipLaunchKernelGGL(k_trmv, dim3(gk), dim3(256), 0, s, A->Linv, k, A->t, dx);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return 0;
   }
   hipLaunchKernelGGL(k_gather, dim3(g), dim3(256), 0, s, drhs, A->perm, n, A->rp);
   // y = A11 \ rp = L^{-T} (L^{-1} rp)
   hipLaunchKernelGGL(k_trmv, dim3(gk), dim3(256), 0, s, A->LinvT, k, A->rp, A->t);
   hipLaunchKernelGGL(k_trmv, dim3(gk), dim3(256), 0, s, A->Linv, k, A->t, A->y);
   if (A->op) {
      // K12^T y1 = (A u)[Schur points] with u = y1 at the landmarks and 0 elsewhere: the operator's kernel part is
      // the AFN's kernel, and its mu term meets only zeros at the points read back; then K12 y2 the same way
      hipLaunchKernelGGL(k_afn_place, dim3(g), dim3(256), 0, s, (const double*)A->y, A->perm, n, k, 0, A->u);
      const double* xin[1] = {A->u};
      double* yout[1] = {A->w};
      if (additive_matvec_multi(A->op, 1, 1.0, xin, 0.0, yout)) return -1;
      hipLaunchKernelGGL(k_afn_sub, dim3((n2 + 255) / 256), dim3(256), 0, s, (const double*)A->w, A->perm, k, n, A->rp);
      if (A->S) {
         if (fsai_apply_dev(A->S, y2, rp2, s)) return -1;
      } else {
         hipLaunchKernelGGL(k_scale_into, dim3((n2 + 255) / 256), dim3(256), 0, s, rp2, n2, A->schur_scale, y2);
      }
      hipLaunchKernelGGL(k_afn_place, dim3(g), dim3(256), 0, s, (const double*)A->y, A->perm, n, k, 1, A->u);
      if (additive_matvec_multi(A->op, 1, 1.0, xin, 0.0, yout)) return -1;
      hipLaunchKernelGGL(k_afn_sub, dim3((k + 255) / 256), dim3(256), 0, s, (const double*)A->w, A->perm, 0, k, A->rp);
      hipLaunchKernelGGL(k_trmv, dim3(gk), dim3(256), 0, s, A->LinvT, k, A->rp, A->t);
      hipLaunchKernelGGL(k_trmv, dim3(gk), dim3(256), 0, s, A->Linv, k, A->t, A->y);
      hipLaunchKernelGGL(k_scatter, dim3(g), dim3(256), 0, s, A->y, A->perm, n, dx);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return 0;
   }
   // S^{-1} = schur_scale I: both K12 passes in one (k_a12_fused_*; NFFT4GP_AMD_AFN_FUSED=0 keeps the two)
   if (!A->S && a12_fused(A->K12, A->K12f, k, n2, A->cols, A->nblk, A->y, rp2, A->schur_scale, y2, A->part, s)) {
      hipLaunchKernelGGL(k_a12_reduce, dim3((k + 15) / 16), dim3(1024), 0, s, A->part, A->nblk, k, A->rp);
      hipLaunchKernelGGL(k_trmv, dim3(gk), dim3(256), 0, s, A->LinvT, k, A->rp, A->t);
      hipLaunchKernelGGL(k_trmv, dim3(gk), dim3(256), 0, s, A->Linv, k, A->t, A->y);
      hipLaunchKernelGGL(k_scatter, dim3(g), dim3(256), 0, s, A->y, A->perm, n, dx);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return 0;
   }
   // rp2 -= A12^T y
   const dim3 ga((n2 + 4 * kA12tCols - 1) / (4 * kA12tCols));
   if (A->K12f) {
      if (k <= kA12tLdsMax)
         hipLaunchKernelGGL((k_a12t<true, float>), ga, dim3(256), sizeof(double) * k, s, (const float*)A->K12f, k, n2,
                            A->y, rp2);
      else
         hipLaunchKernelGGL((k_a12t<false, float>), ga, dim3(256), 0, s, (const float*)A->K12f, k, n2, A->y, rp2);
   } else if (k <= kA12tLdsMax) {
      hipLaunchKernelGGL(k_a12t<true>, ga, dim3(256), sizeof(double) * k, s, (const double*)A->K12, k, n2, A->y, rp2);
   } else {
      hipLaunchKernelGGL(k_a12t<false>, ga, dim3(256), 0, s, (const double*)A->K12, k, n2, A->y, rp2);
   }
   // y2 = FSAI(rp2), or rp2 / noise (schur_opt 0)
   if (A->S) {
      if (fsai_apply_dev(A->S, y2, rp2, s)) return -1;
   } else {
      hipLaunchKernelGGL(k_scale_into, dim3((n2 + 255) / 256), dim3(256), 0, s, rp2, n2, A->schur_scale, y2);
   }
   // rp -= A12 y2
   if (A->K12f)
      hipLaunchKernelGGL(k_a12_part<float>, dim3(A->nblk), dim3(256), 0, s, (const float*)A->K12f, k, n2, A->cols, y2,
                         A->part);
   else
      hipLaunchKernelGGL(k_a12_part<double>, dim3(A->nblk), dim3(256), 0, s, (const double*)A->K12, k, n2, A->cols,
                         y2, A->part);
   hipLaunchKernelGGL(k_a12_reduce, dim3((k + 15) / 16), dim3(1024), 0, s, A->part, A->nblk, k, A->rp);
   // y = A11 \ rp
   hipLaunchKernelGGL(k_trmv, dim3(gk), dim3(256), 0, s, A->LinvT, k, A->rp, A->t);
   hipLaunchKernelGGL(k_trmv, dim3(gk), dim3(256), 0, s, A->Linv, k, A->t, A->y);
   hipLaunchKernelGGL(k_scatter, dim3(g), dim3(256), 0, s, A->y, A->perm, n, dx);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

// ---- the AFN apply split over row shards (afn.c:82-143 with the rows of the operator's shards) ----------
// Each rank keeps, for the points of its own rows [rb, re): which of them are landmarks (their index in
// perm[:k]) and which are Schur points (their position in perm[k:]), the K12 columns of its Schur points,
// and the rows of the Schur FSAI G and of G^T that belong to its Schur points (sub-CSRs with global column
// indices).  The k x k factors are replicated.  An apply exchanges: the landmark entries of the rhs (one
// k all-reduce), the K12 y2 partial sums (one k all-reduce) and -- with the Schur FSAI -- the Schur vector
// before each of the two sparse products (an all-gather, as an n2 all-reduce of a zero-padded vector).
struct AfnShard {
   int n = 0, k = 0, n2 = 0, m1 = 0, m2 = 0;
   Comm* comm = nullptr;
   int *lm_idx = nullptr, *lm_row = nullptr;  // m1: landmark index a in [0, k), local row
   int *nl_pos = nullptr, *nl_row = nullptr;  // m2: Schur position p in [0, n2), local row
   double *Linv = nullptr, *LinvT = nullptr, *K12 = nullptr;  // k x k, k x k, k x m2
   FsaiDev G, GT;  // rows of G / G^T at this rank's Schur points (ia, ja, aa, part; ja global)
   // a shard set up by its own rank (afn_shard_from_parts): G's own rows only, so G^T w is formed as this rank's
   // partial sums over its rows -- GTp, one CSR row per Schur column its rows touch (tcols), entries in
   // ascending row order, x = this rank's w -- scattered into the Schur vector and summed over the ranks
   bool gt_scatter = false;
   long long g_nnz = 0;  // entries of G's rows this rank holds
   FsaiDev GTp;
   int* tcols = nullptr;
   double* tbuf = nullptr;
   bool fsai = false;
   double schur_scale = 0.0;
   double *rp1 = nullptr, *y1 = nullptr, *t = nullptr, *w = nullptr;  // k
   double *rp2 = nullptr, *y2 = nullptr, *v = nullptr;                 // m2
   double *gbuf = nullptr;                                              // n2
   double* part = nullptr;
   int nblk = 0, cols = 1;
};

__global__ void k_take(const double* __restrict__ src, const int* __restrict__ idx, int m, double* __restrict__ dst)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < m) dst[i] = src[idx[i]];
}

__global__ void k_put(const double* __restrict__ src, const int* __restrict__ idx, int m, double* __restrict__ dst)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < m) dst[idx[i]] = src[i];
}

// dst[idx_dst[i]] = src[idx_src[i]]
__global__ void k_move(const double* __restrict__ src, const int* __restrict__ idx_src, const int* __restrict__ idx_dst,
                       int m, double* __restrict__ dst)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < m) dst[idx_dst[i]] = src[idx_src[i]];
}

__global__ void k_add_into(double* __restrict__ y, const double* __restrict__ w, int k)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < k) y[i] += w[i];
}

// out[:, i] = K12[:, cols[i]] (k x n2 column-major -> k x m)
__global__ void k_take_cols(const double* __restrict__ K12, int k, const int* __restrict__ cols, int m,
                            double* __restrict__ out)
{
   const int i = blockIdx.y;
   const double* src = K12 + (size_t)cols[i] * k;
   double* dst = out + (size_t)i * k;
   for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < k; r += gridDim.x * blockDim.x) dst[r] = src[r];
}

void csr_free_parts(FsaiDev& F)
{
   for (void* p : {(void*)F.ia, (void*)F.ja, (void*)F.aa, (void*)F.part}) (void)hipFree(p);
   F = FsaiDev();
}

// rows `rows` of a host CSR (ia, ja, aa) as a device CSR with its workgroup spans
int csr_rows_upload(const std::vector<int>& ia, const std::vector<int>& ja, const std::vector<double>& aa,
                    const std::vector<int>& rows, FsaiDev& F)
{
   std::vector<int> sia(rows.size() + 1, 0), sja;
   std::vector<double> saa;
   for (size_t i = 0; i < rows.size(); i++) {
      for (int j = ia[rows[i]]; j < ia[rows[i] + 1]; j++) {
         sja.push_back(ja[j]);
         saa.push_back(aa[j]);
      }
      sia[i + 1] = (int)sja.size();
   }
   F.n = (int)rows.size();
   const std::vector<int> p = csr_partition(F.n, sia.data());
   F.nparts = (int)p.size() - 1;
   if (up(&F.ia, sia.data(), sia.size()) || up(&F.ja, sja.data(), sja.size()) || up(&F.aa, saa.data(), saa.size()) ||
       up(&F.part, p.data(), p.size()))
      return -1;
   return 0;
}

void afn_shard_free(AfnShard* S)
{
   if (!S) return;
   (void)hipStreamSynchronize(current_stream());
   for (void* p : {(void*)S->lm_idx, (void*)S->lm_row, (void*)S->nl_pos, (void*)S->nl_row, (void*)S->Linv,
                   (void*)S->LinvT, (void*)S->K12, (void*)S->rp1, (void*)S->y1, (void*)S->t, (void*)S->w,
                   (void*)S->rp2, (void*)S->y2, (void*)S->v, (void*)S->gbuf, (void*)S->part})
      (void)hipFree(p);
   csr_free_parts(S->G);
   csr_free_parts(S->GT);
   csr_free_parts(S->GTp);
   (void)hipFree(S->tcols);
   (void)hipFree(S->tbuf);
   delete S;
}

template <class T>
int dl(std::vector<T>& h, const T* d, size_t count)
{
   h.resize(count);
   if (count) NFFT4GP_HIP_CHECK(hipMemcpy(h.data(), d, sizeof(T) * count, hipMemcpyDeviceToHost));
   return 0;
}

AfnShard* afn_shard_create(const AfnDev* A, int rb, int re, Comm* comm)
{
   const int n = A->n, k = A->k, n2 = A->n2;
   if (k <= 0 || n2 <= 0 || rb < 0 || re > n || rb > re) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnShard needs 0 < k < n and rows within [0, %d)\n", n);
      return nullptr;
   }
   std::vector<int> perm;
   if (dl(perm, A->perm, (size_t)n)) return nullptr;
   AfnShard* S = new AfnShard();
   S->n = re - rb;
   S->k = k;
   S->n2 = n2;
   S->comm = comm;
   S->fsai = A->S != nullptr;
   S->schur_scale = A->schur_scale;
   std::vector<int> lm_idx, lm_row, nl_pos, nl_row;
   for (int p = 0; p < n; p++) {
      const int row = perm[p];
      if (row < rb || row >= re) continue;
      if (p < k) {
         lm_idx.push_back(p);
         lm_row.push_back(row - rb);
      } else {
         nl_pos.push_back(p - k);
         nl_row.push_back(row - rb);
      }
   }
   S->m1 = (int)lm_idx.size();
   S->m2 = (int)nl_pos.size();
   a12_shape(std::max(1, S->m2), S->cols, S->nblk);
   hipStream_t s = current_stream();
   const size_t kk = (size_t)k * k;
   bool ok = !up(&S->lm_idx, lm_idx.data(), lm_idx.size()) && !up(&S->lm_row, lm_row.data(), lm_row.size()) &&
             !up(&S->nl_pos, nl_pos.data(), nl_pos.size()) && !up(&S->nl_row, nl_row.data(), nl_row.size());
   for (double** p : {&S->Linv, &S->LinvT})
      ok = ok && hipMalloc((void**)p, sizeof(double) * kk) == hipSuccess;
   ok = ok && hipMalloc((void**)&S->K12, sizeof(double) * std::max<size_t>(1, (size_t)k * S->m2)) == hipSuccess;
   for (double** p : {&S->rp1, &S->y1, &S->t, &S->w})
      ok = ok && hipMalloc((void**)p, sizeof(double) * k) == hipSuccess;
   for (double** p : {&S->rp2, &S->y2, &S->v})
      ok = ok && hipMalloc((void**)p, sizeof(double) * std::max(1, S->m2)) == hipSuccess;
   ok = ok && hipMalloc((void**)&S->gbuf, sizeof(double) * n2) == hipSuccess &&
        hipMalloc((void**)&S->part, sizeof(double) * (size_t)S->nblk * k) == hipSuccess;
   ok = ok && hipMemcpyAsync(S->Linv, A->Linv, sizeof(double) * kk, hipMemcpyDeviceToDevice, s) == hipSuccess &&
        hipMemcpyAsync(S->LinvT, A->LinvT, sizeof(double) * kk, hipMemcpyDeviceToDevice, s) == hipSuccess;
   if (ok && S->m2 > 0) {
      hipLaunchKernelGGL(k_take_cols, dim3((k + 255) / 256, S->m2), dim3(256), 0, s, (const double*)A->K12, k,
                         (const int*)S->nl_pos, S->m2, S->K12);
      ok = hipGetLastError() == hipSuccess;
   }
   if (ok && S->fsai) {
      const FsaiDev* F = A->S;
      std::vector<int> ia, ja, tia, tja;
      std::vector<double> aa, taa;
      ok = !dl(ia, F->ia, (size_t)n2 + 1) && !dl(tia, F->tia, (size_t)n2 + 1);
      ok = ok && !dl(ja, F->ja, (size_t)ia[n2]) && !dl(aa, F->aa, (size_t)ia[n2]) && !dl(tja, F->tja, (size_t)tia[n2]) &&
           !dl(taa, F->taa, (size_t)tia[n2]);
      ok = ok && !csr_rows_upload(ia, ja, aa, nl_pos, S->G) && !csr_rows_upload(tia, tja, taa, nl_pos, S->GT);
      for (int p : nl_pos) S->g_nnz += ia[p + 1] - ia[p];
   }
   if (!ok || hipStreamSynchronize(s) != hipSuccess) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnShard: allocation or copy failed\n");
      afn_shard_free(S);
      return nullptr;
   }
   return S;
}

int afn_shard_apply(AfnShard* S, double* x, const double* r, hipStream_t s)
{
   const int k = S->k, m1 = S->m1, m2 = S->m2;
   const int gk = (k + 3) / 4, g1 = (m1 + 255) / 256 + 1, g2 = (m2 + 255) / 256 + 1;
   // [rp1; rp2] = r(perm): the landmark entries are spread over the ranks (one owner each)
   NFFT4GP_HIP_CHECK(hipMemsetAsync(S->rp1, 0, sizeof(double) * k, s));
   hipLaunchKernelGGL(k_move, dim3(g1), dim3(256), 0, s, r, (const int*)S->lm_row, (const int*)S->lm_idx, m1, S->rp1);
   if (S->comm->allreduce(S->rp1, (size_t)k, s)) return -1;
   hipLaunchKernelGGL(k_take, dim3(g2), dim3(256), 0, s, r, (const int*)S->nl_row, m2, S->rp2);
   // y1 = A11 \ rp1
   hipLaunchKernelGGL(k_trmv, dim3(gk), dim3(256), 0, s, S->LinvT, k, S->rp1, S->t);
   hipLaunchKernelGGL(k_trmv, dim3(gk), dim3(256), 0, s, S->Linv, k, S->t, S->y1);
   // S^{-1} = schur_scale I: this rank's columns in one K12 pass (y2 and the partials of K12 y2)
   const bool fused = !S->fsai && m2 > 0 &&
                      a12_fused(S->K12, nullptr, k, m2, S->cols, S->nblk, S->y1, S->rp2, S->schur_scale, S->y2,
                                S->part, s);
   // rp2 -= A12^T y1 on this rank's columns
   if (m2 > 0 && !fused) {
      const dim3 ga((m2 + 4 * kA12tCols - 1) / (4 * kA12tCols));
      if (k <= kA12tLdsMax)
         hipLaunchKernelGGL(k_a12t<true>, ga, dim3(256), sizeof(double) * k, s, (const double*)S->K12, k, m2, S->y1,
                            S->rp2);
      else
         hipLaunchKernelGGL(k_a12t<false>, ga, dim3(256), 0, s, (const double*)S->K12, k, m2, S->y1, S->rp2);
   }
   // y2 = G^T G rp2 (each product reads the whole Schur vector: all-gathered), or rp2 / noise
   if (S->fsai) {
      NFFT4GP_HIP_CHECK(hipMemsetAsync(S->gbuf, 0, sizeof(double) * S->n2, s));
      hipLaunchKernelGGL(k_put, dim3(g2), dim3(256), 0, s, S->rp2, (const int*)S->nl_pos, m2, S->gbuf);
      if (S->comm->allreduce(S->gbuf, (size_t)S->n2, s)) return -1;
      if (m2 > 0)
         hipLaunchKernelGGL(k_csr_staged, dim3(S->G.nparts), dim3(kCsrT), 0, s, S->G.ia, S->G.ja, S->G.aa, S->gbuf,
                            S->v, S->G.part);
      NFFT4GP_HIP_CHECK(hipMemsetAsync(S->gbuf, 0, sizeof(double) * S->n2, s));
      if (S->gt_scatter) {
         // (G^T v)_j = sum over every rank's rows i of G_ij v_i: this rank's partial sums at the columns its rows
         // touch, scattered into the Schur vector, summed over the ranks, own entries taken
         const int nt = S->GTp.n;
         if (nt > 0) {
            hipLaunchKernelGGL(k_csr_staged, dim3(S->GTp.nparts), dim3(kCsrT), 0, s, S->GTp.ia, S->GTp.ja, S->GTp.aa,
                               S->v, S->tbuf, S->GTp.part);
            hipLaunchKernelGGL(k_put, dim3((nt + 255) / 256 + 1), dim3(256), 0, s, S->tbuf, (const int*)S->tcols, nt,
                               S->gbuf);
         }
         if (S->comm->allreduce(S->gbuf, (size_t)S->n2, s)) return -1;
         if (m2 > 0) hipLaunchKernelGGL(k_take, dim3(g2), dim3(256), 0, s, S->gbuf, (const int*)S->nl_pos, m2, S->y2);
      } else {
         hipLaunchKernelGGL(k_put, dim3(g2), dim3(256), 0, s, S->v, (const int*)S->nl_pos, m2, S->gbuf);
         if (S->comm->allreduce(S->gbuf, (size_t)S->n2, s)) return -1;
         if (m2 > 0)
            hipLaunchKernelGGL(k_csr_staged, dim3(S->GT.nparts), dim3(kCsrT), 0, s, S->GT.ia, S->GT.ja, S->GT.aa,
                               S->gbuf, S->y2, S->GT.part);
      }
   } else if (m2 > 0 && !fused) {
      hipLaunchKernelGGL(k_scale_into, dim3(g2), dim3(256), 0, s, S->rp2, m2, S->schur_scale, S->y2);
   }
   // rp1 -= A12 y2: this rank's columns' partial sum (negated by k_a12_reduce), summed over the ranks
   NFFT4GP_HIP_CHECK(hipMemsetAsync(S->w, 0, sizeof(double) * k, s));
   if (m2 > 0) {
      if (!fused)
         hipLaunchKernelGGL(k_a12_part<double>, dim3(S->nblk), dim3(256), 0, s, (const double*)S->K12, k, m2, S->cols,
                            S->y2, S->part);
      hipLaunchKernelGGL(k_a12_reduce, dim3((k + 15) / 16), dim3(1024), 0, s, S->part, S->nblk, k, S->w);
   }
   if (S->comm->allreduce(S->w, (size_t)k, s)) return -1;
   hipLaunchKernelGGL(k_add_into, dim3((k + 255) / 256), dim3(256), 0, s, S->rp1, S->w, k);
   // y1 = A11 \ rp1, then x(perm) = [y1; y2] on this rank's rows
   hipLaunchKernelGGL(k_trmv, dim3(gk), dim3(256), 0, s, S->LinvT, k, S->rp1, S->t);
   hipLaunchKernelGGL(k_trmv, dim3(gk), dim3(256), 0, s, S->Linv, k, S->t, S->y1);
   hipLaunchKernelGGL(k_move, dim3(g1), dim3(256), 0, s, S->y1, (const int*)S->lm_idx, (const int*)S->lm_row, m1, x);
   hipLaunchKernelGGL(k_put, dim3(g2), dim3(256), 0, s, S->y2, (const int*)S->nl_row, m2, x);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

}  // namespace

// A row shard of the AFN apply from the pieces one rank's sharded setup computed (afn_setup.hip,
// Nfft4GPAmdAfnShardSetup): its landmarks (lm_idx: index in perm[:k], lm_row: local row), its Schur points
// (nl_pos: Schur position, ascending; nl_row: local row), the replicated L11^{-1} and its transpose, K12's
// columns at its Schur points (k x m2), and G's rows at its Schur points as host CSR (gia over the m2 rows,
// gja global Schur positions).  Takes ownership of d_Linv, d_LinvT and d_K12.
void* afn_shard_from_parts(int n_local, int k, int n2, Comm* comm, const std::vector<int>& lm_idx,
                           const std::vector<int>& lm_row, const std::vector<int>& nl_pos,
                           const std::vector<int>& nl_row, double* d_Linv, double* d_LinvT, double* d_K12, bool fsai,
                           double schur_scale, const std::vector<int>& gia, const std::vector<int>& gja,
                           const std::vector<double>& gaa)
{
   AfnShard* S = new AfnShard();
   S->n = n_local;
   S->k = k;
   S->n2 = n2;
   S->comm = comm;
   S->fsai = fsai;
   S->schur_scale = schur_scale;
   S->m1 = (int)lm_idx.size();
   S->m2 = (int)nl_pos.size();
   S->Linv = d_Linv;
   S->LinvT = d_LinvT;
   S->K12 = d_K12;
   a12_shape(std::max(1, S->m2), S->cols, S->nblk);
   bool ok = !up(&S->lm_idx, lm_idx.data(), lm_idx.size()) && !up(&S->lm_row, lm_row.data(), lm_row.size()) &&
             !up(&S->nl_pos, nl_pos.data(), nl_pos.size()) && !up(&S->nl_row, nl_row.data(), nl_row.size());
   for (double** p : {&S->rp1, &S->y1, &S->t, &S->w})
      ok = ok && hipMalloc((void**)p, sizeof(double) * k) == hipSuccess;
   for (double** p : {&S->rp2, &S->y2, &S->v})
      ok = ok && hipMalloc((void**)p, sizeof(double) * std::max(1, S->m2)) == hipSuccess;
   ok = ok && hipMalloc((void**)&S->gbuf, sizeof(double) * n2) == hipSuccess &&
        hipMalloc((void**)&S->part, sizeof(double) * (size_t)S->nblk * k) == hipSuccess;
   if (ok && fsai) {
      std::vector<int> rows(S->m2);
      for (int i = 0; i < S->m2; i++) rows[i] = i;
      ok = !csr_rows_upload(gia, gja, gaa, rows, S->G);
      S->g_nnz = (long long)gja.size();
      // the transpose of the own rows, grouped by column: counting sort over the columns touched, rows ascending
      std::vector<int> cnt(n2 + 1, 0);
      for (int j : gja) cnt[j + 1]++;
      std::vector<int> tcols, tia(1, 0);
      std::vector<int> where(n2, -1);
      for (int c = 0; c < n2; c++)
         if (cnt[c + 1]) {
            where[c] = (int)tcols.size();
            tcols.push_back(c);
            tia.push_back(tia.back() + cnt[c + 1]);
         }
      std::vector<int> tja(gja.size()), fill(tia.begin(), tia.end() - 1);
      std::vector<double> taa(gja.size());
      for (int i = 0; i < S->m2; i++)
         for (int e = gia[i]; e < gia[i + 1]; e++) {
            const int slot = fill[where[gja[e]]]++;
            tja[slot] = i;
            taa[slot] = gaa[e];
         }
      std::vector<int> trows(tcols.size());
      for (size_t t = 0; t < tcols.size(); t++) trows[t] = (int)t;
      ok = ok && !csr_rows_upload(tia, tja, taa, trows, S->GTp) && !up(&S->tcols, tcols.data(), tcols.size()) &&
           hipMalloc((void**)&S->tbuf, sizeof(double) * std::max<size_t>(1, tcols.size())) == hipSuccess;
      S->gt_scatter = true;
   }
   if (!ok || hipStreamSynchronize(current_stream()) != hipSuccess) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnShardSetup: allocation or copy failed\n");
      afn_shard_free(S);
      return nullptr;
   }
   return S;
}

// ---- the FSAI handle from a device CSR: L^T by one radix sort of (column, row) keys -------------------------------
// key of entry p of row i: column ja[p] above, row i below, so the sorted order is L^T's rows (the columns of L) with
// each one's entries in ascending row order -- the order fsai_create's host counting sort produces
__global__ void k_csr_tkeys(const int* __restrict__ ia, const int* __restrict__ ja, int n,
                            unsigned long long* __restrict__ keys, int* __restrict__ vals, int* __restrict__ tcnt)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i >= n) return;
   for (int p = ia[i]; p < ia[i + 1]; p++) {
      keys[p] = ((unsigned long long)(unsigned)ja[p] << 32) | (unsigned)i;
      vals[p] = p;
      atomicAdd(tcnt + ja[p] + 1, 1);  // counts: any order gives the same sums
   }
}

__global__ void k_csr_tfill(const unsigned long long* __restrict__ keys, const int* __restrict__ vals,
                            const double* __restrict__ aa, size_t nnz, int* __restrict__ tja, double* __restrict__ taa)
{
   const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
   if (p >= nnz) return;
   tja[p] = (int)(unsigned)(keys[p] & 0xFFFFFFFFull);
   taa[p] = aa[vals[p]];
}

__global__ void k_count_nonfinite(const double* __restrict__ a, size_t count, unsigned long long* __restrict__ out)
{
   unsigned long long c = 0;
   for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x)
      c += isfinite(a[i]) ? 0ull : 1ull;
   if (c) atomicAdd(out, c);
}

long long count_nonfinite(const double* d, size_t count, hipStream_t s)
{
   unsigned long long* dc = nullptr;
   unsigned long long h = 0;
   if (hipMalloc((void**)&dc, sizeof(unsigned long long)) != hipSuccess) return -1;
   bool ok = hipMemsetAsync(dc, 0, sizeof(unsigned long long), s) == hipSuccess;
   if (ok && count) hipLaunchKernelGGL(k_count_nonfinite, dim3(1024), dim3(256), 0, s, d, count, dc);
   ok = ok && hipMemcpyAsync(&h, dc, sizeof(h), hipMemcpyDeviceToHost, s) == hipSuccess &&
        hipStreamSynchronize(s) == hipSuccess;
   (void)hipFree(dc);
   return ok ? (long long)h : -1;
}

void* fsai_create_from_device(int n, int* dia, int* dja, double* daa, const std::vector<int>& hia, hipStream_t s)
{
   FsaiDev* F = new FsaiDev();
   F->n = n;
   F->ia = dia;
   F->ja = dja;
   F->aa = daa;
   const size_t nnz = (size_t)hia[n];
   unsigned long long *k_in = nullptr, *k_out = nullptr;
   int *v_in = nullptr, *v_out = nullptr;
   void* tmp = nullptr;
   size_t tmp_bytes = 0;
   auto done = [&](bool ok) -> void* {
      (void)hipStreamSynchronize(s);
      for (void* p : {(void*)k_in, (void*)k_out, (void*)v_in, (void*)v_out, tmp}) (void)hipFree(p);
      if (!ok) {
         fprintf(stderr, "nfft4gp_amd: FSAI handle on the device: allocation or sort failed\n");
         fsai_free(F);
         return nullptr;
      }
      return F;
   };
   if (hipMalloc((void**)&F->tia, sizeof(int) * ((size_t)n + 1)) != hipSuccess ||
       hipMalloc((void**)&F->tja, sizeof(int) * std::max<size_t>(1, nnz)) != hipSuccess ||
       hipMalloc((void**)&F->taa, sizeof(double) * std::max<size_t>(1, nnz)) != hipSuccess ||
       hipMalloc((void**)&F->work, sizeof(double) * std::max(1, n)) != hipSuccess ||
       hipMalloc((void**)&k_in, sizeof(unsigned long long) * std::max<size_t>(1, nnz)) != hipSuccess ||
       hipMalloc((void**)&k_out, sizeof(unsigned long long) * std::max<size_t>(1, nnz)) != hipSuccess ||
       hipMalloc((void**)&v_in, sizeof(int) * std::max<size_t>(1, nnz)) != hipSuccess ||
       hipMalloc((void**)&v_out, sizeof(int) * std::max<size_t>(1, nnz)) != hipSuccess ||
       hipMemsetAsync(F->tia, 0, sizeof(int) * ((size_t)n + 1), s) != hipSuccess)
      return done(false);
   hipLaunchKernelGGL(k_csr_tkeys, dim3((n + 255) / 256), dim3(256), 0, s, (const int*)dia, (const int*)dja, n, k_in,
                      v_in, F->tia);
   int end_bit = 32;
   while (end_bit < 64 && (1ull << (end_bit - 32)) < (unsigned long long)n) end_bit++;
   if (hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, k_in, k_out, v_in, v_out, (int)nnz, 0, end_bit, s) !=
           hipSuccess ||
       hipMalloc(&tmp, std::max<size_t>(1, tmp_bytes)) != hipSuccess ||
       hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, k_in, k_out, v_in, v_out, (int)nnz, 0, end_bit, s) !=
           hipSuccess)
      return done(false);
   (void)hipFree(tmp);
   tmp = nullptr;
   tmp_bytes = 0;
   // tia: counts -> pointers (inclusive sum over tia[1..n])
   if (hipcub::DeviceScan::InclusiveSum(nullptr, tmp_bytes, F->tia + 1, F->tia + 1, n, s) != hipSuccess ||
       hipMalloc(&tmp, std::max<size_t>(1, tmp_bytes)) != hipSuccess ||
       hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, F->tia + 1, F->tia + 1, n, s) != hipSuccess)
      return done(false);
   if (nnz)
      hipLaunchKernelGGL(k_csr_tfill, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, (const unsigned long long*)k_out,
                         (const int*)v_out, (const double*)daa, nnz, F->tja, F->taa);
   // the workgroups' row spans of L and L^T (csr_partition, on the host pointers)
   std::vector<int> htia((size_t)n + 1);
   if (hipGetLastError() != hipSuccess ||
       hipMemcpyAsync(htia.data(), F->tia, sizeof(int) * ((size_t)n + 1), hipMemcpyDeviceToHost, s) != hipSuccess ||
       hipStreamSynchronize(s) != hipSuccess)
      return done(false);
   const std::vector<int> p = csr_partition(n, hia.data()), tp = csr_partition(n, htia.data());
   F->nparts = (int)p.size() - 1;
   F->ntparts = (int)tp.size() - 1;
   if (up(&F->part, p.data(), p.size()) || up(&F->tpart, tp.data(), tp.size())) return done(false);
   return done(true);
}

// an AFN apply object from factors already in HBM (afn_setup.hip); takes ownership of d_perm, d_Linv,
// d_K12 (hipMalloc'ed) and of the Schur FSAI handle S (an Nfft4GPAmdFsaiCreate handle of size n - k)
void* afn_create_device(int n, int k, int* d_perm, double* d_Linv, double* d_LinvT, double* d_K12, void* S,
                        double schur_scale)
{
   AfnDev* A = new AfnDev();
   A->schur_scale = schur_scale;
   A->n = n;
   A->k = k;
   A->n2 = n - k;
   A->S = (FsaiDev*)S;
   A->own_S = true;
   A->perm = d_perm;
   A->Linv = d_Linv;
   A->LinvT = d_LinvT;
   A->K12 = d_K12;
   a12_shape(A->n2, A->cols, A->nblk);
   if (hipMalloc((void**)&A->rp, sizeof(double) * n) != hipSuccess ||
       hipMalloc((void**)&A->y, sizeof(double) * n) != hipSuccess ||
       hipMalloc((void**)&A->t, sizeof(double) * std::max(1, k)) != hipSuccess ||
       hipMalloc((void**)&A->part, sizeof(double) * std::max<size_t>(1, (size_t)A->nblk * k)) != hipSuccess) {
      Nfft4GPAmdAfnFree(A);
      return nullptr;
   }
   return A;
}

}  // namespace nfft4gp_amd

using namespace nfft4gp_amd;

extern "C" {

void* Nfft4GPAmdFsaiCreate(int n, const int* ia, const int* ja, const double* aa)
{
   if (!device_ok()) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdFsaiCreate: no HIP device visible (no CPU fallback).\n");
      return nullptr;
   }
   return fsai_create(n, ia, ja, aa);
}

int Nfft4GPAmdFsaiSolve(void* fsai, int n, double* x, double* rhs)
{
   FsaiDev* F = (FsaiDev*)fsai;
   if (!F || n != F->n) return -1;
   return with_device_vectors(n, x, rhs, &fsai_apply_obj, F);
}

void Nfft4GPAmdFsaiFree(void* fsai) { fsai_free((FsaiDev*)fsai); }

void* Nfft4GPAmdAfnCreate(int n, int k, const int* perm, const double* L11, const double* K12, void* fsai_schur)
{
   if (!device_ok()) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnCreate: no HIP device visible (no CPU fallback).\n");
      return nullptr;
   }
   FsaiDev* S = (FsaiDev*)fsai_schur;
   const bool ok = n > 0 && k >= 0 && k <= n && (k == 0 || L11) && (k == n || (S && S->n == n - k)) &&
                   (k == 0 || k == n || (perm && K12));
   if (!ok) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnCreate: needs 0 <= k <= n, L11 (k > 0), an FSAI of size n - k "
                      "(k < n), perm and K12 (0 < k < n)\n");
      return nullptr;
   }
   // L11^{-1} on the host (k x k lower triangular inverse)
   std::vector<double> L(L11, L11 + (size_t)k * k), G((size_t)k * k, 0.0);
   for (int j = 0; j < k; j++) {
      G[j + (size_t)j * k] = 1.0 / L[j + (size_t)j * k];
      for (int i = j + 1; i < k; i++) {
         double v = 0.0;
         for (int m = j; m < i; m++) v += L[i + (size_t)m * k] * G[m + (size_t)j * k];
         G[i + (size_t)j * k] = -v / L[i + (size_t)i * k];
      }
   }
   std::vector<double> GT((size_t)k * k);
   for (int j = 0; j < k; j++)
      for (int i = 0; i < k; i++) GT[j + (size_t)i * k] = G[i + (size_t)j * k];
   AfnDev* A = new AfnDev();
   A->n = n;
   A->k = k;
   A->n2 = n - k;
   A->S = S;
   a12_shape(A->n2, A->cols, A->nblk);
   const bool mid = k > 0 && k < n;
   if ((mid && up(&A->perm, perm, (size_t)n)) || up(&A->Linv, G.data(), G.size()) ||
       up(&A->LinvT, GT.data(), GT.size()) ||
       (mid && up(&A->K12, K12, (size_t)k * A->n2)) || hipMalloc((void**)&A->rp, sizeof(double) * n) != hipSuccess ||
       hipMalloc((void**)&A->y, sizeof(double) * n) != hipSuccess ||
       hipMalloc((void**)&A->t, sizeof(double) * std::max(1, k)) != hipSuccess ||
       hipMalloc((void**)&A->part, sizeof(double) * std::max<size_t>(1, (size_t)A->nblk * k)) != hipSuccess) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnCreate: allocation failed\n");
      Nfft4GPAmdAfnFree(A);
      return nullptr;
   }
   return A;
}

int Nfft4GPAmdAfnSolve(void* afn, int n, double* x, double* rhs)
{
   AfnDev* A = (AfnDev*)afn;
   if (!A || n != A->n) return -1;
   return with_device_vectors(n, x, rhs, &afn_apply_obj, A);
}

void Nfft4GPAmdAfnFree(void* afn)
{
   AfnDev* A = (AfnDev*)afn;
   if (!A) return;
   for (void* p : {(void*)A->perm, (void*)A->Linv, (void*)A->LinvT, (void*)A->K12, (void*)A->K12f, (void*)A->rp,
                   (void*)A->y, (void*)A->t, (void*)A->part, (void*)A->u, (void*)A->w})
      (void)hipFree(p);
   // the Schur complement's FSAI handle stays with its creator (Nfft4GPAmdFsaiFree) unless the AFN was
   // set up on the device (Nfft4GPAmdAfnSetup), which owns it
   if (A->own_S) fsai_free(A->S);
   delete A;
}

__global__ void k_afn_to_f32(const double* __restrict__ a, size_t count, float* __restrict__ b)
{
   for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x)
      b[i] = (float)a[i];
}

int Nfft4GPAmdAfnSetStorage(void* afn, int bits)
{
   AfnDev* A = (AfnDev*)afn;
   if (!A || (bits != 32 && bits != 64)) return -1;
   hipStream_t s = current_stream();
   if (bits == 64) {
      if (A->K12f) {
         NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
         NFFT4GP_HIP_CHECK(hipFree(A->K12f));
         A->K12f = nullptr;
      }
      return 0;
   }
   if (A->K12f || !A->K12) return 0;
   const size_t count = (size_t)A->k * A->n2;
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&A->K12f, sizeof(float) * std::max<size_t>(1, count)));
   hipLaunchKernelGGL(k_afn_to_f32, dim3(4096), dim3(256), 0, s, (const double*)A->K12, count, A->K12f);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int Nfft4GPAmdAfnSetOperator(void* afn, void* op)
{
   AfnDev* A = (AfnDev*)afn;
   if (!A) return -1;
   if (!op) {
      A->op = nullptr;
      return 0;
   }
   int nl = 0, ng = 0, rb = 0;
   if (additive_rows(op, &nl, &ng, &rb) || nl != A->n || ng != A->n) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAfnSetOperator: needs this library's additive handle over the AFN's "
                      "%d points (whole rows, after its setup)\n", A->n);
      return -1;
   }
   if (A->k == 0 || A->k == A->n) return 0;  // no K12 products (afn.c:101-110)
   if (!A->u) NFFT4GP_HIP_CHECK(hipMalloc((void**)&A->u, sizeof(double) * A->n));
   if (!A->w) NFFT4GP_HIP_CHECK(hipMalloc((void**)&A->w, sizeof(double) * A->n));
   A->op = op;
   return 0;
}

void* Nfft4GPAmdAfnShard(void* afn, int row_begin, int row_end, void* comm)
{
   if (!afn || !comm) return nullptr;
   return afn_shard_create((const AfnDev*)afn, row_begin, row_end, (Comm*)comm);
}

int Nfft4GPAmdDistAfnSolve(void* dafn, int n, double* x, double* rhs)
{
   AfnShard* S = (AfnShard*)dafn;
   if (!S || n != S->n) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdDistAfnSolve: size %d, this rank holds %d rows\n", n, S ? S->n : -1);
      return -1;
   }
   if (n > 0 && (!is_device_ptr(x) || !is_device_ptr(rhs))) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdDistAfnSolve takes device vectors\n");
      return -1;
   }
   return afn_shard_apply(S, x, rhs, current_stream());
}

void Nfft4GPAmdDistAfnFree(void* dafn) { afn_shard_free((AfnShard*)dafn); }

int Nfft4GPAmdAfnShardInfo(void* dafn, int* m1, int* m2, long long* k12_doubles, long long* g_nnz)
{
   const AfnShard* S = (const AfnShard*)dafn;
   if (!S) return -1;
   if (m1) *m1 = S->m1;
   if (m2) *m2 = S->m2;
   if (k12_doubles) *k12_doubles = (long long)S->k * S->m2;
   if (g_nnz) *g_nnz = S->g_nnz;
   return 0;
}

int Nfft4GPAmdAfnInfo(void* afn, int* k, int* perm, int* ia, int* ja, double* aa)
{
   AfnDev* A = (AfnDev*)afn;
   if (!A) return -1;
   if (k) *k = A->k;
   if (perm && A->perm) NFFT4GP_HIP_CHECK(hipMemcpy(perm, A->perm, sizeof(int) * A->n, hipMemcpyDeviceToHost));
   if (!A->S) return 0;
   const int n2 = A->S->n;
   int nnz = 0;
   NFFT4GP_HIP_CHECK(hipMemcpy(&nnz, A->S->ia + n2, sizeof(int), hipMemcpyDeviceToHost));
   if (ia) NFFT4GP_HIP_CHECK(hipMemcpy(ia, A->S->ia, sizeof(int) * (n2 + 1), hipMemcpyDeviceToHost));
   if (ja) NFFT4GP_HIP_CHECK(hipMemcpy(ja, A->S->ja, sizeof(int) * nnz, hipMemcpyDeviceToHost));
   if (aa) NFFT4GP_HIP_CHECK(hipMemcpy(aa, A->S->aa, sizeof(double) * nnz, hipMemcpyDeviceToHost));
   return nnz;
}

}  // extern "C"
