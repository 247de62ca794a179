// csr.hpp -- CSR rows times a gathered vector, each row summed in column order (device code).
//
// r += a[j] * x[ja[j]] for j in [j0, j1) in order -- the reference's Nfft4GPCsrMv accumulation
// (matops.c:139-272), unfused, so the result is bitwise the reference's.
#pragma once

#include <hip/hip_runtime.h>

namespace nfft4gp_amd {

// The rows [r0, r0 + T) of one workgroup (T = blockDim.x threads, a thread per row).  The rows' entries
// [ia[r0], ia[r0 + T]) are contiguous, so the workgroup takes them in chunks of CH entries: every thread
// loads CH / T of them coalesced, gathers their x values (all in flight together) and stores the rounded
// products a[j] * x[ja[j]] in LDS; then each thread adds its own row's products in column order.  With
// contraction off, r += a * x is round(r + round(a * x)), so the sums are bitwise csr_row_dot's, and the
// gathers of a long row (a column of a KNN pattern's transpose can hold thousands) are spread over the
// whole workgroup instead of running 8 at a time on one thread.  beta_one: rows start from y.
// Rows [r0, r1) (r1 - r0 <= T): a workgroup's rows, a fixed T of them or a span sized by entry count.
template <int T, int CH>
__device__ __forceinline__ void csr_rows_staged(const int* __restrict__ ia, const int* __restrict__ ja,
                                                const double* __restrict__ a, const double* __restrict__ x,
                                                double* __restrict__ y, int r0, int r1, bool beta_one)
{
#pragma clang fp contract(off)
   static_assert(CH % T == 0, "chunk must be a multiple of the workgroup");
   constexpr int K = CH / T;
   __shared__ double s_p[CH];
   const int tid = threadIdx.x;
   const int row = r0 + tid;
   const int e0 = ia[r0];
   const int e1 = ia[r1];
   int j0 = 0, j1 = 0;
   double r = 0.0;
   if (row < r1) {
      j0 = ia[row];
      j1 = ia[row + 1];
      if (beta_one) r = y[row];
   }
   for (int c = e0; c < e1; c += CH) {
      const int m = min(CH, e1 - c);
      int cj[K];
      double ca[K], xv[K];
#pragma unroll
      for (int k = 0; k < K; k++) {
         const int i = tid + k * T;
         cj[k] = i < m ? ja[c + i] : 0;
         ca[k] = i < m ? a[c + i] : 0.0;
      }
#pragma unroll
      for (int k = 0; k < K; k++) xv[k] = tid + k * T < m ? x[cj[k]] : 0.0;
      if (c != e0) __syncthreads();  // every thread has summed the previous chunk
#pragma unroll
      for (int k = 0; k < K; k++) s_p[tid + k * T] = ca[k] * xv[k];
      __syncthreads();
      const int je = min(j1, c + m) - c;
      for (int j = max(j0, c) - c; j < je; j++) r += s_p[j];
   }
   if (row < r1) y[row] = r;
}

}  // namespace nfft4gp_amd
