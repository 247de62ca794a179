// csr.hpp -- one CSR row's dot product with a gathered vector, in column order (device code).
//
// r += a[j] * x[ja[j]] for j in [j0, j1) in order -- the reference's Nfft4GPCsrMv accumulation
// (matops.c:139-272), unfused, so the result is bitwise the reference's -- with the row taken 8 entries
// at a time: their column indices and values, then their 8 gathers of x, are in flight together, so a
// row costs about two memory latencies per 8 entries instead of two per entry (a KNN pattern's gathers
// are scattered over x).
#pragma once

#include <hip/hip_runtime.h>

namespace nfft4gp_amd {

__device__ __forceinline__ double csr_row_dot(const int* __restrict__ ja, const double* __restrict__ a,
                                              const double* __restrict__ x, int j0, int j1, double r)
{
#pragma clang fp contract(off)
   constexpr int U = 8;
   for (int jb = j0; jb < j1; jb += U) {
      int c[U];
      double av[U], xv[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
         const bool ok = jb + u < j1;
         c[u] = ok ? ja[jb + u] : 0;
         av[u] = ok ? a[jb + u] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < U; u++) xv[u] = jb + u < j1 ? x[c[u]] : 0.0;
#pragma unroll
      for (int u = 0; u < U; u++)
         if (jb + u < j1) r += av[u] * xv[u];
   }
   return r;
}

}  // namespace nfft4gp_amd
