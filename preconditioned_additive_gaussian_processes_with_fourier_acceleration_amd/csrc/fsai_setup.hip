// fsai_setup.hip -- the FSAI preconditioner built on the GPU, with gradients, behind the reference's
// interface (SRC/preconds/fsai.h:46-207):
//
//   Nfft4GPAmdPrecondFsaiCreate / SetLfil / Reset / Free          fsai.c:3-104
//   Nfft4GPAmdPrecondFsaiSetupWithKernel (precond_kernel_setup)   fsai.c:302-312 -> :314-673
//       pattern  Nfft4GPDistanceEuclidKnn (kernels.c:121-278): row i < lfil is dense (0..i); row i >= lfil
//                holds the lfil-1 nearest points among 0..i-1, then i.  k_knn: one workgroup per row, an
//                MSB-first radix select on the bits of the squared distances (non-negative doubles order
//                like their bit patterns), then a rank sort of the survivors by (distance, index).
//       values   per row, the kernel submatrix K_a of its points, L_a = chol(K_a), A_ai = K_a^{-1} e_k /
//                sqrt(e_k' K_a^{-1} e_k); with gradients dA_g = K_a^{-1}(-dK_g A_ai) - 1/2 (.)_k dd A_ai
//                (fsai.c:530-563).  k_fsai_rows: one wave per row, K_a in LDS.
//   Nfft4GPAmdPrecondFsaiSolve  (func_solve)   x = L^T (L rhs)                 fsai.c:106-123
//   Nfft4GPAmdPrecondFsaiInvL / InvLT          L^{-1} rhs, L^{-T} rhs          fsai.c:675-728
//   Nfft4GPAmdPrecondFsaiDvp    (func_dvp)                                     fsai.c:125-216
//   Nfft4GPAmdPrecondFsaiTrace  (func_trace)   2 sum_i dL_g(i,i) / L(i,i)      fsai.c:218-276
//   Nfft4GPAmdPrecondFsaiLogdet (func_logdet)  2 sum_i log(1 / L(i,i))         fsai.c:278-301
//
// The triangular solves are CSR SpTRSVs over level sets computed once at setup (a row's level is one
// more than its dependencies'; ~250 levels for 2e4 KNN rows): ONE workgroup walks the levels with a
// barrier between them, so there is no grid-wide synchronisation and no spinning.  Each row sums in the
// reference's order with unfused multiply-add, so given the same factors the solves, products and Dvp
// are bitwise the reference's.
//
// Kernel: the plain (non-additive) Gaussian or Matern-1/2 kernel of all d columns of `data` with the
// parameters of `fkernel_params` (_params[0] = f, _params[1] = l, _noise_level = mu; kernels.c:680-1289,
// :2390-3033), as the reference's FSAI runs on Nfft4GPKernelGaussianKernel.  The reference's FSAI on its
// additive kernel would evaluate buffer rows instead of the pattern's points (kernels.c:3160 ignores
// the data argument); this library does not reproduce that.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "callbacks.hpp"
#include "csr.hpp"
#include "internal.h"
#include "kernel_eval.hpp"

using namespace nfft4gp_amd;

namespace {

constexpr int kFsaiMaxK = 64;      // entries per row (lfil) the per-row kernel holds in LDS
constexpr int kKnnThreads = 256;
constexpr int kKnnGather = 256;    // survivors of the radix select sorted directly
constexpr int kMaxDims = 256;      // features of `data`
constexpr int kTrsvThreads = 1024;
int knn_fallback_rows = 0;  // rows of the last FSAI setup that k_knn_bounded handed to k_knn

__device__ __forceinline__ double sqdist(const double* __restrict__ X, int ldim, int d, const double* xi, int j)
{
   double s = 0.0;
   for (int c = 0; c < d; c++) {
      const double t = X[(size_t)c * ldim + j] - xi[c];
      s = fma(t, t, s);
   }
   return s;
}

// pattern rows i in [lfil, n): ja[ia[i] .. ia[i] + lfil - 2] = the lfil-1 nearest of 0..i-1 by
// (squared distance, index), ja[ia[i] + lfil - 1] = i.  Grid-stride over rows, or over the rows of
// `rows` (nrows of them) when given: the rows k_knn_bounded could not settle.
__global__ __launch_bounds__(kKnnThreads) void k_knn(const double* __restrict__ X, int ldim, int n, int d, int lfil,
                                                     const int* __restrict__ ia, int* __restrict__ ja,
                                                     const int* __restrict__ rows, int nrows)
{
   __shared__ unsigned int hist[256];
   __shared__ double s_xi[kMaxDims];
   __shared__ unsigned long long s_key[kKnnGather + kFsaiMaxK];
   __shared__ int s_idx[kKnnGather + kFsaiMaxK];
   __shared__ int s_nsel, s_ngat;
   __shared__ unsigned long long s_prefix;
   __shared__ int s_bits, s_need, s_eq;
   const int tid = threadIdx.x;
   const int K = lfil - 1;
   const int nloop = rows ? nrows : n - lfil;
   for (int it = blockIdx.x; it < nloop; it += gridDim.x) {
      const int i = rows ? rows[it] : lfil + it;
      for (int c = tid; c < d; c += kKnnThreads) s_xi[c] = X[(size_t)c * ldim + i];
      if (tid == 0) {
         s_prefix = 0ull;
         s_bits = 0;
         s_need = K;
         s_eq = i;
      }
      __syncthreads();
      // MSB-first radix select: narrow the prefix of the K-th smallest key byte by byte until the
      // candidates that share it fit the gather buffer
      while (s_bits < 64 && s_eq > kKnnGather) {
         const int bits = s_bits;
         const unsigned long long prefix = s_prefix;
         for (int b = tid; b < 256; b += kKnnThreads) hist[b] = 0u;
         __syncthreads();
         for (int j = tid; j < i; j += kKnnThreads) {
            const unsigned long long u = (unsigned long long)__double_as_longlong(sqdist(X, ldim, d, s_xi, j));
            if (bits == 0 || (u >> (64 - bits)) == prefix) atomicAdd(&hist[(u >> (56 - bits)) & 255ull], 1u);
         }
         __syncthreads();
         if (tid == 0) {
            unsigned int cum = 0;
            int b = 0;
            for (; b < 255; b++) {
               if (cum + hist[b] >= (unsigned)s_need) break;
               cum += hist[b];
            }
            s_need -= (int)cum;
            s_eq = (int)hist[b];
            s_prefix = (prefix << 8) | (unsigned long long)b;
            s_bits = bits + 8;
         }
         __syncthreads();
      }
      // collect: keys below the prefix are in; keys equal to it compete for the remaining s_need slots
      if (tid == 0) {
         s_nsel = 0;
         s_ngat = 0;
      }
      __syncthreads();
      {
         const int bits = s_bits;
         const unsigned long long prefix = s_prefix;
         for (int j = tid; j < i; j += kKnnThreads) {
            const unsigned long long u = (unsigned long long)__double_as_longlong(sqdist(X, ldim, d, s_xi, j));
            const unsigned long long top = bits == 0 ? 0ull : (u >> (64 - bits));
            if (bits > 0 && top < prefix) {
               const int p = atomicAdd(&s_nsel, 1);
               s_key[kKnnGather + p] = u;
               s_idx[kKnnGather + p] = j;
            } else if (bits == 0 || top == prefix) {
               const int p = atomicAdd(&s_ngat, 1);
               if (p < kKnnGather) {
                  s_key[p] = u;
                  s_idx[p] = j;
               }
            }
         }
      }
      __syncthreads();
      // rank the gathered candidates by (key, index); the first s_need join the selection
      const int ng = min(s_ngat, kKnnGather);
      const int nsel0 = s_nsel;
      __syncthreads();
      for (int e = tid; e < ng; e += kKnnThreads) {
         const unsigned long long ke = s_key[e];
         const int ie = s_idx[e];
         int rank = 0;
         for (int o = 0; o < ng; o++) {
            const unsigned long long ko = s_key[o];
            rank += (ko < ke || (ko == ke && s_idx[o] < ie)) ? 1 : 0;
         }
         if (rank < K - nsel0) {
            s_key[kKnnGather + nsel0 + rank] = ke;
            s_idx[kKnnGather + nsel0 + rank] = ie;
         }
      }
      __syncthreads();
      // final order of the K neighbours: by (key, index), then the point itself
      const int row = ia[i];
      for (int e = tid; e < K; e += kKnnThreads) {
         const unsigned long long ke = s_key[kKnnGather + e];
         const int ie = s_idx[kKnnGather + e];
         int rank = 0;
         for (int o = 0; o < K; o++) {
            const unsigned long long ko = s_key[kKnnGather + o];
            rank += (ko < ke || (ko == ke && s_idx[kKnnGather + o] < ie)) ? 1 : 0;
         }
         ja[row + rank] = ie;
      }
      if (tid == 0) ja[row + K] = i;
      __syncthreads();
   }
}

// The same pattern rows, kKnnRows consecutive rows per workgroup sharing every load of a point (the
// scan is bound by the on-chip bandwidth of re-reading the earlier points, so the rows per workgroup
// set the speed), in two passes over the earlier points instead of k_knn's three to four:
//   sample  the squared distances to points 0..S-1 (S = min(i0, 4096)) histogrammed by exponent (256
//           bins over 2^-224 .. 2^31, clamped) give the bin of the sample's (lfil-1)-th smallest, so
//           every true neighbour has a key below tau = the bin's upper end;
//   count   keys below tau, binned by (exponent - (E-16), 4 top mantissa bits) with tau = 2^E -- 256
//           monotone bins over [2^(E-16), tau), smaller keys in bin 0 -- locate the bin b* of the
//           (lfil-1)-th key;
//   collect keys in bins below b* are in, keys in b* (at most kKnnGather2) are ranked by (key, index).
// Only keys below tau touch the LDS histograms (a few percent of them).  A row whose bin b* holds more
// than kKnnGather2 keys (duplicates, pathological data) is appended to `fail` for k_knn.  d <= 64.
constexpr int kKnnRows = 16;
constexpr int kKnnPoints = 2;  // points per thread in the distance scans (knn_scan)
constexpr int kKnnSample = 4096;
constexpr int kKnnGather2 = 128;
constexpr int kKnnMaxDims2 = 64;
constexpr int kExpBase = 1023 - 224;
__device__ __forceinline__ int knn_bin(unsigned long long u, int base)
{
   const int e = (int)(u >> 52);
   return (e < base) ? 0 : (((e - base) << 4) | (int)((u >> 48) & 15ull));
}

// The squared distances of points j in [0, jend) to the workgroup's R query rows (q in LDS), P points
// per thread so that every LDS read of a query coordinate serves P distances, and the next feature's
// loads issued before the current feature's arithmetic.  Each distance is the same sum as sqdist's:
// t = x_j - q, s = fma(t, t, s) over the features in order.  f(j, acc) sees the R keys of point j.
template <int P, int R, typename F>
__device__ __forceinline__ void knn_scan(const double* __restrict__ X, int ldim, int d, const double (*q)[R],
                                         int jend, F&& f)
{
   constexpr int T = kKnnThreads;
   for (int jb = threadIdx.x; jb < jend; jb += T * P) {
      double acc[P][R];
#pragma unroll
      for (int p = 0; p < P; p++)
#pragma unroll
         for (int r = 0; r < R; r++) acc[p][r] = 0.0;
      double xn[P];
#pragma unroll
      for (int p = 0; p < P; p++) xn[p] = jb + p * T < jend ? X[jb + p * T] : 0.0;
      for (int c = 0; c < d; c++) {
         double xc[P];
#pragma unroll
         for (int p = 0; p < P; p++) xc[p] = xn[p];
         if (c + 1 < d) {
#pragma unroll
            for (int p = 0; p < P; p++)
               xn[p] = jb + p * T < jend ? X[(size_t)(c + 1) * ldim + jb + p * T] : 0.0;
         }
#pragma unroll
         for (int r = 0; r < R; r++) {
            const double qv = q[c][r];
#pragma unroll
            for (int p = 0; p < P; p++) {
               const double t = xc[p] - qv;
               acc[p][r] = fma(t, t, acc[p][r]);
            }
         }
      }
#pragma unroll
      for (int p = 0; p < P; p++)
         if (jb + p * T < jend) f(jb + p * T, acc[p]);
   }
}

template <int P>
__global__ __launch_bounds__(kKnnThreads) void k_knn_bounded(const double* __restrict__ X, int ldim, int n, int d,
                                                             int lfil, const int* __restrict__ ia,
                                                             int* __restrict__ ja, int* __restrict__ fail,
                                                             int* __restrict__ nfail, const int* __restrict__ rows,
                                                             int nrows)
{
   constexpr int R = kKnnRows;
   __shared__ double q[kKnnMaxDims2][R];
   __shared__ unsigned int h0[R][256];
   __shared__ unsigned int h1[R][256];
   __shared__ unsigned long long s_key[R][kKnnGather2 + kFsaiMaxK];
   __shared__ int s_idx[R][kKnnGather2 + kFsaiMaxK];
   __shared__ unsigned long long s_tau[R];
   __shared__ int s_base[R], s_bstar[R], s_ok[R];
   __shared__ int s_nsel[R], s_ngat[R], s_row[R];
   const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
   const int K = lfil - 1;
   // rows: ascending row indices (nrows of them) instead of lfil..n-1
   const int nall = rows ? nrows : n - lfil;
   const int ngroups = (nall + R - 1) / R;
   for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
      const int nr = min(R, nall - g * R);
      const int i0 = rows ? rows[g * R] : lfil + g * R;
      if (tid < R) s_row[tid] = tid < nr ? (rows ? rows[g * R + tid] : i0 + tid) : n;
      __syncthreads();
      for (int e = tid; e < R * d; e += kKnnThreads) {
         const int r = e / d, c = e % d;
         q[c][r] = (r < nr) ? X[(size_t)c * ldim + s_row[r]] : 0.0;
      }
      for (int e = tid; e < R * 256; e += kKnnThreads) {
         h0[e / 256][e % 256] = 0u;
         h1[e / 256][e % 256] = 0u;
      }
      if (tid < R) {
         s_nsel[tid] = 0;
         s_ngat[tid] = 0;
      }
      __syncthreads();
      // sample: exponent histogram of keys to points 0..S-1 (S <= i0 <= every row's i)
      const int S = min(i0, kKnnSample);
      knn_scan<P, R>(X, ldim, d, q, S, [&](int, const double* acc) {
#pragma unroll
         for (int r = 0; r < R; r++)
            if (r < nr) {
               const int e = (int)((unsigned long long)__double_as_longlong(acc[r]) >> 52);
               atomicAdd(&h0[r][min(255, max(0, e - kExpBase))], 1u);
            }
      });
      __syncthreads();
      // one wave per row: the first bin where the cumulative count reaches K
      for (int r = wave; r < nr; r += kKnnThreads / 64) {
         unsigned int loc = 0;
         for (int b = 0; b < 4; b++) loc += h0[r][lane * 4 + b];
         unsigned int incl = loc;
         for (int off = 1; off < 64; off <<= 1) {
            const unsigned int o = __shfl_up(incl, off, 64);
            if (lane >= off) incl += o;
         }
         const unsigned long long hit = __ballot(incl >= (unsigned)K);
         const int first = __ffsll((long long)hit) - 1;
         if (lane == first) {
            unsigned int cum = incl - loc;
            int b = lane * 4;
            for (;; b++) {
               cum += h0[r][b];
               if (cum >= (unsigned)K) break;
            }
            const int E = b + kExpBase + 1;  // keys of bin b have exponents < E (bin 255: any)
            s_tau[r] = (b == 255) ? ~0ull : ((unsigned long long)E << 52);
            s_base[r] = ((b == 255) ? 2047 : E) - 16;
         }
      }
      __syncthreads();
      // count: keys below tau by (exponent, 4 mantissa bits)
      const int jmax = s_row[nr - 1];
      knn_scan<P, R>(X, ldim, d, q, jmax, [&](int j, const double* acc) {
#pragma unroll
         for (int r = 0; r < R; r++) {
            const unsigned long long u = (unsigned long long)__double_as_longlong(acc[r]);
            if (r < nr && j < s_row[r] && u < s_tau[r]) atomicAdd(&h1[r][knn_bin(u, s_base[r])], 1u);
         }
      });
      __syncthreads();
      for (int r = wave; r < nr; r += kKnnThreads / 64) {
         unsigned int loc = 0;
         for (int b = 0; b < 4; b++) loc += h1[r][lane * 4 + b];
         unsigned int incl = loc;
         for (int off = 1; off < 64; off <<= 1) {
            const unsigned int o = __shfl_up(incl, off, 64);
            if (lane >= off) incl += o;
         }
         const unsigned long long hit = __ballot(incl >= (unsigned)K);
         const int first = __ffsll((long long)hit) - 1;
         if (lane == first) {
            unsigned int cum = incl - loc;
            int b = lane * 4;
            for (;; b++) {
               if (cum + h1[r][b] >= (unsigned)K) break;
               cum += h1[r][b];
            }
            s_bstar[r] = b;
            s_ok[r] = (h1[r][b] <= (unsigned)kKnnGather2) ? 1 : 0;
         }
      }
      __syncthreads();
      // collect
      knn_scan<P, R>(X, ldim, d, q, jmax, [&](int j, const double* acc) {
#pragma unroll
         for (int r = 0; r < R; r++) {
            const unsigned long long u = (unsigned long long)__double_as_longlong(acc[r]);
            if (r < nr && s_ok[r] && j < s_row[r] && u < s_tau[r]) {
               const int b = knn_bin(u, s_base[r]);
               if (b < s_bstar[r]) {
                  const int p = atomicAdd(&s_nsel[r], 1);
                  s_key[r][kKnnGather2 + p] = u;
                  s_idx[r][kKnnGather2 + p] = j;
               } else if (b == s_bstar[r]) {
                  const int p = atomicAdd(&s_ngat[r], 1);
                  s_key[r][p] = u;
                  s_idx[r][p] = j;
               }
            }
         }
      });
      __syncthreads();
      // rank the bin-b* keys by (key, index); the first K - below join (one wave per row)
      for (int r = wave; r < nr; r += kKnnThreads / 64) {
         if (!s_ok[r]) continue;
         const int ng = s_ngat[r], nsel0 = s_nsel[r];
         for (int e = lane; e < ng; e += 64) {
            const unsigned long long ke = s_key[r][e];
            const int ie = s_idx[r][e];
            int rank = 0;
            for (int o = 0; o < ng; o++) {
               const unsigned long long ko = s_key[r][o];
               rank += (ko < ke || (ko == ke && s_idx[r][o] < ie)) ? 1 : 0;
            }
            if (rank < K - nsel0) {
               s_key[r][kKnnGather2 + nsel0 + rank] = ke;
               s_idx[r][kKnnGather2 + nsel0 + rank] = ie;
            }
         }
      }
      __syncthreads();
      for (int r = wave; r < nr; r += kKnnThreads / 64) {
         const int i = s_row[r];
         if (!s_ok[r]) {
            if (lane == 0) fail[atomicAdd(nfail, 1)] = i;
            continue;
         }
         const int row = ia[i];
         for (int e = lane; e < K; e += 64) {
            const unsigned long long ke = s_key[r][kKnnGather2 + e];
            const int ie = s_idx[r][kKnnGather2 + e];
            int rank = 0;
            for (int o = 0; o < K; o++) {
               const unsigned long long ko = s_key[r][kKnnGather2 + o];
               rank += (ko < ke || (ko == ke && s_idx[r][kKnnGather2 + o] < ie)) ? 1 : 0;
            }
            ja[row + rank] = ie;
         }
         if (lane == 0) ja[row + K] = i;
      }
      __syncthreads();
   }
}

// The same pattern rows from fp32 screening keys: the scans of k_knn_bounded run on an fp32 copy of the
// points with the key of point j to row r kept as acc = -(|x_j|^2 + |q_r|^2) / 2 + x_j.q_r, so key~ =
// max(0, -2 acc) and "key~ < T" is the single compare acc > -T/2 against a workgroup-uniform value (one
// packed fp32 FMA per two (point, row) pairs per feature, half the bytes per point, 32 rows per workgroup;
// the fp64 scan spends a subtract and an FMA per pair per feature).  Only the few candidates left are
// ranked by the exact fp64 key sqdist() computes:
//   sample  two passes over points 0..S-1 (S = min(i0, 4096)): exponent histogram, then 16 bins per
//           octave below it; T1 = the upper end of the bin of the sample's (lfil-1)-th smallest key~;
//   count   key~ < T1 over all earlier points by (exponent, 4 mantissa bits), 16 octaves below T1: U = the
//           upper end of the bin b* holding the (lfil-1)-th smallest, so lfil-1 points have key~ < U;
//   collect every earlier point with key~ <= U + 2 m, where m bounds |key~ - key| (below);
//   exact   one wave per row: key = sqdist's sum, rank the candidates by (key, index), the first lfil-1
//           are the row.
// |key~ - key| <= m: rounding the coordinates to fp32 moves sqrt(key) by at most u (|x_j| + |q|) (u =
// 2^-24); the fp32 norms, the start value and the d-term sum add at most (6 d + 6) u M^2, with M^2 =
// max_j |x_j|^2, so |key~ - key| <= (6 d + 15) u M^2; m = (8 d + 64) u M^2.  The lfil-1 points with key~ <
// U have key < U + m, so every true neighbour (key <= the (lfil-1)-th smallest) has key~ < U + 2 m in any
// scan and is collected; ranking the collected set by the exact key is therefore the exact selection, ties
// by index included.  A row with more than kScrCap candidates (duplicates, coordinates far from the origin
// against their spread) goes to `fail` for k_knn, as does every row when M^2 is not finite.
constexpr int kScrRowBlocks = 1;  // 32-row MFMA tiles per workgroup; each point tile is read by that many waves (2: same time)
constexpr int kScrRows = 32 * kScrRowBlocks;
constexpr int kScrThreads = 512;
constexpr int kScrCap = 160;
constexpr int kScrSample = 4096;
// the count scan over a 1/sub subset of the points before the group once there are kScrSubFrom of them (sub = 2;
// NFFT4GP_AMD_KNN_SUB overrides, 1 = every point).  Config-C AFN setup (profiles/r04_knn_sub_ab.txt): sub 1 / 2
// / 3 / 4: 1.37-1.43 / 1.18-1.22 / 1.19-1.21 / 1.27-1.28 s -- at 4 the collect overflows its 160 candidates in
// ~3 % of the rows (d = 32) and those rows take the fp64 fallback
constexpr int kScrSubFrom = 65536;
#ifndef KNN_SCR_WAVES
#define KNN_SCR_WAVES 2  // waves per SIMD the screen kernels are compiled for
#endif

// Xf = fp32 copy of X (column-major, leading dimension n, zero features d..dp-1), nx = fl32 squared norms,
// *m2 = bits of max nx
__global__ __launch_bounds__(256) void k_knn_prep(const double* __restrict__ X, int ldim, int n, int d, int dp,
                                                  float* __restrict__ Xf, float* __restrict__ nx,
                                                  unsigned int* __restrict__ m2)
{
   unsigned int mx = 0u;
   for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
      float a = 0.f;
      for (int c = 0; c < d; c++) {
         const float v = (float)X[(size_t)c * ldim + j];
         Xf[(size_t)c * n + j] = v;
         a = fmaf(v, v, a);
      }
      for (int c = d; c < dp; c++) Xf[(size_t)c * n + j] = 0.f;
      nx[j] = a;
      mx = max(mx, __float_as_uint(a));  // non-negative floats order like their bits (NaN above inf)
   }
   for (int off = 32; off > 0; off >>= 1) mx = max(mx, (unsigned int)__shfl_xor((int)mx, off, 64));
   if ((threadIdx.x & 63) == 0) atomicMax(m2, mx);
}

__device__ __forceinline__ int knn_bin32(unsigned int u, int base)
{
   const int e = (int)(u >> 23);
   return (e < base) ? 0 : (((e - base) << 4) | (int)((u >> 19) & 15u));
}

struct ScrShared {
   float q[kKnnMaxDims2][kScrRows];  // the rows' fp32 coordinates
   float nqh[kScrRows];              // -|q_r|^2 / 2
   union {
      unsigned int h[kScrRows][256];
      double key[kScrRows][kScrCap];
      float ck[kScrRows][kScrCap];  // the one-pass collect's candidate accumulators
   } u;
   int idx[kScrRows][kScrCap];
   float thr[kScrRows];  // -T_r / 2 of the current scan (rows beyond nr: +inf, never pass)
   int base[kScrRows], cnt[kScrRows];
   int row[kScrRows];    // the rows' indices (a row counts only points before it)
};

// One scan of points j in [j0, j1) against the workgroup's R = 32 rows on v_mfma_f32_32x32x2_f32: each
// wave takes tiles of 32 points; the rows' coordinates are the A operand, held in registers for the whole
// scan (lane l: row l & 31, features 2s + (l >> 5)), the points' the B operand (one coalesced fp32 load per
// step), and the 32 x 32 accumulator starts at -(|x_j|^2 + |q_r|^2) / 2 (lane l: point l & 31, rows
// (v & 3) + 8 (v >> 2) + 4 (l >> 5) of its 16 values).  MODE 0: exponent histogram of every key~; 1 / 2:
// keys below the row's threshold binned 16 per octave from base; 3: append keys <= the threshold to the
// row's candidates.  CHECK: only points before the row (j < S.row[r]) count.  STEPS = ceil(d / 2) bound.
typedef float f32x16 __attribute__((ext_vector_type(16)));
// sub > 1: only every sub-th round of W tiles (a systematic 1/sub subset of [j0, j1))
template <int MODE, bool CHECK, int STEPS>
__device__ __forceinline__ void knn_scan_mfma(ScrShared& S, const float* __restrict__ Xf,
                                              const float* __restrict__ nx, int n, int d, int i0, int j0, int j1,
                                              int sub = 1)
{
   // wave w: row tile w % kScrRowBlocks (rows rt .. rt + 31), point stream w / kScrRowBlocks of W; the waves
   // of one point stream read the same points at the same time (one fetch beyond L2 serves all of them)
   constexpr int W = kScrThreads / 64 / kScrRowBlocks;
   const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
   const int rt = 32 * ((threadIdx.x >> 6) % kScrRowBlocks), wave = (threadIdx.x >> 6) / kScrRowBlocks;
   float a[STEPS];
#pragma unroll
   for (int st = 0; st < STEPS; st++) a[st] = S.q[2 * st + h][rt + col];  // zero beyond d
   float nqh[16], thr[16];
   int rlim[16];
#pragma unroll
   for (int v = 0; v < 16; v++) {
      const int r = rt + (v & 3) + 8 * (v >> 2) + 4 * h;
      nqh[v] = S.nqh[r];
      thr[v] = S.thr[r];
      rlim[v] = CHECK ? S.row[r] : 0;
   }
   // the loads run two tiles ahead of the MFMAs (software pipelining over the memory latency)
   float b0[STEPS], b1[STEPS], a00 = 0.f, a01 = 0.f;
   auto load = [&](int jb, float (&b)[STEPS], float& a0) {
      const int jl = min(jb + col, j1 - 1);  // a valid point for the lanes past the end (their keys are dropped)
      a0 = nx[jl];
#pragma unroll
      for (int st = 0; st < STEPS; st++) b[st] = Xf[(size_t)(2 * st + h) * n + jl];  // Xf zero-padded to 2 STEPS
   };
   const int step = W * 32 * sub;
   if (j0 + wave * 32 < j1) load(j0 + wave * 32, b0, a00);
   if (j0 + wave * 32 + step < j1) load(j0 + wave * 32 + step, b1, a01);
   for (int jb = j0 + wave * 32; jb < j1; jb += step) {
      const int j = jb + col;
      const bool ok = j < j1;
      f32x16 c;
      float bc[STEPS];
#pragma unroll
      for (int v = 0; v < 16; v++) c[v] = fmaf(a00, -0.5f, nqh[v]);
#pragma unroll
      for (int st = 0; st < STEPS; st++) {
         bc[st] = b0[st];
         b0[st] = b1[st];
      }
      a00 = a01;
      if (jb + 2 * step < j1) load(jb + 2 * step, b1, a01);
#pragma unroll
      for (int st = 0; st < STEPS; st++) c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[st], bc[st], c, 0, 0, 0);
      if (!ok) continue;
      if (MODE == 0) {
#pragma unroll
         for (int v = 0; v < 16; v++) {
            if (c[v] < thr[v]) continue;  // rows beyond nr (thr +inf)
            const int r = rt + (v & 3) + 8 * (v >> 2) + 4 * h;
            atomicAdd(&S.u.h[r][__float_as_uint(fmaxf(0.f, -2.f * c[v])) >> 23], 1u);
         }
         continue;
      }
      bool any = false;
#pragma unroll
      for (int v = 0; v < 16; v++) any |= (MODE == 3 ? c[v] >= thr[v] : c[v] > thr[v]);
      if (!any) continue;
#pragma unroll
      for (int v = 0; v < 16; v++) {
         const int r = rt + (v & 3) + 8 * (v >> 2) + 4 * h;
         const bool pass = MODE == 3 ? c[v] >= thr[v] : c[v] > thr[v];
         if (!pass || (CHECK && j >= rlim[v])) continue;
         if (MODE == 3) {
            const int slot = atomicAdd(&S.cnt[r], 1);
            if (slot < kScrCap) S.idx[r][slot] = j;
         } else {
            const float key = fmaxf(0.f, -2.f * c[v]);
            atomicAdd(&S.u.h[r][knn_bin32(__float_as_uint(key), S.base[r])], 1u);
         }
      }
   }
}

// The one-pass collect (PHASE 2): every point j in [j0, j1) with key~ <= the row's limit L (acc >= S.thr = -L/2)
// appends (j, acc) to the row's candidates, and at round boundaries the workgroup stops and each row holding
// more than `trigger` candidates tightens L to V + 2m, V = the (lfil-1)-th smallest key~ it holds, and drops
// the candidates above it.  Invariant: the candidates are every scanned point with key~ <= L, and L >= the
// true (lfil-1)-th smallest key + m (the lfil-1 candidates with key~ <= V have key <= V + m), so every true
// neighbour is still a candidate when the scan ends.  The boundaries fall every 16 rounds of 256 points up to
// 16384 points, then every quarter of the points seen, so the appends between two boundaries stay near
// (lfil - 1) / 4; a row that overflows kScrCap anyway goes to the fallback (cnt > kScrCap).
template <bool CHECK, int STEPS>
__device__ __forceinline__ void knn_stream_mfma(ScrShared& S, const float* __restrict__ Xf,
                                                const float* __restrict__ nx, int n, int j0, int j1, int nr, int K,
                                                float margin2)
{
   static_assert(kScrRowBlocks == 1, "the stream keeps one row tile per workgroup");
   constexpr int W = kScrThreads / 64, CAP = kScrCap;
   const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31, wave = threadIdx.x >> 6;
   const int trigger = min(CAP - 48, max(64, 2 * K));
   float a[STEPS];
#pragma unroll
   for (int st = 0; st < STEPS; st++) a[st] = S.q[2 * st + h][col];
   float nqh[16], thr[16];
   int rlim[16];
#pragma unroll
   for (int v = 0; v < 16; v++) {
      const int r = (v & 3) + 8 * (v >> 2) + 4 * h;
      nqh[v] = S.nqh[r];
      thr[v] = S.thr[r];
      rlim[v] = CHECK ? S.row[r] : 0;
   }
   float b0[STEPS], b1[STEPS], a00 = 0.f, a01 = 0.f;
   auto load = [&](int jb, float (&b)[STEPS], float& a0) {
      const int jl = min(jb + col, j1 - 1);
      a0 = nx[jl];
#pragma unroll
      for (int st = 0; st < STEPS; st++) b[st] = Xf[(size_t)(2 * st + h) * n + jl];
   };
   constexpr int step = W * 32;
   const int nrounds = (j1 - j0 + step - 1) / step;  // workgroup-uniform: every wave meets every boundary
   if (j0 + wave * 32 < j1) load(j0 + wave * 32, b0, a00);
   if (j0 + wave * 32 + step < j1) load(j0 + wave * 32 + step, b1, a01);
   int next = 16;  // the round after which the next boundary falls
   for (int k = 0; k < nrounds; k++) {
      const int jb = j0 + wave * 32 + k * step;
      if (jb < j1) {
         const int j = jb + col;
         const bool ok = j < j1;
         f32x16 c;
         float bc[STEPS];
#pragma unroll
         for (int v = 0; v < 16; v++) c[v] = fmaf(a00, -0.5f, nqh[v]);
#pragma unroll
         for (int st = 0; st < STEPS; st++) {
            bc[st] = b0[st];
            b0[st] = b1[st];
         }
         a00 = a01;
         if (jb + 2 * step < j1) load(jb + 2 * step, b1, a01);
#pragma unroll
         for (int st = 0; st < STEPS; st++) c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[st], bc[st], c, 0, 0, 0);
         bool any = false;
#pragma unroll
         for (int v = 0; v < 16; v++) any |= c[v] >= thr[v];
         if (ok && any) {
#pragma unroll
            for (int v = 0; v < 16; v++) {
               const int r = (v & 3) + 8 * (v >> 2) + 4 * h;
               if (!(c[v] >= thr[v]) || (CHECK && j >= rlim[v])) continue;
               const int slot = atomicAdd(&S.cnt[r], 1);
               if (slot < CAP) {
                  S.idx[r][slot] = j;
                  S.u.ck[r][slot] = c[v];
               }
            }
         }
      }
      if (k + 1 != next || k + 1 == nrounds) continue;
      next = (k + 1 < 64) ? k + 17 : k + 1 + (k + 1) / 4;
      __syncthreads();
      for (int r = wave; r < nr; r += W) {
         const int cnt = S.cnt[r];
         if (cnt <= trigger || cnt > CAP) continue;
         // V = the K-th smallest key~ held: the largest key~ of rank < K (rank = the number strictly below)
         float vmax = 0.f;
         for (int e = lane; e < cnt; e += 64) {
            const float ke = fmaxf(0.f, -2.f * S.u.ck[r][e]);
            int rank = 0;
            for (int o = 0; o < cnt; o++) rank += (fmaxf(0.f, -2.f * S.u.ck[r][o]) < ke) ? 1 : 0;
            if (rank < K) vmax = fmaxf(vmax, ke);
         }
         for (int off = 32; off > 0; off >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, off, 64));
         const float tnew = -0.5f * ((vmax + margin2) * 1.000001f);
         if (!(tnew > S.thr[r])) continue;  // wave-uniform
         // keep acc >= tnew, in order (the writes of a 64-chunk land at or below its reads)
         int kept = 0;
         for (int e0 = 0; e0 < cnt; e0 += 64) {
            const int e = e0 + lane;
            const float ce = e < cnt ? S.u.ck[r][e] : 0.f;
            const int je = e < cnt ? S.idx[r][e] : 0;
            const bool keep = e < cnt && ce >= tnew;
            const unsigned long long m = __ballot(keep);
            const int pos = kept + __popcll(m & ((1ull << lane) - 1ull));
            if (keep) {
               S.u.ck[r][pos] = ce;
               S.idx[r][pos] = je;
            }
            kept += __popcll(m);
         }
         if (lane == 0) {
            S.cnt[r] = kept;
            S.thr[r] = tnew;
         }
      }
      __syncthreads();
#pragma unroll
      for (int v = 0; v < 16; v++) thr[v] = S.thr[(v & 3) + 8 * (v >> 2) + 4 * h];
   }
}

// Two launches, so that each holds only its own scans' registers: PHASE 0 = sample and count, leaving each
// row's collect limit U + 2m in lim (NaN: the row goes to the fallback); PHASE 1 = collect, exact keys, rank.
// PHASE 2 = the one-launch screen: the sample, then the one-pass collect above from the sample's limit
// T1 + 2m, exact keys, rank.
template <int STEPS, int PHASE>
__global__ __launch_bounds__(kScrThreads, KNN_SCR_WAVES) void k_knn_screen(const double* __restrict__ X, int ldim,
                                                               const float* __restrict__ Xf,
                                                               const float* __restrict__ nx, int n, int d, int lfil,
                                                               float margin2, float* __restrict__ lim,
                                                               const int* __restrict__ ia,
                                                               int* __restrict__ ja, int* __restrict__ fail,
                                                               int* __restrict__ nfail, const int* __restrict__ rows,
                                                               int nrows_list, int kScrSub)
{
   constexpr int R = kScrRows, CAP = kScrCap, W = kScrThreads / 64;
   __shared__ ScrShared S;
   const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
   const int K = lfil - 1;
   // rows (ascending, all >= lfil; nrows_list of them) instead of lfil .. n-1: a row shard's own rows
   const int nall = rows ? nrows_list : n - lfil;
   const int ngroups = (nall + R - 1) / R;
   const float inf = __int_as_float(0x7f800000);
   // the first bin where the cumulative count of h[r] reaches K (one wave per row; every lane returns it),
   // -1 when the histogram holds fewer than K keys (the scans' roundings may differ; such a row goes to k_knn)
   auto kth_bin = [&](int r) {
      unsigned int loc = 0;
      for (int b = 0; b < 4; b++) loc += S.u.h[r][lane * 4 + b];
      unsigned int incl = loc;
      for (int off = 1; off < 64; off <<= 1) {
         const unsigned int o = __shfl_up(incl, off, 64);
         if (lane >= off) incl += o;
      }
      const unsigned long long hit = __ballot(incl >= (unsigned)K);
      if (!hit) return -1;
      const int first = __ffsll((long long)hit) - 1;
      int b = lane * 4;
      if (lane == first) {
         unsigned int cum = incl - loc;
         for (; b < lane * 4 + 3; b++) {
            if (cum + S.u.h[r][b] >= (unsigned)K) break;
            cum += S.u.h[r][b];
         }
      }
      return __shfl(b, first, 64);
   };
   auto give_up = [&](int r) {  // lane 0 of the row's wave
      S.thr[r] = inf;
      S.cnt[r] = CAP + 1;
   };
   // upper end of bin b of the 16-per-octave bins from base (bin 0 also holds every exponent below base)
   auto bin_top = [](int base, int b) {
      const int e = base + (b >> 4);
      return (e < 0) ? 0.f : __uint_as_float(((unsigned)e << 23) + ((unsigned)((b & 15) + 1) << 19));
   };
   auto clear_h = [&]() {
      for (int e = tid; e < R * 256; e += kScrThreads) S.u.h[e / 256][e % 256] = 0u;
   };
   for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
      const int lp0 = g * R;  // list position of the group's first row
      const int nr = min(R, nall - lp0);
      const int i0 = rows ? rows[lp0] : lfil + lp0;
      const int ilast = rows ? rows[lp0 + nr - 1] : i0 + nr - 1;
      auto row_of = [&](int r) { return rows ? rows[lp0 + r] : i0 + r; };
      for (int e = tid; e < R * 2 * STEPS; e += kScrThreads) {
         const int r = e % R, c = e / R;
         S.q[c][r] = (r < nr) ? Xf[(size_t)c * n + row_of(r)] : 0.f;
      }
      clear_h();
      if (tid < R) {
         S.row[tid] = tid < nr ? row_of(tid) : 0;
         S.nqh[tid] = (tid < nr) ? -0.5f * nx[row_of(tid)] : 0.f;
      }
      if (tid < R) {
         S.cnt[tid] = 0;
         if (PHASE != 1) {
            S.thr[tid] = (tid < nr) ? -inf : inf;
         } else {
            const float L = (tid < nr) ? lim[lp0 + tid] : inf;
            S.thr[tid] = (L != L || tid >= nr) ? inf : -0.5f * L;
            if (tid < nr && L != L) S.cnt[tid] = CAP + 1;
         }
      }
      __syncthreads();
      if constexpr (PHASE != 1) {
      const int Sn = min(i0, kScrSample);
      knn_scan_mfma<0, false, STEPS>(S, Xf, nx, n, d, i0, 0, Sn);
      __syncthreads();
      for (int r = wave; r < nr; r += W) {
         const int b = kth_bin(r);  // exponent bin: keys there are below 2^(b - 126)
         if (lane == 0 && b < 0) give_up(r);
         if (lane == 0 && b >= 0) {
            S.thr[r] = (b == 255) ? -inf : -0.5f * __uint_as_float((unsigned)(b + 1) << 23);
            S.base[r] = ((b == 255) ? 255 : b + 1) - 16;
         }
      }
      __syncthreads();
      clear_h();
      __syncthreads();
      knn_scan_mfma<1, false, STEPS>(S, Xf, nx, n, d, i0, 0, Sn);
      __syncthreads();
      for (int r = wave; r < nr; r += W) {
         const int b = kth_bin(r);
         if (lane == 0 && b < 0 && S.thr[r] != inf) give_up(r);
         if (lane == 0 && b >= 0) {
            const float T1 = (S.thr[r] == -inf) ? inf : bin_top(S.base[r], b);
            S.thr[r] = -0.5f * T1;
            S.base[r] = (T1 == inf) ? 255 - 16 : (int)(__float_as_uint(T1) >> 23) + ((__float_as_uint(T1) & 0x7fffffu) ? 1 : 0) - 16;
         }
      }
      __syncthreads();
      }
      if constexpr (PHASE == 0) {
      clear_h();
      __syncthreads();
      // count over the earlier points: [0, i0) before all rows (a systematic half of it once i0 is large: the
      // (lfil-1)-th smallest key of any subset bounds the row's from above, so U + 2m still collects every
      // neighbour, with about 2 (lfil - 1) candidates), [i0, i0 + nr - 1) before some
      knn_scan_mfma<2, false, STEPS>(S, Xf, nx, n, d, i0, 0, i0, i0 >= kScrSubFrom ? kScrSub : 1);
      knn_scan_mfma<2, true, STEPS>(S, Xf, nx, n, d, i0, i0, ilast);
      __syncthreads();
      for (int r = wave; r < nr; r += W) {
         const int b = kth_bin(r);
         if (lane == 0) {
            const bool gave_up = S.thr[r] == inf;
            lim[lp0 + r] = (gave_up || b < 0) ? __int_as_float(0x7fc00000)
                                              : (bin_top(S.base[r], b) + margin2) * 1.000001f;
         }
      }
      __syncthreads();
      } else {
      if constexpr (PHASE == 1) {
         knn_scan_mfma<3, false, STEPS>(S, Xf, nx, n, d, i0, 0, i0);
         knn_scan_mfma<3, true, STEPS>(S, Xf, nx, n, d, i0, i0, ilast);
      } else {
         // the sample's limit T1 + 2m (thr = -T1 / 2 here; inf: gave up, -inf: T1 = inf)
         if (tid < nr) {
            const float t = S.thr[tid];
            if (t != inf && t != -inf) S.thr[tid] = -0.5f * ((-2.f * t + margin2) * 1.000001f);
         }
         __syncthreads();
         knn_stream_mfma<false, STEPS>(S, Xf, nx, n, 0, i0, nr, K, margin2);
         knn_stream_mfma<true, STEPS>(S, Xf, nx, n, i0, ilast, nr, K, margin2);
      }
      __syncthreads();
      // exact keys of the candidates (the histogram space is free now)
      for (int r = wave; r < nr; r += W) {
         const int i = S.row[r], cnt = S.cnt[r];
         if (cnt > CAP || cnt < K) continue;
         for (int e = lane; e < cnt; e += 64) {
            const int j = S.idx[r][e];
            double a = 0.0;
            for (int c = 0; c < d; c++) {
               const double t = X[(size_t)c * ldim + j] - X[(size_t)c * ldim + i];
               a = fma(t, t, a);
            }
            S.u.key[r][e] = a;
         }
      }
      __syncthreads();
      for (int r = wave; r < nr; r += W) {
         const int i = S.row[r], cnt = S.cnt[r];
         if (cnt > CAP || cnt < K) {
            if (lane == 0) fail[atomicAdd(nfail, 1)] = i;
            continue;
         }
         const int row = ia[i];
         for (int e = lane; e < cnt; e += 64) {
            const double ke = S.u.key[r][e];
            const int ie = S.idx[r][e];
            int rank = 0;
            for (int o = 0; o < cnt; o++) {
               const double ko = S.u.key[r][o];
               rank += (ko < ke || (ko == ke && S.idx[r][o] < ie)) ? 1 : 0;
            }
            if (rank < K) ja[row + rank] = ie;
         }
         if (lane == 0) ja[row + K] = i;
      }
      __syncthreads();
      }
   }
}

// ---- the one-launch tiled screen (variant 4, the default for d <= 32 and lfil <= 25) ----
// 256 rows per workgroup, 32 per wave; the earlier points stream once through LDS in stages of 64, each
// stage read by all eight waves, so the HBM / L2 traffic per (point, row) pair is an eighth of the
// 32-row screens'.  key~ comes from v_mfma_f32_32x32x16_bf16 on a three-term bf16 split of the
// coordinates: x = xh + xl + ex with xh = bf16(x), xl = bf16(x - xh), |ex| <= 2^-18 |x|, and
// x.q ~ xh.qh + xh.ql + xl.qh (bf16 products are exact in fp32).  Error of key~ = |x|^2 + |q|^2 - 2 x.q
// (fp32 norms of the fp32-rounded coordinates, as the 32-row screens):
//   split       2 * 3.02 * 2^-18 |x||q|                     <= 387 * 2^-24 M^2
//   MFMA sums   2 * 3d additions of partial sums <= 2.02 M^2 <= 12.2 d * 2^-24 M^2 (one fp32 rounding each)
//   norms       2 (d + 2) * 2^-24 M^2, start value 4 * 2^-24 M^2
// so |key~ - key| <= (14.2 d + 395) 2^-24 M^2 and m = (16 d + 448) 2^-24 M^2 (M^2 = max |x_j|^2 >= 2^-60, so
// bf16 subnormal flushes stay far below it).  Each row keeps its candidates (index, acc) in LDS, at most
// kTileCap: it starts accepting every earlier point; whenever a row holds more than kTileCap - 32 after a
// 32-point tile, its wave tightens the row's limit to V + 2m (V = the (lfil-1)-th smallest key~ held) and
// drops the candidates above it (the invariant of knn_stream_mfma), so a tile can never overflow a row that
// the limit has settled; rows that overflow anyway (many equal keys) go to the fallback.  The rows are the
// wave's own, so the selections need no barrier; the exact fp64 keys and the (key, index) ranking run on
// one candidate per lane.
constexpr int kTileRows = 256;
constexpr int kTileCap = 64;
constexpr int kTileStep = 64;  // Xb's padding: n rounded up to 64 points
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct TileShared {
   int idx[kTileRows][kTileCap];
   float ck[kTileRows][kTileCap];
   float thr[kTileRows];
   int cnt[kTileRows];
   int row[kTileRows];
};

__device__ __forceinline__ unsigned int bf16_rn(float f)  // bits of the nearest bf16 (finite f)
{
   const unsigned int u = __float_as_uint(f);
   return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// Xb: per 32-point block, [chunk KCH][hi, lo][half][point 32] x 16 B (features 16 ch + 8 half + 0..7),
// zero past d and past n; nx = fp32 squared norms (+inf past n, so padded points never pass); *m2 = bits
// of max nx over the n points.  npad = n rounded up to kTileStep.
template <int KCH>
__global__ __launch_bounds__(256) void k_knn_prep_bf(const double* __restrict__ X, int ldim, int n, int npad, int d,
                                                     uint4* __restrict__ Xb, float* __restrict__ nx,
                                                     unsigned int* __restrict__ m2)
{
   constexpr int BLK = KCH * 2 * 2 * 32;
   unsigned int mx = 0u;
   for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < npad; j += gridDim.x * blockDim.x) {
      float a = 0.f;
      uint4* blk = Xb + (size_t)(j >> 5) * BLK + (j & 31);
#pragma unroll
      for (int ch = 0; ch < KCH; ch++) {
#pragma unroll
         for (int half = 0; half < 2; half++) {
            unsigned int hw[4] = {0u, 0u, 0u, 0u}, lw[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int e = 0; e < 8; e++) {
               const int c = 16 * ch + 8 * half + e;
               const double x = (j < n && c < d) ? X[(size_t)c * ldim + j] : 0.0;
               const float f = (float)x;
               a = fmaf(f, f, a);
               const unsigned int hb = bf16_rn(f);
               const unsigned int lb = bf16_rn((float)(x - (double)__uint_as_float(hb << 16)));
               hw[e >> 1] |= hb << (16 * (e & 1));
               lw[e >> 1] |= lb << (16 * (e & 1));
            }
            blk[((ch * 2 + 0) * 2 + half) * 32] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
            blk[((ch * 2 + 1) * 2 + half) * 32] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
         }
      }
      nx[j] = j < n ? a : __int_as_float(0x7f800000);
      if (j < n) mx = max(mx, __float_as_uint(a));
   }
   for (int off = 32; off > 0; off >>= 1) mx = max(mx, (unsigned int)__shfl_xor((int)mx, off, 64));
   if ((threadIdx.x & 63) == 0) atomicMax(m2, mx);
}

// Every wave loads its B fragments from global memory itself (the eight waves read the same lines close
// together: L1 / L2 hits), two tiles ahead in registers -- no LDS stages and no barriers in the scan (an
// LDS-staged scan with a barrier per 64 points, loads four stages ahead, measured 0.221 s against 0.174 s at
// n = 1e6, d = 32, and was removed)
template <int KCH>
__global__ __launch_bounds__(512, 2) void k_knn_tile(const double* __restrict__ X, int ldim,
                                                     const uint4* __restrict__ Xb, const float* __restrict__ nx,
                                                     int n, int d, int lfil, float margin2,
                                                     const int* __restrict__ ia, int* __restrict__ ja,
                                                     int* __restrict__ fail, int* __restrict__ nfail,
                                                     const int* __restrict__ rows, int nrows_list, int probe)
{
   constexpr int R = kTileRows, CAP = kTileCap, BLK = KCH * 2 * 2 * 32;
   __shared__ TileShared S;
   const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, col = lane & 31;
   const int K = lfil - 1;
   const int nall = rows ? nrows_list : n - lfil;
   const int ngroups = (nall + R - 1) / R;
   const float inf = __int_as_float(0x7f800000);
   for (int gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {
      const int g = ngroups - 1 - gi;  // the longest scans first
      const int lp0 = g * R, nr = min(R, nall - lp0);
      auto row_of = [&](int r) { return rows ? rows[lp0 + r] : lfil + lp0 + r; };
      const int ilast = row_of(nr - 1);  // the rows see points [0, ilast) at most
      if (tid < R) {
         S.row[tid] = tid < nr ? row_of(tid) : 0;
         S.cnt[tid] = 0;
         S.thr[tid] = (tid < nr && !probe) ? -__FLT_MAX__ : inf;  // probe: the scan alone (timing)
      }
      // the wave's 32 rows as the A operand (lane: row 32 wave + col, features 8 h + 0..7 of each chunk)
      const int iA = (32 * wave + col < nr) ? row_of(32 * wave + col) : row_of(0);
      bf16x8 ah[KCH], al[KCH];
      {
         const uint4* blk = Xb + (size_t)(iA >> 5) * BLK + (iA & 31);
#pragma unroll
         for (int ch = 0; ch < KCH; ch++) {
            const uint4 hv = blk[((ch * 2 + 0) * 2 + h) * 32], lv = blk[((ch * 2 + 1) * 2 + h) * 32];
            ah[ch] = __builtin_bit_cast(bf16x8, hv);
            al[ch] = __builtin_bit_cast(bf16x8, lv);
         }
      }
      float nqh[16], thr[16];
      int rlim[16];
#pragma unroll
      for (int v = 0; v < 16; v++) {
         const int r = 32 * wave + (v & 3) + 8 * (v >> 2) + 4 * h;
         nqh[v] = r < nr ? -0.5f * nx[row_of(r)] : 0.f;
         rlim[v] = r < nr ? row_of(r) : 0;
      }
      const int rowmin = row_of(0);
      const unsigned long long below = (1ull << lane) - 1ull;
      int cntv = 0;  // lane l < 32: candidates of the wave's row l
      __syncthreads();
#pragma unroll
      for (int v = 0; v < 16; v++) thr[v] = S.thr[32 * wave + (v & 3) + 8 * (v >> 2) + 4 * h];
      // test a tile's keys against the rows' limits (points j0 + col), append, tighten
      auto test_tile = [&](const f32x16& c, int j0) {
         const int j = j0 + col;
         // per group of 4 rows of the lane (v = 4 g .. 4 g + 3) the largest margin; NaN keys drop out
         float mg[4];
#pragma unroll
         for (int g = 0; g < 4; g++)
            mg[g] = fmaxf(fmaxf(c[4 * g] - thr[4 * g], c[4 * g + 1] - thr[4 * g + 1]),
                          fmaxf(c[4 * g + 2] - thr[4 * g + 2], c[4 * g + 3] - thr[4 * g + 3]));
         const float mx = fmaxf(fmaxf(mg[0], mg[1]), fmaxf(mg[2], mg[3]));
         if (!__ballot(mx >= 0.f)) return;
         // append: the wave owns its rows, so each (v, lane half) pair's slots come from one ballot
         // (lanes 0-31: row rl = (v & 3) + 8 (v >> 2), lanes 32-63: rl + 4) and the counts live in cntv
         // a point at or after a row never counts for it (rlim: the lane's 16 rows' indices; jj = -1 while
         // every point of the tile precedes every row)
         const int jj = (j0 + 31 < rowmin) ? -1 : j;
#pragma unroll
         for (int g = 0; g < 4; g++) {
            if (!__ballot(mg[g] >= 0.f)) continue;  // no lane passes in this group of 4 rows
#pragma unroll
            for (int vv = 0; vv < 4; vv++) {
               const int v = 4 * g + vv;
               const int rl = (v & 3) + 8 * (v >> 2);
               const bool pass = c[v] >= thr[v] && jj < rlim[v];
               const unsigned long long m = __ballot(pass);
               if (!m) continue;
               const unsigned int mlo = (unsigned int)m, mhi = (unsigned int)(m >> 32);
               const int blo = __builtin_amdgcn_readlane(cntv, rl), bhi = __builtin_amdgcn_readlane(cntv, rl + 4);
               if (pass) {
                  const int base = h ? bhi : blo;
                  const int pos = base + __popcll(m & below) - (h ? __popc(mlo) : 0);
                  if (pos < CAP) {
                     S.idx[32 * wave + rl + 4 * h][pos] = j;
                     S.ck[32 * wave + rl + 4 * h][pos] = c[v];
                  }
               }
               cntv += (lane == rl) ? __popc(mlo) : (lane == rl + 4) ? __popc(mhi) : 0;
            }
         }
         // the wave's rows that another tile could overflow: tighten them (wave-uniform loop)
         unsigned long long todo = __ballot(lane < 32 && cntv > CAP - 32);
         if (!todo) return;
         while (todo) {
            const int rl = __ffsll((long long)todo) - 1;
            todo &= todo - 1;
            const int r = 32 * wave + rl;
            const int cnt = __builtin_amdgcn_readlane(cntv, rl);
            if (cnt > CAP) {  // overflowed: the fallback takes the row
               if (lane == 0) S.thr[r] = inf;
               continue;
            }
            const float ce = lane < cnt ? S.ck[r][lane] : -inf;
            const int je = lane < cnt ? S.idx[r][lane] : 0;
            const float ke = lane < cnt ? fmaxf(0.f, -2.f * ce) : inf;
            int rank = 0;
            for (int o = 0; o < cnt; o++)
               rank += (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(ke), o)) < ke) ? 1 : 0;
            float vk = (lane < cnt && rank < K) ? ke : 0.f;
            for (int off = 32; off > 0; off >>= 1) vk = fmaxf(vk, __shfl_xor(vk, off, 64));
            const float tnew = -0.5f * ((vk + margin2) * 1.000001f);
            if (!(tnew > S.thr[r])) continue;
            const bool keep = lane < cnt && ce >= tnew;
            const unsigned long long m = __ballot(keep);
            if (keep) {
               const int pos = __popcll(m & ((1ull << lane) - 1ull));
               S.ck[r][pos] = ce;
               S.idx[r][pos] = je;
            }
            if (lane == rl) cntv = __popcll(m);
            if (lane == 0) S.thr[r] = tnew;
         }
#pragma unroll
         for (int v = 0; v < 16; v++) thr[v] = S.thr[32 * wave + (v & 3) + 8 * (v >> 2) + 4 * h];
      };
      // software pipeline: a tile's tests run under the next tile's MFMAs (c1 carries the previous tile)
      f32x16 c0, c1;
      {
         const int ntl = (ilast + 31) / 32;  // 32-point tiles
         uint4 bh0[KCH], bl0[KCH], bh1[KCH], bl1[KCH];
         float nx0, nx1;
         auto fetchf = [&](int t, uint4 (&fh)[KCH], uint4 (&fl)[KCH], float& fn) {
            t = min(t, ntl - 1);
            const uint4* blk = Xb + (size_t)t * BLK + col;
#pragma unroll
            for (int ch = 0; ch < KCH; ch++) {
               fh[ch] = blk[((ch * 2 + 0) * 2 + h) * 32];
               fl[ch] = blk[((ch * 2 + 1) * 2 + h) * 32];
            }
            fn = nx[(size_t)t * 32 + col];
         };
         auto mfma_frag = [&](const uint4 (&fh)[KCH], const uint4 (&fl)[KCH], float fn) {
            f32x16 c;
#pragma unroll
            for (int v = 0; v < 16; v++) c[v] = fmaf(fn, -0.5f, nqh[v]);
#pragma unroll
            for (int ch = 0; ch < KCH; ch++) {
               const bf16x8 bh = __builtin_bit_cast(bf16x8, fh[ch]), bl = __builtin_bit_cast(bf16x8, fl[ch]);
               c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[ch], bl, c, 0, 0, 0);
               c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[ch], bh, c, 0, 0, 0);
               c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[ch], bh, c, 0, 0, 0);
            }
            return c;
         };
         fetchf(0, bh0, bl0, nx0);
         fetchf(1, bh1, bl1, nx1);
         for (int t0 = 0; t0 < ntl; t0 += 2) {
            c0 = mfma_frag(bh0, bl0, nx0);
            fetchf(t0 + 2, bh0, bl0, nx0);
            if (t0 > 0) test_tile(c1, t0 * 32 - 32);
            if (t0 + 1 < ntl) {
               c1 = mfma_frag(bh1, bl1, nx1);
               fetchf(t0 + 3, bh1, bl1, nx1);
            }
            test_tile(c0, t0 * 32);
         }
         if (ntl % 2 == 0) test_tile(c1, (ntl - 1) * 32);
      }
      if (lane < 32) S.cnt[32 * wave + lane] = cntv;
      // exact fp64 keys of the candidates (one per lane) and the (key, index) ranking; the wave's rows
      for (int rl = 0; rl < 32; rl++) {
         const int r = 32 * wave + rl;
         if (r >= nr) break;
         const int i = S.row[r], cnt = S.cnt[r];
         if (cnt > CAP || cnt < K) {
            if (lane == 0) fail[atomicAdd(nfail, 1)] = i;
            continue;
         }
         double ke = 0.0;
         int ie = 0x7fffffff;
         if (lane < cnt) {
            ie = S.idx[r][lane];
            for (int c = 0; c < d; c++) {
               const double t = X[(size_t)c * ldim + ie] - X[(size_t)c * ldim + i];
               ke = fma(t, t, ke);
            }
         }
         int rank = 0;
         for (int o = 0; o < cnt; o++) {
            const double ko = __shfl(ke, o, 64);
            const int io = __builtin_amdgcn_readlane(ie, o);
            rank += (ko < ke || (ko == ke && io < ie)) ? 1 : 0;
         }
         const int rp = ia[i];
         if (lane < cnt && rank < K) ja[rp + rank] = ie;
         if (lane == 0) ja[rp + K] = i;
      }
      __syncthreads();
   }
}

template <class T>
int upload(T** d, const T* h, size_t count);

// KNN pattern rows [lfil, n) into dja (CSR row pointers dia): variant 4 (default) the tiled one-launch screen
// (k_knn_tile; d <= 32 and lfil <= 25, else variant 3), 3 the one-launch 32-row screen (k_knn_screen PHASE 2),
// 1 the two-launch count + collect screens,
// 0 the fp64 k_knn_bounded, 2 the radix-select k_knn for every row; the rows the bounded variants leave go
// to k_knn.  Returns the number of such rows, or -1.
int knn_pattern(const double* dX, int n, int ldim, int d, int lfil, const int* dia, int* dja, hipStream_t s,
                int variant, const int* d_rows = nullptr, int nrows_list = 0)
{
   if (n <= lfil || (d_rows && nrows_list <= 0)) return 0;
   if (variant < 0) {
      const char* e = getenv("NFFT4GP_AMD_KNN");
      variant = e ? atoi(e) : 4;
   }
   if (d > kKnnMaxDims2) variant = 2;
   const int nrows = d_rows ? nrows_list : n - lfil;
   if (variant == 2) {
      hipLaunchKernelGGL(k_knn, dim3(std::min(nrows, 4096)), dim3(kKnnThreads), 0, s, dX, ldim, n, d, lfil, dia, dja,
                         d_rows, d_rows ? nrows : 0);
      return hipGetLastError() == hipSuccess ? nrows : -1;
   }
   int* dfail = nullptr;
   float *Xf = nullptr, *nx = nullptr;
   int nfail = -1;
   unsigned int m2bits = 0u;
   auto done = [&](int rc) {
      (void)hipStreamSynchronize(s);
      (void)hipFree(dfail);
      (void)hipFree(Xf);
      (void)hipFree(nx);
      return rc;
   };
   if (upload(&dfail, (const int*)nullptr, (size_t)nrows + 2) ||
       hipMemsetAsync(dfail + nrows, 0, 2 * sizeof(int), s) != hipSuccess)
      return done(-1);
   if (variant == 4 && (d > 32 || lfil - 1 > 24)) variant = 3;
   if (variant == 4) {
      const int kch = d <= 16 ? 1 : 2;
      const int npad = (n + kTileStep - 1) / kTileStep * kTileStep;
      if (hipMalloc((void**)&Xf, (size_t)npad * kch * 64) != hipSuccess ||
          hipMalloc((void**)&nx, sizeof(float) * (size_t)npad) != hipSuccess)
         return done(-1);
      if (kch == 1)
         hipLaunchKernelGGL(k_knn_prep_bf<1>, dim3(std::min((npad + 255) / 256, 4096)), dim3(256), 0, s, dX, ldim, n,
                            npad, d, (uint4*)Xf, nx, (unsigned int*)(dfail + nrows + 1));
      else
         hipLaunchKernelGGL(k_knn_prep_bf<2>, dim3(std::min((npad + 255) / 256, 4096)), dim3(256), 0, s, dX, ldim, n,
                            npad, d, (uint4*)Xf, nx, (unsigned int*)(dfail + nrows + 1));
      if (hipMemcpyAsync(&m2bits, dfail + nrows + 1, sizeof(unsigned int), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
         return done(-1);
      float m2;
      memcpy(&m2, &m2bits, sizeof(float));
      const double margin = (16.0 * d + 448.0) * std::ldexp(1.0, -24) * (double)m2;
      if (std::isfinite(m2) && m2 >= std::ldexp(1.0f, -60) && std::isfinite((float)(2.0 * margin))) {
         const int ngroups = (nrows + kTileRows - 1) / kTileRows;
         auto tile = kch == 1 ? k_knn_tile<1> : k_knn_tile<2>;
         hipLaunchKernelGGL(tile, dim3(std::min(ngroups, 65535)), dim3(kScrThreads), 0, s, dX, ldim, (const uint4*)Xf,
                            (const float*)nx, n, d, lfil, (float)(2.0 * margin) * 1.0001f, dia, dja, dfail,
                            dfail + nrows, d_rows, nrows, getenv("NFFT4GP_AMD_KNN_TILE_PROBE") ? 1 : 0);
      } else {
         variant = 3;  // the fp32 screens decide (and route non-finite data to k_knn)
         (void)hipFree(Xf);
         (void)hipFree(nx);
         Xf = nx = nullptr;
         if (hipMemsetAsync(dfail + nrows, 0, 2 * sizeof(int), s) != hipSuccess) return done(-1);
      }
   }
   if (variant == 1 || variant == 3) {
      const int steps = d <= 4 ? 2 : d <= 8 ? 4 : d <= 16 ? 8 : d <= 32 ? 16 : 32;
      if (hipMalloc((void**)&Xf, sizeof(float) * (size_t)n * 2 * steps) != hipSuccess ||
          hipMalloc((void**)&nx, sizeof(float) * (size_t)n) != hipSuccess)
         return done(-1);
      hipLaunchKernelGGL(k_knn_prep, dim3(std::min((n + 255) / 256, 4096)), dim3(256), 0, s, dX, ldim, n, d, 2 * steps, Xf, nx,
                         (unsigned int*)(dfail + nrows + 1));
      if (hipMemcpyAsync(&m2bits, dfail + nrows + 1, sizeof(unsigned int), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
         return done(-1);
      float m2;
      memcpy(&m2, &m2bits, sizeof(float));
      const double margin = (8.0 * d + 64.0) * std::ldexp(1.0, -24) * (double)m2;
      if (!std::isfinite(m2) || !std::isfinite((float)(2.0 * margin))) {
         variant = 2;  // every row to k_knn
      } else {
         const int ngroups = (nrows + kScrRows - 1) / kScrRows;
         static const int sub = getenv("NFFT4GP_AMD_KNN_SUB") ? std::max(1, atoi(getenv("NFFT4GP_AMD_KNN_SUB"))) : 2;
         float* lim = nullptr;
         if (hipMalloc((void**)&lim, sizeof(float) * (size_t)nrows) != hipSuccess) return done(-1);
         if (variant == 3) {
            auto screen = steps == 2    ? k_knn_screen<2, 2>
                          : steps == 4  ? k_knn_screen<4, 2>
                          : steps == 8  ? k_knn_screen<8, 2>
                          : steps == 16 ? k_knn_screen<16, 2>
                                        : k_knn_screen<32, 2>;
            hipLaunchKernelGGL(screen, dim3(std::min(ngroups, 4096)), dim3(kScrThreads), 0, s, dX, ldim,
                               (const float*)Xf, (const float*)nx, n, d, lfil, (float)(2.0 * margin) * 1.0001f, lim,
                               dia, dja, dfail, dfail + nrows, d_rows, nrows, sub);
         }
         for (int phase = 0; phase < (variant == 3 ? 0 : 2); phase++) {
            auto screen = phase == 0 ? (steps == 2    ? k_knn_screen<2, 0>
                                        : steps == 4  ? k_knn_screen<4, 0>
                                        : steps == 8  ? k_knn_screen<8, 0>
                                        : steps == 16 ? k_knn_screen<16, 0>
                                                      : k_knn_screen<32, 0>)
                                     : (steps == 2    ? k_knn_screen<2, 1>
                                        : steps == 4  ? k_knn_screen<4, 1>
                                        : steps == 8  ? k_knn_screen<8, 1>
                                        : steps == 16 ? k_knn_screen<16, 1>
                                                      : k_knn_screen<32, 1>);
            hipLaunchKernelGGL(screen, dim3(std::min(ngroups, 4096)), dim3(kScrThreads), 0, s, dX, ldim,
                               (const float*)Xf, (const float*)nx, n, d, lfil, (float)(2.0 * margin) * 1.0001f, lim,
                               dia, dja, dfail, dfail + nrows, d_rows, nrows, sub);
         }
         (void)hipStreamSynchronize(s);
         (void)hipFree(lim);
      }
   } else if (variant == 0) {
      const int ngroups = (nrows + kKnnRows - 1) / kKnnRows;
      // 2 points per thread: 5.6 -> 4.0 s for the n = 1e6, d = 32, lfil = 20 setup; 4 drop to 1 wave per SIMD
      hipLaunchKernelGGL(k_knn_bounded<kKnnPoints>, dim3(std::min(ngroups, 8192)), dim3(kKnnThreads), 0, s, dX, ldim,
                         n, d, lfil, dia, dja, dfail, dfail + nrows, d_rows, d_rows ? nrows : 0);
   }
   if (variant == 2) {
      hipLaunchKernelGGL(k_knn, dim3(std::min(nrows, 4096)), dim3(kKnnThreads), 0, s, dX, ldim, n, d, lfil, dia, dja,
                         d_rows, d_rows ? nrows : 0);
      return done(hipGetLastError() == hipSuccess ? nrows : -1);
   }
   if (hipGetLastError() != hipSuccess ||
       hipMemcpyAsync(&nfail, dfail + nrows, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
       hipStreamSynchronize(s) != hipSuccess)
      return done(-1);
   if ((variant == 1 || variant == 3 || variant == 4) && nfail > 64) {
      // many rows the fp32 screen could not settle (clustered data far from the origin against its spread):
      // the fp64 two-pass scan on them, in ascending order, before the radix select on what it leaves
      std::vector<int> hrows(nfail);
      if (hipMemcpy(hrows.data(), dfail, sizeof(int) * nfail, hipMemcpyDeviceToHost) != hipSuccess) return done(-1);
      std::sort(hrows.begin(), hrows.end());
      int* drows = nullptr;
      if (upload(&drows, hrows.data(), hrows.size()) ||
          hipMemsetAsync(dfail + nrows, 0, sizeof(int), s) != hipSuccess) {
         (void)hipFree(drows);
         return done(-1);
      }
      const int ngroups = (nfail + kKnnRows - 1) / kKnnRows;
      hipLaunchKernelGGL(k_knn_bounded<kKnnPoints>, dim3(std::min(ngroups, 8192)), dim3(kKnnThreads), 0, s, dX, ldim,
                         n, d, lfil, dia, dja, dfail, dfail + nrows, (const int*)drows, nfail);
      const int nscreen = nfail;
      if (hipGetLastError() != hipSuccess ||
          hipMemcpyAsync(&nfail, dfail + nrows, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess) {
         (void)hipFree(drows);
         return done(-1);
      }
      (void)hipFree(drows);
      if (nfail > 0)
         hipLaunchKernelGGL(k_knn, dim3(std::min(nfail, 4096)), dim3(kKnnThreads), 0, s, dX, ldim, n, d, lfil, dia,
                            dja, dfail, nfail);
      return done(hipGetLastError() == hipSuccess ? nscreen : -1);
   }
   if (nfail > 0)
      hipLaunchKernelGGL(k_knn, dim3(std::min(nfail, 4096)), dim3(kKnnThreads), 0, s, dX, ldim, n, d, lfil, dia, dja,
                         dfail, nfail);
   return done(hipGetLastError() == hipSuccess ? nfail : -1);
}

// In place on the wave's LDS vector b: b = L^{-1} b (trans = 0) or L^{-T} b (trans = 1), L lower in A.
template <int LD>
__device__ void wave_trsv(double (*A)[LD], int k, double* b, int trans)
{
   const int lane = threadIdx.x;
   if (!trans) {
      for (int m = 0; m < k; m++) {
         if (lane == 0) b[m] /= A[m][m];
         __syncthreads();
         if (lane > m && lane < k) b[lane] -= A[lane][m] * b[m];
         __syncthreads();
      }
   } else {
      for (int m = k - 1; m >= 0; m--) {
         if (lane == 0) b[m] /= A[m][m];
         __syncthreads();
         if (lane < m) b[lane] -= A[m][lane] * b[m];
         __syncthreads();
      }
   }
}

// one wave per row i: A_ai (and dA_ai for the three gradients) into aa / da (fsai.c:353-398, :493-563)
//
// W (kw x n column-major, optional): the Schur-complement kernel K(x_r, x_c) - W(:, r)' W(:, c) of the AFN
// setup (Nfft4GPKernelSchurCombineKernel, kernels.c:3599-3760, with W = L11^{-1} K12), staged through LDS
// kSchurChunk rows of W at a time so each row reads its lfil columns of W once.
// Gradients of the Schur kernel (MATLAB schurCombinedKernelMat.m): with B_g = L11^{-1} dK12_g (GB, g = f, l;
// zero for mu) and C_g = (L11^{-1} dK11_g L11^{-T}) W (GC, g = f, l, mu), both kw x n per g,
//   dS_g(r, c) = dK_g(r, c) - W_r' B_g,c - B_g,r' W_c + W_r' C_g,c,
// so (dS_g a)_r = (dK_g a)_r - W_r' (B_g a - C_g a) - B_g,r' (W a) with the kw-vectors W a = sum_c W_c a_c etc.
// KM: the LDS arrays' row capacity (>= lfil); KM = 32 takes 17 KB per workgroup (9 per CU) where 64
// takes 51 KB (3 per CU).
constexpr int kSchurChunk = 32;
// KM = 20 (the reference's default lfil) takes 8.8 KB, so 18 row-waves share a CU instead of 9 at KM = 32: the
// Schur rows are bound by the latency of their W-chunk loads, and twice the rows in flight hide twice as much
template <int KM>
__global__ __launch_bounds__(64) void k_fsai_rows(const double* __restrict__ X, long long ldim,
                                                  const int* __restrict__ ia, const int* __restrict__ ja,
                                                  KernelParams P, const double* __restrict__ W, int kw, int grad,
                                                  int nnz, double* __restrict__ aa, double* __restrict__ da,
                                                  const double* __restrict__ GB, const double* __restrict__ GC,
                                                  const int* __restrict__ wcol)
{
   __shared__ double A[KM][KM + 1];
   __shared__ double Ws[KM][kSchurChunk + 1];
   __shared__ double a[KM], u[KM];
   __shared__ int idx[KM], widx[KM];
   const int i = blockIdx.x;
   const int lane = threadIdx.x;
   const int j1 = ia[i];
   const int k = ia[i + 1] - j1;
   if (lane < k) {
      idx[lane] = ja[j1 + lane];
      // W's column of the entry: the point itself, or (a row shard's chunk of W) its position in the chunk
      widx[lane] = wcol ? wcol[j1 + lane] : idx[lane];
   }
   __syncthreads();
   // K_a (lower triangle is all the factorisation reads)
   for (int e = lane; e < k * k; e += 64) {
      const int r = e % k, c = e / k;
      if (c > r) continue;
      double K, dK[3];
      kern_pair(P, X, ldim, idx[r], idx[c], r == c, K, dK);
      A[r][c] = K;
   }
   __syncthreads();
   if (W) {
      // the next chunk's W entries are loaded into registers while this chunk's products run
      constexpr int kPerLane = (KM * kSchurChunk + 63) / 64;
      double wr[kPerLane];
      auto fetch_chunk = [&](int t0) {
         const int tc = min(kSchurChunk, kw - t0);
#pragma unroll
         for (int q = 0; q < kPerLane; q++) {
            const int e = lane + 64 * q;
            wr[q] = e < k * tc ? W[(size_t)widx[e / tc] * kw + t0 + e % tc] : 0.0;
         }
      };
      fetch_chunk(0);
      for (int t0 = 0; t0 < kw; t0 += kSchurChunk) {
         const int tc = min(kSchurChunk, kw - t0);
#pragma unroll
         for (int q = 0; q < kPerLane; q++) {
            const int e = lane + 64 * q;
            if (e < k * tc) Ws[e / tc][e % tc] = wr[q];
         }
         __syncthreads();
         if (t0 + kSchurChunk < kw) fetch_chunk(t0 + kSchurChunk);
         for (int e = lane; e < k * k; e += 64) {
            const int r = e % k, c = e / k;
            if (c > r) continue;
            double acc = 0.0;
            for (int tt = 0; tt < tc; tt++) acc = fma(Ws[r][tt], Ws[c][tt], acc);
            A[r][c] -= acc;
         }
         __syncthreads();
      }
   }
   // Cholesky, lower (dpotrf 'L')
   for (int j = 0; j < k; j++) {
      if (lane == 0) A[j][j] = sqrt(A[j][j]);
      __syncthreads();
      if (lane > j && lane < k) A[lane][j] /= A[j][j];
      __syncthreads();
      if (lane > j && lane < k) {
         const double arj = A[lane][j];
         for (int c = j + 1; c <= lane; c++) A[lane][c] -= arj * A[c][j];
      }
      __syncthreads();
   }
   // A_ai = K_a^{-1} e_k, scaled by 1/sqrt(its last entry)
   if (lane < k) a[lane] = (lane == k - 1) ? 1.0 : 0.0;
   __syncthreads();
   wave_trsv(A, k, a, 0);
   wave_trsv(A, k, a, 1);
   const double dd_scale = 1.0 / sqrt(a[k - 1]);
   __syncthreads();
   if (lane < k) {
      a[lane] *= dd_scale;
      aa[j1 + lane] = a[lane];
   }
   __syncthreads();
   if (!grad) return;
   for (int g = 0; g < 3; g++) {
      // u = -dK_g A_ai (dK_g recomputed from the coordinates: K_a's storage now holds its factor)
      if (lane < k) {
         double acc = 0.0;
         for (int c = 0; c < k; c++) {
            double K, dK[3];
            kern_pair(P, X, ldim, idx[lane], idx[c], lane == c, K, dK);
            acc = fma(dK[g], a[c], acc);
         }
         u[lane] = -acc;
      }
      __syncthreads();
      if (W && GC) {
         // the Schur terms, kSchurChunk entries of the kw-vectors at a time: Ws holds (W a, B_g a - C_g a)
         const double* Bg = g < 2 ? GB + (size_t)g * kw * ((size_t)gridDim.x) : nullptr;
         const double* Cg = GC + (size_t)g * kw * ((size_t)gridDim.x);
         double acc = 0.0;
         for (int t0 = 0; t0 < kw; t0 += kSchurChunk) {
            const int tc = min(kSchurChunk, kw - t0);
            if (lane < tc) {
               double wa = 0.0, ba = 0.0, ca = 0.0;
               for (int c = 0; c < k; c++) {
                  const size_t o = (size_t)widx[c] * kw + t0 + lane;
                  wa = fma(W[o], a[c], wa);
                  if (Bg) ba = fma(Bg[o], a[c], ba);
                  ca = fma(Cg[o], a[c], ca);
               }
               Ws[0][lane] = wa;
               Ws[1][lane] = ba - ca;
            }
            __syncthreads();
            if (lane < k) {
               const size_t o = (size_t)widx[lane] * kw + t0;
               for (int tt = 0; tt < tc; tt++) {
                  acc = fma(W[o + tt], Ws[1][tt], acc);
                  if (Bg) acc = fma(Bg[o + tt], Ws[0][tt], acc);
               }
            }
            __syncthreads();
         }
         if (lane < k) u[lane] += acc;  // u = -(dS_g a)
         __syncthreads();
      }
      wave_trsv(A, k, u, 0);
      wave_trsv(A, k, u, 1);
      const double t = -0.5 * u[k - 1] * dd_scale;
      __syncthreads();
      if (lane < k) da[(size_t)g * nnz + j1 + lane] = fma(t, a[lane], u[lane]);
      __syncthreads();
   }
}

// the row kernel with the smallest LDS rows for the pattern (NFFT4GP_AMD_FSAI_KM=32 forces the 32-row one, A/B)
typedef void (*FsaiRowsFn)(const double*, long long, const int*, const int*, KernelParams, const double*, int, int,
                           int, double*, double*, const double*, const double*, const int*);
static FsaiRowsFn fsai_rows_kernel(int lfil)
{
   static const int force = getenv("NFFT4GP_AMD_FSAI_KM") ? atoi(getenv("NFFT4GP_AMD_FSAI_KM")) : 0;
   if (lfil <= 20 && force != 32) return k_fsai_rows<20>;
   if (lfil <= 32) return k_fsai_rows<32>;
   return k_fsai_rows<kFsaiMaxK>;
}

// ---- level-scheduled CSR triangular solves: one workgroup, a barrier between levels ----------------
// x = L^{-1} rhs (fsai.c:675-699): x[i] = (rhs[i] - sum_{j < diag} L_ij x_j) / L_ii in the row's order
__global__ __launch_bounds__(kTrsvThreads) void k_trsv_lower(const int* __restrict__ lev_ptr, int nlev,
                                                             const int* __restrict__ lev_rows,
                                                             const int* __restrict__ ia, const int* __restrict__ ja,
                                                             const double* __restrict__ aa,
                                                             const double* __restrict__ rhs, double* x)
{
#pragma clang fp contract(off)  // the reference's host build: separate multiply and subtract
   for (int lv = 0; lv < nlev; lv++) {
      for (int e = lev_ptr[lv] + threadIdx.x; e < lev_ptr[lv + 1]; e += kTrsvThreads) {
         const int i = lev_rows[e];
         const int j2 = ia[i + 1] - 1;
         double s = rhs[i];
         for (int j = ia[i]; j < j2; j++) s -= aa[j] * x[ja[j]];
         x[i] = s / aa[j2];
      }
      __syncthreads();
   }
}

// x = L^{-T} rhs (fsai.c:701-728) through L^T stored as CSR (tia/tja/taa: column c of L, rows ascending,
// diagonal first): the reference subtracts L_ic x_i from x[c] for i descending, then divides by L_cc
__global__ __launch_bounds__(kTrsvThreads) void k_trsv_upper(const int* __restrict__ lev_ptr, int nlev,
                                                             const int* __restrict__ lev_rows,
                                                             const int* __restrict__ tia,
                                                             const int* __restrict__ tja,
                                                             const double* __restrict__ taa,
                                                             const double* __restrict__ rhs, double* x)
{
#pragma clang fp contract(off)
   for (int lv = 0; lv < nlev; lv++) {
      for (int e = lev_ptr[lv] + threadIdx.x; e < lev_ptr[lv + 1]; e += kTrsvThreads) {
         const int c = lev_rows[e];
         const int p0 = tia[c];
         double s = rhs[c];
         for (int p = tia[c + 1] - 1; p > p0; p--) s -= taa[p] * x[tja[p]];
         x[c] = s / taa[p0];
      }
      __syncthreads();
   }
}

// y = beta y + A x for a CSR A (matops.c:139-272 with alpha = 1, beta in {0, 1}): the row accumulates
// into y[i] itself (matops.c:247), in row order, unfused
__global__ __launch_bounds__(256) void k_csr_mv(const int* __restrict__ ia, const int* __restrict__ ja,
                                                const double* __restrict__ a, const double* __restrict__ x,
                                                double* __restrict__ y, int n, int beta_one)
{
   const int r0 = blockIdx.x * 256;
   csr_rows_staged<256, 2048>(ia, ja, a, x, y, r0, min(r0 + 256, n), beta_one != 0);  // csr.hpp: entries via LDS
}

// out[blk] = sum over the block's rows of num[diag_i] / den[diag_i] (or log(1 / den[diag_i]) when num is
// NULL), diag_i = ia[i+1] - 1; the host sums the blocks in order
__global__ __launch_bounds__(256) void k_diag_sum(const int* __restrict__ ia, int n, const double* __restrict__ num,
                                                  const double* __restrict__ den, double* __restrict__ out)
{
   __shared__ double s[4];
   const int i = blockIdx.x * 256 + threadIdx.x;
   double v = 0.0;
   if (i < n) {
      const int p = ia[i + 1] - 1;
      v = num ? num[p] / den[p] : log(1.0 / den[p]);
   }
   for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
   if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
   __syncthreads();
   if (threadIdx.x == 0) out[blockIdx.x] = (s[0] + s[1]) + (s[2] + s[3]);
}

__global__ void k_gather_vals(const double* __restrict__ src, const int* __restrict__ map, int count,
                              double* __restrict__ dst)
{
   const int p = blockIdx.x * blockDim.x + threadIdx.x;
   if (p < count) dst[p] = src[map[p]];
}

// the reference's precond_fsai, restated, with the device factors
struct PrecondFsaiAmd {
   int lfil = 50;  // fsai.c:12
   int kernel = 0;
   int n = 0, nnz = 0;
   bool grad = false;
   int *ia = nullptr, *ja = nullptr, *tia = nullptr, *tja = nullptr, *tmap = nullptr;
   double *aa = nullptr, *taa = nullptr, *da = nullptr, *tda = nullptr;  // da, tda: 3 nnz
   int *lev_ptr = nullptr, *lev_rows = nullptr, *rlev_ptr = nullptr, *rlev_rows = nullptr;
   int nlev = 0, nrlev = 0;
   double *work = nullptr, *part = nullptr;
   void release()
   {
      (void)hipStreamSynchronize(current_stream());
      for (int* p : {ia, ja, tia, tja, tmap, lev_ptr, lev_rows, rlev_ptr, rlev_rows}) (void)hipFree(p);
      for (double* p : {aa, taa, da, tda, work, part}) (void)hipFree(p);
      ia = ja = tia = tja = tmap = lev_ptr = lev_rows = rlev_ptr = rlev_rows = nullptr;
      aa = taa = da = tda = work = part = nullptr;
      n = nnz = nlev = nrlev = 0;
      grad = false;
   }
};

template <class T>
int upload(T** d, const T* h, size_t count)
{
   NFFT4GP_HIP_CHECK(hipMalloc((void**)d, sizeof(T) * std::max<size_t>(1, count)));
   if (count && h) NFFT4GP_HIP_CHECK(hipMemcpy(*d, h, sizeof(T) * count, hipMemcpyHostToDevice));
   return 0;
}

// level sets of the lower solve (a row after all its dependencies) and of the transposed solve
void level_sets(int n, const std::vector<int>& ia, const std::vector<int>& ja, std::vector<int>& ptr,
                std::vector<int>& rows, bool transposed)
{
   std::vector<int> lev(n, 0);
   int maxlev = 0;
   if (!transposed) {
      for (int i = 0; i < n; i++) {
         int l = 0;
         for (int p = ia[i]; p < ia[i + 1] - 1; p++) l = std::max(l, lev[ja[p]] + 1);
         lev[i] = l;
         maxlev = std::max(maxlev, l);
      }
   } else {
      for (int j = n - 1; j >= 0; j--)
         for (int p = ia[j]; p < ia[j + 1] - 1; p++) lev[ja[p]] = std::max(lev[ja[p]], lev[j] + 1);
      for (int i = 0; i < n; i++) maxlev = std::max(maxlev, lev[i]);
   }
   ptr.assign(maxlev + 2, 0);
   for (int i = 0; i < n; i++) ptr[lev[i] + 1]++;
   for (int l = 0; l <= maxlev; l++) ptr[l + 1] += ptr[l];
   rows.assign(n, 0);
   std::vector<int> pos(ptr.begin(), ptr.end() - 1);
   for (int i = 0; i < n; i++) rows[pos[lev[i]]++] = i;
}

// device factors from host CSR (ia, ja, aa [, da 3 nnz]): L, L^T (column entries in ascending row order,
// the order Nfft4GPCsrMv('T') accumulates in), the map between them, the level sets
int fsai_load(PrecondFsaiAmd* F, int n, const int* ia, const int* ja, const double* aa, const double* da)
{
   F->release();
   const int nnz = ia[n];
   std::vector<int> hia(ia, ia + n + 1), hja(ja, ja + nnz);
   std::vector<int> tcnt(n + 1, 0), tia(n + 1, 0), tja(nnz), tmap(nnz);
   for (int p = 0; p < nnz; p++) tcnt[ja[p] + 1]++;
   for (int c = 0; c < n; c++) tia[c + 1] = tia[c] + tcnt[c + 1];
   std::vector<int> pos(tia.begin(), tia.end() - 1);
   for (int i = 0; i < n; i++)
      for (int p = ia[i]; p < ia[i + 1]; p++) {
         const int q = pos[ja[p]]++;
         tja[q] = i;
         tmap[q] = p;
      }
   std::vector<int> lp, lr, rp, rr;
   level_sets(n, hia, hja, lp, lr, false);
   level_sets(n, hia, hja, rp, rr, true);
   F->n = n;
   F->nnz = nnz;
   F->nlev = (int)lp.size() - 1;
   F->nrlev = (int)rp.size() - 1;
   // reverse the transposed levels: the first processed holds the rows with no later dependents
   if (upload(&F->ia, hia.data(), hia.size()) || upload(&F->ja, hja.data(), hja.size()) ||
       upload(&F->tia, tia.data(), tia.size()) || upload(&F->tja, tja.data(), tja.size()) ||
       upload(&F->tmap, tmap.data(), tmap.size()) || upload(&F->lev_ptr, lp.data(), lp.size()) ||
       upload(&F->lev_rows, lr.data(), lr.size()) || upload(&F->rlev_ptr, rp.data(), rp.size()) ||
       upload(&F->rlev_rows, rr.data(), rr.size()) || upload(&F->aa, aa, (size_t)nnz) ||
       upload(&F->taa, (const double*)nullptr, (size_t)nnz) || upload(&F->work, (const double*)nullptr, 3 * (size_t)n) ||
       upload(&F->part, (const double*)nullptr, (size_t)(n + 255) / 256 + 1))
      return -1;
   hipStream_t s = current_stream();
   hipLaunchKernelGGL(k_gather_vals, dim3((nnz + 255) / 256), dim3(256), 0, s, F->aa, F->tmap, nnz, F->taa);
   if (da) {
      if (upload(&F->da, da, 3 * (size_t)nnz) || upload(&F->tda, (const double*)nullptr, 3 * (size_t)nnz)) return -1;
      for (int g = 0; g < 3; g++)
         hipLaunchKernelGGL(k_gather_vals, dim3((nnz + 255) / 256), dim3(256), 0, s, F->da + (size_t)g * nnz, F->tmap,
                            nnz, F->tda + (size_t)g * nnz);
      F->grad = true;
   }
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int inv_l(PrecondFsaiAmd* F, double* x, const double* rhs, hipStream_t s)
{
   hipLaunchKernelGGL(k_trsv_lower, dim3(1), dim3(kTrsvThreads), 0, s, F->lev_ptr, F->nlev, F->lev_rows, F->ia, F->ja,
                      F->aa, rhs, x);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int inv_lt(PrecondFsaiAmd* F, double* x, const double* rhs, hipStream_t s)
{
   hipLaunchKernelGGL(k_trsv_upper, dim3(1), dim3(kTrsvThreads), 0, s, F->rlev_ptr, F->nrlev, F->rlev_rows, F->tia,
                      F->tja, F->taa, rhs, x);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

void csr_mv(const int* ia, const int* ja, const double* a, const double* x, double* y, int n, int beta_one,
            hipStream_t s)
{
   hipLaunchKernelGGL(k_csr_mv, dim3((n + 255) / 256), dim3(256), 0, s, ia, ja, a, x, y, n, beta_one);
}

// fsai.c:163-200 for gradient g on device vectors; y: n entries
int dvp_one(PrecondFsaiAmd* F, int g, const double* x, double* y, hipStream_t s)
{
   const int n = F->n;
   double* w1 = F->work;
   double* w2 = F->work + n;
   const double* dl = F->da + (size_t)g * F->nnz;
   const double* tdl = F->tda + (size_t)g * F->nnz;
   if (inv_lt(F, w1, x, s)) return -1;            // work = L^{-T} x
   csr_mv(F->tia, F->tja, tdl, w1, y, n, 0, s);   // y = dL^T work
   if (inv_lt(F, w2, y, s)) return -1;            // work2 = L^{-T} y
   if (inv_l(F, y, w1, s)) return -1;             // y = L^{-1} work
   csr_mv(F->ia, F->ja, dl, y, w2, n, 1, s);      // work2 += dL y
   csr_mv(F->tia, F->tja, F->taa, w2, y, n, 0, s);  // y = L^T work2
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

double diag_sum(PrecondFsaiAmd* F, const double* num, hipStream_t s)
{
   const int nb = (F->n + 255) / 256;
   hipLaunchKernelGGL(k_diag_sum, dim3(nb), dim3(256), 0, s, F->ia, F->n, num, F->aa, F->part);
   std::vector<double> h(nb);
   if (hipMemcpyAsync(h.data(), F->part, sizeof(double) * nb, hipMemcpyDeviceToHost, s) != hipSuccess ||
       hipStreamSynchronize(s) != hipSuccess)
      return NAN;
   double v = 0.0;
   for (double t : h) v += t;
   return v;
}

}  // namespace

namespace nfft4gp_amd {

int additive_buffer_info(void* str, const double** xw, int* n, int* nw, int* dw, int* skip_last, int* kernel);

// The kernel a setup evaluates: this library's additive NFFT handle as fkernel_params gives the dense
// additive kernel of its gathered window buffer (uploaded to *owned), anything else the plain kernel of
// the points with _params / _noise_level of the nfft4gp_kernel.  The kernel type comes from fkernel
// when it is one of this library's setup functions, else from `kernel`.  Returns 1 (additive), 0
// (plain) or -1.
int kernel_spec_of(void* fkernel_params, func_kernel fkernel, int kernel, int n, KernelSpec& K, double** owned)
{
   *owned = nullptr;
   const nfft4gp_kernel* kp = (const nfft4gp_kernel*)fkernel_params;
   if (!kp) return -1;
   K.kernel = kernel ? 1 : 0;
   if (fkernel == &Nfft4GPNFFTAdditiveKernelGaussianKernel) K.kernel = 0;
   else if (fkernel == &Nfft4GPNFFTAdditiveKernelMatern12Kernel) K.kernel = 1;
   K.f = kp->_params[0];
   K.l = kp->_params[1];
   K.mu = kp->_noise_level;
   K.Xk = nullptr;
   const double* xw = nullptr;
   int nn = 0, nw = 0, dw = 0, skip = 0, pk = -1;
   if (additive_buffer_info(fkernel_params, &xw, &nn, &nw, &dw, &skip, &pk)) return 0;
   if (nn != n || nw <= 0 || dw <= 0 || skip >= dw) {
      fprintf(stderr, "nfft4gp_amd: the additive handle holds %d points, the setup got %d\n", nn, n);
      return -1;
   }
   if (fkernel != &Nfft4GPNFFTAdditiveKernelGaussianKernel && fkernel != &Nfft4GPNFFTAdditiveKernelMatern12Kernel &&
       pk >= 0)
      K.kernel = pk;
   const size_t D = (size_t)(nw - 1) * dw + (dw - skip);
   if (upload(owned, xw, D * (size_t)n)) return -1;
   K.Xk = *owned;
   K.ldk = n;
   K.nw = nw;
   K.dw = dw;
   K.last_dw = dw - skip;
   return 1;
}

// The FSAI of a kernel matrix (fsai.c:314-673) from device coordinates: KNN pattern, per-row values (and
// gradients), copied to host CSR.  dW (kw x n, optional): the Schur-complement kernel of the AFN setup.
int fsai_kernel_csr(const double* dX, int n, int ldim, int d, int lfil, const KernelSpec& Ks, const double* dW, int kw,
                    int require_grad, std::vector<int>& hia, std::vector<int>& hja, std::vector<double>& haa,
                    std::vector<double>& hda, hipStream_t s, const double* dGB, const double* dGC, void** keep)
{
   if (n <= 0 || ldim < n || d <= 0 || d > kMaxDims || lfil < 1 || lfil > kFsaiMaxK || (dW && kw <= 0)) {
      fprintf(stderr, "nfft4gp_amd: FSAI setup needs 1 <= lfil <= %d and at most %d features\n", kFsaiMaxK,
              kMaxDims);
      return -1;
   }
   if (require_grad && dW && !dGC) {
      fprintf(stderr, "nfft4gp_amd: FSAI setup: gradients of the Schur-complement kernel need its B / C panels\n");
      return -1;
   }
   // pattern row pointers (kernels.c:133-168): dense rows below lfil, lfil entries after
   hia.assign(n + 1, 0);
   for (int i = 0; i < n; i++) hia[i + 1] = hia[i] + ((n <= lfil || i < lfil) ? i + 1 : lfil);
   const int nnz = hia[n];
   hja.assign((size_t)nnz, 0);
   for (int i = 0; i < std::min(n, n <= lfil ? n : lfil); i++)
      for (int j = 0; j <= i; j++) hja[hia[i] + j] = j;
   double *daa = nullptr, *dda = nullptr;
   int *dia = nullptr, *dja = nullptr;
   auto cleanup = [&](int rc) {
      (void)hipStreamSynchronize(s);
      for (double* p : {daa, dda}) (void)hipFree(p);
      for (int* p : {dia, dja}) (void)hipFree(p);
      return rc;
   };
   if (upload(&dia, hia.data(), hia.size()) || upload(&dja, hja.data(), hja.size()) ||
       upload(&daa, (const double*)nullptr, (size_t)nnz) ||
       (require_grad && upload(&dda, (const double*)nullptr, 3 * (size_t)nnz)))
      return cleanup(-1);
   if (n > lfil) {
      const int nfail = knn_pattern(dX, n, ldim, d, lfil, dia, dja, s, -1);
      if (nfail < 0) return cleanup(-1);
      knn_fallback_rows = nfail;
   }
   const KernelParams P = kernel_params_of(Ks, d);
   const double* Xk = Ks.Xk ? Ks.Xk : dX;
   const long long ldk = Ks.Xk ? Ks.ldk : ldim;
   auto rows_kernel = fsai_rows_kernel(lfil);
   hipLaunchKernelGGL(rows_kernel, dim3(n), dim3(64), 0, s, Xk, ldk, dia, dja, P, dW, kw, require_grad ? 1 : 0, nnz,
                      daa, dda, dGB, dGC, (const int*)nullptr);
   if (keep && !require_grad) {  // the caller builds the handle on the device
      if (hipGetLastError() != hipSuccess) return cleanup(-1);
      keep[0] = dia;
      keep[1] = dja;
      keep[2] = daa;
      dia = nullptr;
      dja = nullptr;
      daa = nullptr;
      hja.clear();
      haa.clear();
      hda.clear();
      return cleanup(0);
   }
   haa.assign((size_t)nnz, 0.0);
   hda.assign(require_grad ? 3 * (size_t)nnz : 0, 0.0);
   if (hipGetLastError() != hipSuccess ||
       hipMemcpyAsync(hja.data(), dja, sizeof(int) * nnz, hipMemcpyDeviceToHost, s) != hipSuccess ||
       hipMemcpyAsync(haa.data(), daa, sizeof(double) * nnz, hipMemcpyDeviceToHost, s) != hipSuccess ||
       (require_grad &&
        hipMemcpyAsync(hda.data(), dda, sizeof(double) * hda.size(), hipMemcpyDeviceToHost, s) != hipSuccess) ||
       hipStreamSynchronize(s) != hipSuccess)
      return cleanup(-1);
   return cleanup(0);
}

// A row shard's rows of the FSAI pattern (kernels.c:121-278): `rows` (ascending) of the n points; rows below
// lfil hold every earlier point, the others the lfil - 1 nearest earlier points and themselves (the
// screened scans over this rank's rows only).  hia: m + 1 pointers over the listed rows, hja: point indices.
int fsai_pattern_rows(const double* dX, int n, int ldim, int d, int lfil, const std::vector<int>& rows,
                      std::vector<int>& hia, std::vector<int>& hja, hipStream_t s)
{
   if (n <= 0 || ldim < n || d <= 0 || d > kMaxDims || lfil < 1 || lfil > kFsaiMaxK) return -1;
   const int m = (int)rows.size();
   hia.assign(m + 1, 0);
   std::vector<int> iav((size_t)n + 1, 0), knn_rows;
   for (int r = 0; r < m; r++) {
      const int i = rows[r];
      const int len = (n <= lfil || i < lfil) ? i + 1 : lfil;
      iav[i] = hia[r];
      hia[r + 1] = hia[r] + len;
      if (!(n <= lfil || i < lfil)) knn_rows.push_back(i);
   }
   hja.assign((size_t)hia[m], 0);
   for (int r = 0; r < m; r++)
      if (n <= lfil || rows[r] < lfil)
         for (int j = 0; j <= rows[r]; j++) hja[hia[r] + j] = j;
   if (knn_rows.empty()) return 0;
   int *dia = nullptr, *dja = nullptr, *drows = nullptr;
   auto cleanup = [&](int rc) {
      (void)hipStreamSynchronize(s);
      for (int* p : {dia, dja, drows}) (void)hipFree(p);
      return rc;
   };
   if (upload(&dia, iav.data(), iav.size()) || upload(&dja, hja.data(), hja.size()) ||
       upload(&drows, knn_rows.data(), knn_rows.size()))
      return cleanup(-1);
   const int nf = knn_pattern(dX, n, ldim, d, lfil, dia, dja, s, -1, drows, (int)knn_rows.size());
   if (nf < 0 || hipMemcpyAsync(hja.data(), dja, sizeof(int) * hja.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
       hipStreamSynchronize(s) != hipSuccess)
      return cleanup(-1);
   knn_fallback_rows = nf;
   return cleanup(0);
}

// Values of `nrows` pattern rows (device ia over those rows, absolute offsets into ja / aa) of the kernel (or,
// with W, the Schur-complement kernel): k_fsai_rows, W's column of each entry from wcol (nullptr: the point).
int fsai_values_rows(const KernelSpec& Ks, const double* dX, long long ldim, int d, int lfil, const int* dia,
                     const int* dja, int nrows, const double* dW, int kw, const int* dwcol, double* daa, hipStream_t s)
{
   if (nrows <= 0) return 0;
   const KernelParams P = kernel_params_of(Ks, d);
   const double* Xk = Ks.Xk ? Ks.Xk : dX;
   const long long ldk = Ks.Xk ? Ks.ldk : ldim;
   auto rows_kernel = fsai_rows_kernel(lfil);
   hipLaunchKernelGGL(rows_kernel, dim3(nrows), dim3(64), 0, s, Xk, ldk, dia, dja, P, dW, kw, 0, 0, daa,
                      (double*)nullptr, (const double*)nullptr, (const double*)nullptr, dwcol);
   return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---- the Schur FSAI's operators for the AFN gradients (afn_grad.hip) ----------------------------------
void* fsai_grad_create(int n, const int* ia, const int* ja, const double* aa, const double* da)
{
   PrecondFsaiAmd* F = new PrecondFsaiAmd();
   if (fsai_load(F, n, ia, ja, aa, da)) {
      F->release();
      delete F;
      return nullptr;
   }
   return F;
}

void fsai_grad_free(void* F)
{
   if (!F) return;
   ((PrecondFsaiAmd*)F)->release();
   delete (PrecondFsaiAmd*)F;
}

// y = G x (op 0), G^T x (1), G^{-1} x (2), G^{-T} x (3), dG_g x (4), dG_g^T x (5); x != y
int fsai_grad_op(void* vF, int op, int g, const double* x, double* y, hipStream_t s)
{
   PrecondFsaiAmd* F = (PrecondFsaiAmd*)vF;
   const int n = F->n;
   switch (op) {
      case 0: csr_mv(F->ia, F->ja, F->aa, x, y, n, 0, s); break;
      case 1: csr_mv(F->tia, F->tja, F->taa, x, y, n, 0, s); break;
      case 2: return inv_l(F, y, x, s);
      case 3: return inv_lt(F, y, x, s);
      case 4: csr_mv(F->ia, F->ja, F->da + (size_t)g * F->nnz, x, y, n, 0, s); break;
      case 5: csr_mv(F->tia, F->tja, F->tda + (size_t)g * F->nnz, x, y, n, 0, s); break;
      default: return -1;
   }
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

// sum_i dG_g(i,i) / G(i,i) (g = 0..2), or sum_i log(1 / G(i,i)) (g < 0)
double fsai_grad_diag(void* vF, int g, hipStream_t s)
{
   PrecondFsaiAmd* F = (PrecondFsaiAmd*)vF;
   return diag_sum(F, g < 0 ? nullptr : F->da + (size_t)g * F->nnz, s);
}

}  // namespace nfft4gp_amd

extern "C" {

void* Nfft4GPAmdPrecondFsaiCreate(void) { return new PrecondFsaiAmd(); }

void Nfft4GPAmdPrecondFsaiSetLfil(void* str, int lfil)
{
   if (str) ((PrecondFsaiAmd*)str)->lfil = lfil;
}

void Nfft4GPAmdPrecondFsaiSetKernel(void* str, int kernel)
{
   if (str) ((PrecondFsaiAmd*)str)->kernel = kernel ? 1 : 0;
}

void Nfft4GPAmdPrecondFsaiReset(void* str)
{
   if (str) ((PrecondFsaiAmd*)str)->release();  // keeps lfil (fsai.c:60-98)
}

void Nfft4GPAmdPrecondFsaiFree(void* str)
{
   PrecondFsaiAmd* F = (PrecondFsaiAmd*)str;
   if (!F) return;
   F->release();
   delete F;
}

int Nfft4GPAmdPrecondFsaiSetupWithKernel(double* data, int n, int ldim, int d, func_kernel fkernel,
                                         void* fkernel_params, int require_grad, void* vfsai_mat)
{
   PrecondFsaiAmd* F = (PrecondFsaiAmd*)vfsai_mat;
   if (!F || !need_device("Nfft4GPAmdPrecondFsaiSetupWithKernel")) return -1;
   if (!fkernel_params || !data || n <= 0 || ldim < n || d <= 0) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdPrecondFsaiSetupWithKernel needs data and kernel parameters\n");
      return -1;
   }
   KernelSpec K;
   double* dXk = nullptr;
   if (kernel_spec_of(fkernel_params, fkernel, F->kernel, n, K, &dXk) < 0) return -1;
   hipStream_t s = current_stream();
   double* dX = nullptr;
   if (upload(&dX, (const double*)nullptr, (size_t)ldim * d) ||
       hipMemcpy(dX, data, sizeof(double) * (size_t)ldim * d, hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(dX);
      (void)hipFree(dXk);
      return -1;
   }
   std::vector<int> hia, hja;
   std::vector<double> haa, hda;
   const int rc = fsai_kernel_csr(dX, n, ldim, d, F->lfil, K, nullptr, 0, require_grad, hia, hja, haa, hda, s);
   (void)hipStreamSynchronize(s);
   (void)hipFree(dX);
   (void)hipFree(dXk);
   if (rc) return -1;
   return fsai_load(F, n, hia.data(), hja.data(), haa.data(), require_grad ? hda.data() : nullptr);
}

int Nfft4GPAmdPrecondFsaiSetCsr(void* vfsai_mat, int n, const int* ia, const int* ja, const double* aa,
                                const double* da)
{
   PrecondFsaiAmd* F = (PrecondFsaiAmd*)vfsai_mat;
   if (!F || !ia || !ja || !aa || !need_device("Nfft4GPAmdPrecondFsaiSetCsr")) return -1;
   return fsai_load(F, n, ia, ja, aa, da);
}

int Nfft4GPAmdPrecondFsaiCsr(void* vfsai_mat, int* ia, int* ja, double* aa, double* da)
{
   PrecondFsaiAmd* F = (PrecondFsaiAmd*)vfsai_mat;
   if (!F || !F->ia) return -1;
   const int n = F->n, nnz = F->nnz;
   if (ia) NFFT4GP_HIP_CHECK(hipMemcpy(ia, F->ia, sizeof(int) * (n + 1), hipMemcpyDeviceToHost));
   if (ja) NFFT4GP_HIP_CHECK(hipMemcpy(ja, F->ja, sizeof(int) * nnz, hipMemcpyDeviceToHost));
   if (aa) NFFT4GP_HIP_CHECK(hipMemcpy(aa, F->aa, sizeof(double) * nnz, hipMemcpyDeviceToHost));
   if (da && F->da) NFFT4GP_HIP_CHECK(hipMemcpy(da, F->da, sizeof(double) * 3 * nnz, hipMemcpyDeviceToHost));
   return nnz;
}

int Nfft4GPAmdPrecondFsaiSolve(void* vfsai_mat, int n, double* x, double* rhs)
{
   PrecondFsaiAmd* F = (PrecondFsaiAmd*)vfsai_mat;
   if (!F || !F->ia || n != F->n) return -1;
   hipStream_t s = current_stream();
   Vec vx, vr;
   if (vx.open(x, n, false) || vr.open(rhs, n, true)) return -1;
   csr_mv(F->ia, F->ja, F->aa, vr.d, F->work, n, 0, s);    // work = L rhs
   csr_mv(F->tia, F->tja, F->taa, F->work, vx.d, n, 0, s);  // x = L^T work
   NFFT4GP_HIP_CHECK(hipGetLastError());
   vr.close(false);
   vx.close(true);
   return 0;
}

int Nfft4GPAmdPrecondFsaiInvL(void* vfsai_mat, int n, double* x, double* rhs)
{
   PrecondFsaiAmd* F = (PrecondFsaiAmd*)vfsai_mat;
   if (!F || !F->ia || n != F->n) return -1;
   Vec vx, vr;
   if (vx.open(x, n, false) || vr.open(rhs, n, true)) return -1;
   const int rc = inv_l(F, vx.d, vr.d, current_stream());
   vr.close(false);
   vx.close(rc == 0);
   return rc;
}

int Nfft4GPAmdPrecondFsaiInvLT(void* vfsai_mat, int n, double* x, double* rhs)
{
   PrecondFsaiAmd* F = (PrecondFsaiAmd*)vfsai_mat;
   if (!F || !F->ia || n != F->n) return -1;
   Vec vx, vr;
   if (vx.open(x, n, false) || vr.open(rhs, n, true)) return -1;
   const int rc = inv_lt(F, vx.d, vr.d, current_stream());
   vr.close(false);
   vx.close(rc == 0);
   return rc;
}

int Nfft4GPAmdPrecondFsaiDvp(void* vfsai_mat, int n, int* mask, double* x, double** yp)
{
   PrecondFsaiAmd* F = (PrecondFsaiAmd*)vfsai_mat;
   if (!F || !F->ia || n != F->n) return -1;
   if (!F->grad) {
      printf("Setup FSAI without gradient, trace not supported.\n");  // fsai.c:139-143
      return -1;
   }
   if (!yp) {
      printf("output pointer cannot be NULL\n");
      return -1;
   }
   if (!*yp) {
      if (is_device_ptr(x)) {
         if (hipMalloc((void**)yp, sizeof(double) * 3 * (size_t)n) != hipSuccess) return -1;
         NFFT4GP_HIP_CHECK(hipMemset(*yp, 0, sizeof(double) * 3 * (size_t)n));
      } else {
         *yp = (double*)calloc(3 * (size_t)n, sizeof(double));
      }
   }
   hipStream_t s = current_stream();
   Vec vx, vy;
   if (vx.open(x, n, true) || vy.open(*yp, 3 * (size_t)n, true)) return -1;
   int rc = 0;
   for (int g = 0; g < 3 && !rc; g++)
      if (!mask || mask[g]) rc = dvp_one(F, g, vx.d, vy.d + (size_t)g * n, s);
   vx.close(false);
   vy.close(rc == 0);
   return rc;
}

int Nfft4GPAmdPrecondFsaiTrace(void* vfsai_mat, double** tracesp)
{
   PrecondFsaiAmd* F = (PrecondFsaiAmd*)vfsai_mat;
   if (!F || !F->ia) return -1;
   if (!F->grad) {
      printf("Setup FSAI without gradient, trace not supported.\n");  // fsai.c:225-229
      return -1;
   }
   if (!tracesp) {
      printf("Trace pointer cannot be NULL\n");
      return -1;
   }
   double* traces = *tracesp ? *tracesp : (double*)calloc(3, sizeof(double));
   hipStream_t s = current_stream();
   // the reference adds to what the array holds, then doubles (fsai.c:256-265)
   for (int g = 0; g < 3; g++) traces[g] = 2.0 * (traces[g] + diag_sum(F, F->da + (size_t)g * F->nnz, s));
   *tracesp = traces;
   return 0;
}

double Nfft4GPAmdPrecondFsaiLogdet(void* vfsai_mat)
{
   PrecondFsaiAmd* F = (PrecondFsaiAmd*)vfsai_mat;
   if (!F || !F->ia) return NAN;
   return 2.0 * diag_sum(F, nullptr, current_stream());
}

// Test hook: the KNN pattern (column indices of rows lfil..n-1, lfil each) of the host points X (n x d,
// leading dimension ldim) with the given variant (knn_pattern); *nfail = rows handed to k_knn.
int Nfft4GPAmdDebugKnn(const double* X, int n, int ldim, int d, int lfil, int variant, int* ja_out, int* nfail)
{
   if (n <= lfil || lfil < 1 || lfil > kFsaiMaxK || d <= 0 || d > kMaxDims || ldim < n) return -1;
   hipStream_t s = current_stream();
   std::vector<int> hia(n + 1, 0);
   for (int i = 0; i < n; i++) hia[i + 1] = hia[i] + (i < lfil ? i + 1 : lfil);
   double* dX = nullptr;
   int *dia = nullptr, *dja = nullptr;
   int rc = -1;
   if (upload(&dX, X, (size_t)ldim * d) == 0 && upload(&dia, hia.data(), hia.size()) == 0 &&
       upload(&dja, (const int*)nullptr, (size_t)hia[n]) == 0) {
      const int nf = knn_pattern(dX, n, ldim, d, lfil, dia, dja, s, variant);
      if (nf >= 0 && hipMemcpyAsync(ja_out, dja + hia[lfil], sizeof(int) * (size_t)(n - lfil) * lfil,
                                    hipMemcpyDeviceToHost, s) == hipSuccess &&
          hipStreamSynchronize(s) == hipSuccess) {
         if (nfail) *nfail = nf;
         rc = 0;
      }
   }
   (void)hipStreamSynchronize(s);
   (void)hipFree(dX);
   (void)hipFree(dia);
   (void)hipFree(dja);
   return rc;
}

}  // extern "C"
