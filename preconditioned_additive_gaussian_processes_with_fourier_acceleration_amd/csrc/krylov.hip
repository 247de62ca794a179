// krylov.hip -- FGMRES, preconditioned Lanczos, stochastic Lanczos quadrature and the GP loss, with
// every n-vector (Krylov bases, iterates, probes) in HBM.
//
//   Nfft4GPSolverFgmres            SRC/solvers/fgmres.c:3-252   restarted flexible GMRES, MGS without
//                                                               re-orthogonalisation, the reference's
//                                                               restart and breakdown behaviour
//   Nfft4GPSolverLanczos           SRC/solvers/lanczos.c:3-419  M-inner-product Lanczos with full MGS2
//                                                               re-orthogonalisation (matops.c:348-440)
//   Nfft4GPLanczosQuadratureLogdet SRC/solvers/lanczos.c:421-610
//   Nfft4GPGpLoss                  SRC/optimizer/gp_loss.c:96-307
//   Nfft4GPTransform               SRC/optimizer/transform.c:4-89
//   Nfft4GPAdditiveNFFTGpPredict   SRC/external/nfft_interface.c:873-1068 (posterior mean, and the
//                                  predictive standard deviation by one solve per prediction point)
//
// The small dense work (Givens rotations, the Cholesky of T, the tridiagonal eigensolve) runs on the
// host on scalars read back once per iteration; each Gram-Schmidt step is one fused launch (apply the
// previous projection, then the next inner product, reduced on the device in a fixed order).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "callbacks.hpp"
#include "internal.h"
#include "reduce.hpp"

using namespace nfft4gp_amd;

namespace {

constexpr int kKThreads = 256;
constexpr int kKEPT = 4;
constexpr int kKMaxBlocks = 2048;  // <= kRedMaxBlocks

int kgrid(size_t n)
{
   size_t g = (n + (size_t)kKThreads * kKEPT - 1) / ((size_t)kKThreads * kKEPT);
   g = std::min<size_t>(g, kKMaxBlocks);
   return (int)(g == 0 ? 1 : g);
}

// w -= (*hprev) * u (when u != nullptr); then *out = (w, v) (v != nullptr) or ||w||^2 (v == nullptr).
// T threads per block: 1024 gives a quarter of the partials for the last block to add (the MGS loop of
// FGMRES runs one of these per projection, so its serial tail is most of a step at n = 1e6).
template <int T, int EPT>
__device__ __forceinline__ void gs_body(double* __restrict__ w, const double* __restrict__ u, double h,
                                        const double* __restrict__ v, size_t n, double* __restrict__ part,
                                        unsigned int* __restrict__ ticket, double* __restrict__ out)
{
   double acc = 0.0;
   const size_t stride = (size_t)gridDim.x * T * EPT;
   for (size_t i0 = (size_t)blockIdx.x * T * EPT + threadIdx.x; i0 < n; i0 += stride) {
      double wv[EPT], uv[EPT], vv[EPT];
#pragma unroll
      for (int e = 0; e < EPT; e++) {
         const size_t i = i0 + (size_t)e * T;
         wv[e] = i < n ? w[i] : 0.0;
         uv[e] = (u && i < n) ? u[i] : 0.0;
         vv[e] = (v && i < n) ? v[i] : 0.0;
      }
#pragma unroll
      for (int e = 0; e < EPT; e++) {
         const size_t i = i0 + (size_t)e * T;
         if (u) {
            wv[e] = fma(-h, uv[e], wv[e]);
            if (i < n) w[i] = wv[e];
         }
         acc = v ? fma(wv[e], vv[e], acc) : fma(wv[e], wv[e], acc);
      }
   }
   acc = block_sum0<T>(acc);
   double tot;
   if (grid_total<T>(acc, part, ticket, &tot) && threadIdx.x == 0) *out = tot;
}

template <int T, int EPT = kKEPT>
__global__ __launch_bounds__(T) void k_gs_step(double* __restrict__ w, const double* __restrict__ u,
                                               const double* __restrict__ hprev, const double* __restrict__ v,
                                               size_t n, double* __restrict__ part, unsigned int* __restrict__ ticket,
                                               double* __restrict__ out)
{
   gs_body<T, EPT>(w, u, u ? *hprev : 0.0, v, n, part, ticket, out);
}

// k_gs_step for several systems of one batch at once (the predict's std solves, fgmres_batch_dev): blockIdx.y
// runs system s = act[y], whose operands sit ld* doubles apart (w + s ldw, ...), its scalars at hprev[s] and
// out[s]; one partials / ticket pair per y.  Per system the arithmetic is k_gs_step's (same grid): bitwise.
template <int T, int EPT>
__global__ __launch_bounds__(T) void k_gs_batch(double* __restrict__ w, size_t ldw, const double* __restrict__ u,
                                                size_t ldu, const double* __restrict__ hprev,
                                                const double* __restrict__ v, size_t ldv, size_t n,
                                                const int* __restrict__ act, double* __restrict__ part,
                                                unsigned int* __restrict__ ticket, double* __restrict__ out)
{
   const int s = act[blockIdx.y];
   gs_body<T, EPT>(w + (size_t)s * ldw, u ? u + (size_t)s * ldu : nullptr, u ? hprev[s] : 0.0,
                   v ? v + (size_t)s * ldv : nullptr, n, part + (size_t)blockIdx.y * kKMaxBlocks,
                   ticket + (size_t)blockIdx.y * kTicketWords, out + s);
}

// The whole MGS sweep of one FGMRES step in ONE launch (Nfft4GPModifiedGS, matops.c:274-346, as the chain of
// k_gs_step launches Ctx::gs makes): w stays in registers across the i projections and the norm, each step
// reads only v_j (v_{j-1}, the previous step's u, is still in registers; v_{j+1}'s loads go out before the
// step's wait), and the grid-wide sum of step j (reduce.hpp's last arriver) reaches every workgroup through
// hd[j] itself: the host presets hd[0..i] to an all-ones NaN pattern (kChainUnset) that no sum of finite data
// produces, the last arriver stores the sum there (agent scope, after its ticket resets have landed) and the
// others poll it until it changes -- no fences, as reduce.hpp.  Needs a grid that is resident at once and covers
// n in one pass (the host checks the occupancy).  Per element and per reduction the arithmetic is k_gs_step's on
// the same grid, so hd[0..i] and w are bitwise the chain's.  A wait that gives up sets *err (host: an error).
// BATCH (fgmres_batch_dev, the predict's std solves): blockIdx.y runs system s = act[y] of a batch of m, whose
// column j is cols[j] + s n (w: column i), its scalars at hd[j m + s], one partials / ticket pair per y
constexpr unsigned long long kChainUnset = ~0ull;  // hd[j] before step j's sum is published

template <int T, int EPT, bool BATCH = false>
__global__ __launch_bounds__(T) void k_mgs_chain(double* __restrict__ w, const double* __restrict__ V, size_t n,
                                                 int i, double* __restrict__ hd, double* __restrict__ part,
                                                 unsigned int* __restrict__ ticket,
                                                 int* __restrict__ err, const double* const* __restrict__ cols = nullptr,
                                                 const int* __restrict__ act = nullptr, int m = 1)
{
   __shared__ double s_h;
   __shared__ int s_fail;
   int hs = 1;  // hd stride between steps
   if (BATCH) {
      const int sy = act[blockIdx.y];
      w = const_cast<double*>(cols[i]) + (size_t)sy * n;
      hd += sy;
      hs = m;
      part += (size_t)blockIdx.y * kKMaxBlocks;
      ticket += (size_t)blockIdx.y * kTicketWords;
   }
   auto col = [&](int j) -> const double* {
      return BATCH ? cols[j] + (size_t)act[blockIdx.y] * n : V + (size_t)j * n;
   };
   const size_t i0 = (size_t)blockIdx.x * T * EPT + threadIdx.x;
   double wv[EPT], pv[EPT], vn[EPT];
   const double* v0 = i > 0 ? col(0) : nullptr;
#pragma unroll
   for (int e = 0; e < EPT; e++) {
      const size_t k = i0 + (size_t)e * T;
      wv[e] = k < n ? w[k] : 0.0;
      pv[e] = 0.0;
      vn[e] = (v0 && k < n) ? v0[k] : 0.0;  // v_0
   }
   if (threadIdx.x == 0) s_fail = 0;
   for (int j = 0; j <= i; j++) {
      if (j > 0) {
         const double h = s_h;
#pragma unroll
         for (int e = 0; e < EPT; e++) wv[e] = fma(-h, pv[e], wv[e]);
      }
      double acc = 0.0;
      if (j < i) {
         double vv[EPT];
#pragma unroll
         for (int e = 0; e < EPT; e++) vv[e] = vn[e];
         // v_{j+1}'s loads go out now: they do not depend on this step's sum, so they overlap its grid-wide wait
         if (j + 1 < i) {
            const double* v1 = col(j + 1);
#pragma unroll
            for (int e = 0; e < EPT; e++) {
               const size_t k = i0 + (size_t)e * T;
               vn[e] = k < n ? v1[k] : 0.0;
            }
         }
#pragma unroll
         for (int e = 0; e < EPT; e++) {
            acc = fma(wv[e], vv[e], acc);
            pv[e] = vv[e];
         }
      } else {
#pragma unroll
         for (int e = 0; e < EPT; e++) acc = fma(wv[e], wv[e], acc);
      }
      acc = block_sum0<T>(acc);
      double tot;
      unsigned long long* slot = reinterpret_cast<unsigned long long*>(hd + (size_t)j * hs);
      if (grid_total<T>(acc, part, ticket, &tot)) {
         if (threadIdx.x == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ticket resets land before the publish
            __hip_atomic_store(slot, (unsigned long long)__double_as_longlong(tot), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            s_h = tot;
         }
      } else if (threadIdx.x == 0) {
         unsigned long long b = kChainUnset;
         for (long spin = 0; spin < (1l << 22); spin++) {
            b = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (b != kChainUnset) break;
            __builtin_amdgcn_s_sleep(1);
         }
         if (b != kChainUnset) {
            s_h = __longlong_as_double((long long)b);
         } else {
            s_fail = 1;
            __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
         }
      }
      __syncthreads();
      if (s_fail) return;  // the others time out at the next step in turn
   }
#pragma unroll
   for (int e = 0; e < EPT; e++) {
      const size_t k = i0 + (size_t)e * T;
      if (k < n) w[k] = wv[e];
   }
}

// The MGS sweep in ONE launch for vectors too long for k_mgs_chain's one-pass grid (config E, n = 1e7): w stays
// in registers across the whole sweep -- S strided passes of 4 elements per thread, exactly the elements and the
// order k_gs_step<1024, 4> visits on the same grid -- while v_{j-1} is re-read for each update instead of being
// held (w, v_{j-1} and v_j would not fit the register file at this n).  Step j: w -= h_{j-1} v_{j-1}, then
// (w, v_j) (the last step ||w||^2), summed by reduce.hpp's last arriver and published into the preset hd[j] as
// k_mgs_chain does (bounded waits, *err).  Per element and per reduction the arithmetic of the per-projection
// chain on this grid (Ctx::mgs_grid): bitwise equal to it.  Moves 2 vectors per projection against the chain's
// 4 (w read and written, v_{j-1}, v_j).
template <int T, int S>
__global__ __launch_bounds__(T) void k_mgs_wide(double* __restrict__ w, const double* __restrict__ V, size_t n, int i,
                                                double* __restrict__ hd, double* __restrict__ part,
                                                unsigned int* __restrict__ ticket, int* __restrict__ err)
{
   constexpr int E = 4;
   __shared__ double s_h;
   __shared__ int s_fail;
   // element (p, e) of this thread is c(p, e) + threadIdx.x with c wave-uniform: the loads take a scalar base and
   // one 32-bit lane offset, so no per-element 64-bit address stays live across the sweep
   const size_t stride = (size_t)gridDim.x * T * E;
   const size_t c0 = (size_t)blockIdx.x * T * E;
   const unsigned tid = threadIdx.x;
   auto cbase = [&](int p, int e) -> size_t { return c0 + (size_t)p * stride + (size_t)e * T; };
   double wv[S][E];
#pragma unroll
   for (int p = 0; p < S; p++)
#pragma unroll
      for (int e = 0; e < E; e++) {
         const size_t c = cbase(p, e);
         wv[p][e] = c + tid < n ? (w + c)[tid] : 0.0;
      }
   if (threadIdx.x == 0) s_fail = 0;
   for (int j = 0; j <= i; j++) {
      const double* u = j > 0 ? V + (size_t)(j - 1) * n : nullptr;
      const double* v = j < i ? V + (size_t)j * n : nullptr;
      const double h = j > 0 ? s_h : 0.0;
      double acc = 0.0;
#pragma unroll
      for (int p = 0; p < S; p++) {
         if (cbase(p, 0) + tid < n) {  // gs_body's grid-stride loop has ended for this thread past here
            double uv[E], vv[E];
#pragma unroll
            for (int e = 0; e < E; e++) {
               const size_t c = cbase(p, e);
               const bool in = c + tid < n;
               uv[e] = (u && in) ? (u + c)[tid] : 0.0;
               vv[e] = (v && in) ? (v + c)[tid] : 0.0;
            }
#pragma unroll
            for (int e = 0; e < E; e++) {
               if (u) wv[p][e] = fma(-h, uv[e], wv[p][e]);
               acc = v ? fma(wv[p][e], vv[e], acc) : fma(wv[p][e], wv[p][e], acc);
            }
         }
         // one pass's 8 loads in flight per thread: hoisting every pass's loads above the arithmetic would need
         // 16 S VGPRs beside w's 8 S
         asm volatile("" ::: "memory");
      }
      acc = block_sum0<T>(acc);
      double tot;
      unsigned long long* slot = reinterpret_cast<unsigned long long*>(hd + j);
      if (grid_total<T>(acc, part, ticket, &tot)) {
         if (threadIdx.x == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ticket resets land before the publish
            __hip_atomic_store(slot, (unsigned long long)__double_as_longlong(tot), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            s_h = tot;
         }
      } else if (threadIdx.x == 0) {
         unsigned long long b = kChainUnset;
         for (long spin = 0; spin < (1l << 22); spin++) {
            b = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (b != kChainUnset) break;
            __builtin_amdgcn_s_sleep(1);
         }
         if (b != kChainUnset) {
            s_h = __longlong_as_double((long long)b);
         } else {
            s_fail = 1;
            __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
         }
      }
      __syncthreads();
      if (s_fail) return;
   }
#pragma unroll
   for (int p = 0; p < S; p++)
#pragma unroll
      for (int e = 0; e < E; e++) {
         const size_t c = cbase(p, e);
         if (c + tid < n) (w + c)[tid] = wv[p][e];
      }
}

// k_mgs_wide's instantiations: passes S per thread
constexpr int kWideS[] = {2, 4, 6, 8, 10, 12};
typedef void (*MgsWideFn)(double*, const double*, size_t, int, double*, double*, unsigned int*, int*);
static MgsWideFn mgs_wide_fn(int S)
{
   switch (S) {
   case 2: return k_mgs_wide<1024, 2>;
   case 4: return k_mgs_wide<1024, 4>;
   case 6: return k_mgs_wide<1024, 6>;
   case 8: return k_mgs_wide<1024, 8>;
   case 10: return k_mgs_wide<1024, 10>;
   case 12: return k_mgs_wide<1024, 12>;
   default: return nullptr;
   }
}

// mgs2's local pass in ONE launch (what Ctx::block_gs(w, V + j0 n, Z + j0 n, ml, h, 1) does in three: h[0..ml) =
// [v_j0, v_j0+1]^T w, h[ml + 1] = ||w||^2 before, w -= Z_loc h, h[ml] = ||w||^2 after).  The ml + 1 grid-wide sums
// of the first half are reduce.hpp's last-arriver sums (one partials / ticket pair each), published into hd
// slots the host preset to kChainUnset; every workgroup waits for the projections (bounded), updates its w
// and forms the norm after, whose last arriver writes hd[ml].  alias: Z_loc == V_loc (no preconditioner), so
// the update reuses the loaded columns.  The same sums as block_gs's up to their order (rounding level).
template <int T, int EPT>
__global__ __launch_bounds__(T) void k_lanczos_local(double* __restrict__ w, const double* __restrict__ V0,
                                                     const double* __restrict__ Z0, int alias, size_t n, int ml,
                                                     double* __restrict__ hd, double* __restrict__ part,
                                                     unsigned int* __restrict__ ticket, int* __restrict__ err)
{
   __shared__ double s_sc[3][T / 64];
   __shared__ int s_last[3];
   __shared__ double s_h[2];
   __shared__ int s_fail;
   const size_t i0 = (size_t)blockIdx.x * T * EPT + threadIdx.x;
   double wv[EPT], v0[EPT], v1[EPT];
#pragma unroll
   for (int e = 0; e < EPT; e++) {
      const size_t k = i0 + (size_t)e * T;
      const bool in = k < n;
      wv[e] = in ? w[k] : 0.0;
      v0[e] = in ? V0[k] : 0.0;
      v1[e] = (in && ml == 2) ? V0[n + k] : 0.0;
   }
   double a0 = 0.0, a1 = 0.0, an = 0.0;
#pragma unroll
   for (int e = 0; e < EPT; e++) {
      a0 = fma(wv[e], v0[e], a0);
      a1 = fma(wv[e], v1[e], a1);
      an = fma(wv[e], wv[e], an);
   }
   if (threadIdx.x == 0) s_fail = 0;
   const double sums[3] = {a0, a1, an};
   // hd slots: [0] (w, v_j0), [1] (w, v_j0+1) when ml == 2, [ml + 1] ||w||^2 before
   const int slot_of[3] = {0, 1, ml + 1};
#pragma unroll
   for (int q = 0; q < 3; q++) {
      if (q == 1 && ml != 2) continue;
      double b = block_sum0_s<T>(sums[q], s_sc[q]);
      double tot;
      if (grid_total_s<T>(b, part + (size_t)q * kKMaxBlocks, ticket + (size_t)q * kTicketWords, &tot, &s_last[q],
                          s_sc[q]) &&
          threadIdx.x == 0) {
         asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ticket resets land before the publish
         __hip_atomic_store(reinterpret_cast<unsigned long long*>(hd + slot_of[q]),
                            (unsigned long long)__double_as_longlong(tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
   }
   if (threadIdx.x == 0) {
      for (int j = 0; j < ml; j++) {
         unsigned long long* sl = reinterpret_cast<unsigned long long*>(hd + j);
         unsigned long long b = kChainUnset;
         for (long spin = 0; spin < (1l << 22); spin++) {
            b = __hip_atomic_load(sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (b != kChainUnset) break;
            __builtin_amdgcn_s_sleep(1);
         }
         if (b == kChainUnset) {
            s_fail = 1;
            __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
         }
         s_h[j] = __longlong_as_double((long long)b);
      }
   }
   __syncthreads();
   if (s_fail) return;
   const double h0 = s_h[0], h1 = ml == 2 ? s_h[1] : 0.0;
   double acc = 0.0;
#pragma unroll
   for (int e = 0; e < EPT; e++) {
      const size_t k = i0 + (size_t)e * T;
      const bool in = k < n;
      const double z0 = alias ? v0[e] : (in ? Z0[k] : 0.0);
      const double z1 = ml == 2 ? (alias ? v1[e] : (in ? Z0[n + k] : 0.0)) : 0.0;
      wv[e] = fma(-h0, z0, wv[e]);
      if (ml == 2) wv[e] = fma(-h1, z1, wv[e]);
      if (in) w[k] = wv[e];
      acc = fma(wv[e], wv[e], acc);
   }
   // the norm after: tickets of pair 0 again (every workgroup is past that pair's publish, so its reset landed)
   const double b = block_sum0_s<T>(acc, s_sc[0]);
   double tot;
   if (grid_total_s<T>(b, part + 3 * (size_t)kKMaxBlocks, ticket, &tot, &s_last[0], s_sc[0]) && threadIdx.x == 0)
      hd[ml] = tot;
}

// a[s] *= fac[s] for the systems act[y] (k_scale2's arithmetic)
__global__ void k_scale_batch(double* __restrict__ a, size_t lda, size_t n, const int* __restrict__ act,
                              const double* __restrict__ fac)
{
   const int s = act[blockIdx.y];
   const double f = fac[s];
   double* p = a + (size_t)s * lda;
   for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] *= f;
}

// x += sum_j c[j] cols[j] (columns in order: k_combine's arithmetic over columns that need not be contiguous)
__global__ void k_combine_cols(double* __restrict__ x, const double* const* __restrict__ cols, size_t n,
                               const double* __restrict__ c, int m)
{
   for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
      double v = x[i];
      for (int j = 0; j < m; j++) v = fma(c[j], cols[j][i], v);
      x[i] = v;
   }
}

// E[s ld + r0 + s] = 1 (unit columns of the predict's K12 / K22 probes; E zeroed before)
__global__ void k_set_units(double* __restrict__ E, size_t ld, size_t r0, int m)
{
   const int s = blockIdx.x * blockDim.x + threadIdx.x;
   if (s < m) E[(size_t)s * ld + r0 + s] = 1.0;
}

// out[s] = Y[s ld + r0 + s]
__global__ void k_pick_diag(double* __restrict__ out, const double* __restrict__ Y, size_t ld, size_t r0, int m)
{
   const int s = blockIdx.x * blockDim.x + threadIdx.x;
   if (s < m) out[s] = Y[(size_t)s * ld + r0 + s];
}

// out[0] = (a, b), out[1] = (b, b): the Lanczos (v, z) and ||z||^2 in one pass
__global__ __launch_bounds__(kKThreads) void k_dot2(const double* __restrict__ a, const double* __restrict__ b,
                                                    size_t n, double* __restrict__ part,
                                                    unsigned int* __restrict__ ticket, double* __restrict__ part2,
                                                    unsigned int* __restrict__ ticket2, double* __restrict__ out)
{
   double ab = 0.0, bb = 0.0;
   const size_t stride = (size_t)gridDim.x * kKThreads * kKEPT;
   for (size_t i0 = (size_t)blockIdx.x * kKThreads * kKEPT + threadIdx.x; i0 < n; i0 += stride) {
      double av[kKEPT], bv[kKEPT];
#pragma unroll
      for (int e = 0; e < kKEPT; e++) {
         const size_t i = i0 + (size_t)e * kKThreads;
         av[e] = i < n ? a[i] : 0.0;
         bv[e] = i < n ? b[i] : 0.0;
      }
#pragma unroll
      for (int e = 0; e < kKEPT; e++) {
         ab = fma(av[e], bv[e], ab);
         bb = fma(bv[e], bv[e], bb);
      }
   }
   ab = block_sum0<kKThreads>(ab);
   double tot;
   if (grid_total<kKThreads>(ab, part, ticket, &tot) && threadIdx.x == 0) out[0] = tot;
   __syncthreads();
   bb = block_sum0<kKThreads>(bb);
   if (grid_total<kKThreads>(bb, part2, ticket2, &tot) && threadIdx.x == 0) out[1] = tot;
}

__global__ void k_scale2(double* __restrict__ a, double* __restrict__ b, size_t n, double s)
{
   for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
      a[i] *= s;
      if (b) b[i] *= s;
   }
}

// x += sum_j c[j] B[:, j] (columns in order, ld = n)
__global__ void k_combine(double* __restrict__ x, const double* __restrict__ B, size_t ld, size_t n,
                          const double* __restrict__ c, int m)
{
   for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
      double v = x[i];
      for (int j = 0; j < m; j++) v = fma(c[j], B[(size_t)j * ld + i], v);
      x[i] = v;
   }
}

// y = a - b
__global__ void k_sub(double* __restrict__ y, const double* __restrict__ a, const double* __restrict__ b, size_t n)
{
   for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
      y[i] = a[i] - b[i];
}

// ---- block (classical) Gram-Schmidt passes for the Lanczos re-orthogonalisation -------------------
// One pass = two launches over the whole basis: h = V^T w (kBD basis vectors per workgroup, every
// block's partials reduced in a fixed order), then w -= Z h with ||w||^2 fused.  This reads the basis
// twice per pass instead of streaming w, z_i and v_i once per basis vector (MGS: 4 vectors moved per
// projection): 2x fewer bytes and 2 launches instead of k + 2.
constexpr int kBD = 8;
constexpr int kBDThreads = 256;
constexpr int kBDMaxBlocks = 512;

int bd_grid(size_t n)
{
   size_t g = (n + (size_t)kBDThreads * 16 - 1) / ((size_t)kBDThreads * 16);
   return (int)std::max<size_t>(1, std::min<size_t>(g, kBDMaxBlocks));
}

// part[blockIdx.x * ldp + i] = sum over this block's rows r of w[r] V[i n + r], i in [g0, g0 + kBD) & < m;
// with_norm: column m is w itself (part[.. + m] sums ||w||^2)
// c_after / c_before (optional): a second pass that runs only when the DGKS test of k_block_update holds
// FOLD: k_block_reduce folded in -- the partials are stored at agent scope, the last arriving workgroup of each
// column group (reduce.hpp's per-XCD tickets, one ticket array per group) sums them in k_block_reduce's order
// and writes h[0..m) (h[m + 1] for the norm column): one launch instead of two, the same bits
// VEC = 2: each thread reads two consecutive rows per column as one 16-byte load (the host picks it when n is even
// and w, V are 16-byte aligned, so every column is)
template <bool FOLD = false, int VEC = 1>
__global__ __launch_bounds__(kBDThreads) void k_block_dots(const double* __restrict__ w, const double* __restrict__ V,
                                                           size_t n, int m, int with_norm, double* __restrict__ part,
                                                           int ldp, const double* __restrict__ c_after = nullptr,
                                                           const double* __restrict__ c_before = nullptr,
                                                           double* __restrict__ h = nullptr,
                                                           unsigned int* __restrict__ tickets = nullptr)
{
   if (c_after && !(sqrt(*c_after) < 0.7071 * sqrt(*c_before))) return;
   __shared__ double s[kBDThreads / 64][kBD];
   const int g0 = blockIdx.y * kBD;
   const int cnt = min(kBD, m + with_norm - g0);
   const int nv = m - g0;  // columns of this group that come from V; the next one (if counted) is w
   double acc[kBD];
#pragma unroll
   for (int j = 0; j < kBD; j++) acc[j] = 0.0;
   const size_t stride = (size_t)gridDim.x * kBDThreads;
   if constexpr (VEC == 1) {
      for (size_t r = (size_t)blockIdx.x * kBDThreads + threadIdx.x; r < n; r += stride) {
         const double wr = w[r];
         double v[kBD];
#pragma unroll
         for (int j = 0; j < kBD; j++) v[j] = j < nv && j < cnt ? V[(size_t)(g0 + j) * n + r] : (j < cnt ? wr : 0.0);
#pragma unroll
         for (int j = 0; j < kBD; j++) acc[j] = fma(v[j], wr, acc[j]);
      }
   } else {
      const size_t n2 = n / 2;
      const double2* __restrict__ w2 = reinterpret_cast<const double2*>(w);
      for (size_t r = (size_t)blockIdx.x * kBDThreads + threadIdx.x; r < n2; r += stride) {
         const double2 wr = w2[r];
         double2 v[kBD];
#pragma unroll
         for (int j = 0; j < kBD; j++)
            v[j] = j < nv && j < cnt ? reinterpret_cast<const double2*>(V + (size_t)(g0 + j) * n)[r]
                                     : (j < cnt ? wr : make_double2(0.0, 0.0));
#pragma unroll
         for (int j = 0; j < kBD; j++) acc[j] = fma(v[j].y, wr.y, fma(v[j].x, wr.x, acc[j]));
      }
   }
   const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
   for (int j = 0; j < kBD; j++) {
      double a = acc[j];
      for (int off = 32; off > 0; off >>= 1) a += __shfl_down(a, off, 64);
      if (lane == 0) s[wave][j] = a;
   }
   __syncthreads();
   if (threadIdx.x < cnt) {
      double t = 0.0;
#pragma unroll
      for (int q = 0; q < kBDThreads / 64; q++) t += s[q][threadIdx.x];
      if (FOLD)
         __hip_atomic_store(part + (size_t)blockIdx.x * ldp + g0 + threadIdx.x, t, __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT);
      else
         part[(size_t)blockIdx.x * ldp + g0 + threadIdx.x] = t;
   }
   if constexpr (FOLD) {
      __shared__ int s_last;
      __shared__ double s_sum[16][kBD];
      unsigned int* ticket = tickets + (size_t)blockIdx.y * kTicketWords;
      if (threadIdx.x == 0) {  // the partial stores are wave 0's (cnt <= kBD lanes)
         asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
         const unsigned G = gridDim.x;
         const unsigned xcd = blockIdx.x % kRedXcds;
         const unsigned members = (G - xcd + kRedXcds - 1) / kRedXcds;
         const unsigned groups = G < kRedXcds ? G : kRedXcds;
         int last = 0;
         const unsigned old = __hip_atomic_fetch_add(ticket + (1 + xcd) * kTicketStride, 1u, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
         if (old == members - 1) {
            const unsigned top = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = (top == groups - 1);
         }
         s_last = last;
      }
      __syncthreads();
      if (!s_last) return;
      // k_block_reduce's sum: 16 strands per column, four accumulators cycled, then the strands in order
      const int col = threadIdx.x % kBD, g = threadIdx.x / kBD;
      if (g < 16) {
         double z[4] = {0.0, 0.0, 0.0, 0.0};
         int u = 0;
         const int nblk = (int)gridDim.x;
         const int ii = col < cnt ? g0 + col : g0 + cnt - 1;
         for (int b = g; b < nblk; b += 16, u = (u + 1) & 3)
            z[u] += __hip_atomic_load(part + (size_t)b * ldp + ii, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
         s_sum[g][col] = (z[0] + z[1]) + (z[2] + z[3]);
      }
      __syncthreads();
      if (threadIdx.x < cnt) {
         double t = 0.0;
#pragma unroll
         for (int q = 0; q < 16; q++) t += s_sum[q][threadIdx.x];
         const int i = g0 + threadIdx.x;
         h[i < m ? i : m + 1] = t;
      }
      if (threadIdx.x <= (unsigned)kRedXcds)
         __hip_atomic_store(ticket + threadIdx.x * kTicketStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
   }
}

// h[i] = sum_b part[b ldp + i] (fixed order: 16 strands over blocks b = g mod 16, then the strands) for
// i < m; column i = m (the norm column of k_block_dots, when mc = m + 1) lands in h[m + 1]
__global__ __launch_bounds__(1024) void k_block_reduce(const double* __restrict__ part, int nblk, int ldp, int mc,
                                                      int m, double* __restrict__ h)
{
   __shared__ double s_sum[16][64];
   const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
   const int i = blockIdx.x * 64 + lane;
   const int ii = i < mc ? i : mc - 1;
   double z[4] = {0.0, 0.0, 0.0, 0.0};
   int u = 0;
   for (int b = g; b < nblk; b += 16, u = (u + 1) & 3) z[u] += part[(size_t)b * ldp + ii];
   s_sum[g][lane] = (z[0] + z[1]) + (z[2] + z[3]);
   __syncthreads();
   if (g == 0 && i < mc) {
      double t = 0.0;
#pragma unroll
      for (int q = 0; q < 16; q++) t += s_sum[q][lane];
      h[i < m ? i : m + 1] = t;
   }
}

// w -= sum_{j < m} h[j] Z[j n + .] (j in order, four columns' loads in flight per step), then *out = ||w||^2
// (fixed-order grid reduction).  c_after / c_before (optional device scalars, the squared norms after and
// before the previous pass): the pass runs only when the DGKS test sqrt(after) < 0.7071 sqrt(before) holds --
// the same in every workgroup -- and *c_flag records the decision (1 / 0) for the host
// VEC = 2: two consecutive rows per 16-byte load (n even, w and Z 16-byte aligned); w's rows get the same bits,
// only the norm's summation order differs
template <int VEC = 1>
__global__ __launch_bounds__(kKThreads) void k_block_update(double* __restrict__ w, const double* __restrict__ Z,
                                                            size_t n, const double* __restrict__ h, int m,
                                                            double* __restrict__ part,
                                                            unsigned int* __restrict__ ticket,
                                                            double* __restrict__ out,
                                                            const double* __restrict__ c_after = nullptr,
                                                            const double* __restrict__ c_before = nullptr,
                                                            double* __restrict__ c_flag = nullptr)
{
   if (c_after) {
      const bool again = sqrt(*c_after) < 0.7071 * sqrt(*c_before);
      if (blockIdx.x == 0 && threadIdx.x == 0) *c_flag = again ? 1.0 : 0.0;
      if (!again) return;
   }
   extern __shared__ double s_h[];
   for (int j = threadIdx.x; j < m; j += kKThreads) s_h[j] = h[j];
   __syncthreads();
   double acc = 0.0;
   if constexpr (VEC == 2) {
      constexpr int E2 = kKEPT / 2;  // pairs per thread per step
      const size_t n2 = n / 2;
      double2* __restrict__ w2 = reinterpret_cast<double2*>(w);
      const size_t stride2 = (size_t)gridDim.x * kKThreads * E2;
      for (size_t p0 = (size_t)blockIdx.x * kKThreads * E2 + threadIdx.x; p0 < n2; p0 += stride2) {
         double2 wv[E2];
         bool in[E2];
#pragma unroll
         for (int e = 0; e < E2; e++) {
            const size_t p = p0 + (size_t)e * kKThreads;
            in[e] = p < n2;
            wv[e] = in[e] ? w2[p] : make_double2(0.0, 0.0);
         }
         int j = 0;
         for (; j + 4 <= m; j += 4) {
            double2 z[4][E2];
#pragma unroll
            for (int q = 0; q < 4; q++)
#pragma unroll
               for (int e = 0; e < E2; e++)
                  z[q][e] = in[e] ? reinterpret_cast<const double2*>(Z + (size_t)(j + q) * n)[p0 + (size_t)e * kKThreads]
                                  : make_double2(0.0, 0.0);
#pragma unroll
            for (int q = 0; q < 4; q++) {
               const double hj = s_h[j + q];
#pragma unroll
               for (int e = 0; e < E2; e++) {
                  wv[e].x = fma(-hj, z[q][e].x, wv[e].x);
                  wv[e].y = fma(-hj, z[q][e].y, wv[e].y);
               }
            }
         }
         for (; j < m; j++) {
            const double hj = s_h[j];
#pragma unroll
            for (int e = 0; e < E2; e++) {
               const double2 z = in[e] ? reinterpret_cast<const double2*>(Z + (size_t)j * n)[p0 + (size_t)e * kKThreads]
                                       : make_double2(0.0, 0.0);
               wv[e].x = fma(-hj, z.x, wv[e].x);
               wv[e].y = fma(-hj, z.y, wv[e].y);
            }
         }
#pragma unroll
         for (int e = 0; e < E2; e++) {
            if (in[e]) w2[p0 + (size_t)e * kKThreads] = wv[e];
            acc = fma(wv[e].y, wv[e].y, fma(wv[e].x, wv[e].x, acc));
         }
      }
      acc = block_sum0<kKThreads>(acc);
      double tot;
      if (grid_total<kKThreads>(acc, part, ticket, &tot) && threadIdx.x == 0) *out = tot;
      return;
   }
   const size_t stride = (size_t)gridDim.x * kKThreads * kKEPT;
   for (size_t i0 = (size_t)blockIdx.x * kKThreads * kKEPT + threadIdx.x; i0 < n; i0 += stride) {
      double wv[kKEPT];
      bool in[kKEPT];
#pragma unroll
      for (int e = 0; e < kKEPT; e++) {
         const size_t i = i0 + (size_t)e * kKThreads;
         in[e] = i < n;
         wv[e] = in[e] ? w[i] : 0.0;
      }
      int j = 0;
      for (; j + 4 <= m; j += 4) {
         double z[4][kKEPT];
#pragma unroll
         for (int q = 0; q < 4; q++)
#pragma unroll
            for (int e = 0; e < kKEPT; e++) z[q][e] = in[e] ? Z[(size_t)(j + q) * n + i0 + (size_t)e * kKThreads] : 0.0;
#pragma unroll
         for (int q = 0; q < 4; q++) {
            const double hj = s_h[j + q];
#pragma unroll
            for (int e = 0; e < kKEPT; e++) wv[e] = fma(-hj, z[q][e], wv[e]);
         }
      }
      for (; j < m; j++) {
         const double hj = s_h[j];
#pragma unroll
         for (int e = 0; e < kKEPT; e++)
            wv[e] = fma(-hj, in[e] ? Z[(size_t)j * n + i0 + (size_t)e * kKThreads] : 0.0, wv[e]);
      }
#pragma unroll
      for (int e = 0; e < kKEPT; e++) {
         const size_t i = i0 + (size_t)e * kKThreads;
         if (i < n) w[i] = wv[e];
         acc = fma(wv[e], wv[e], acc);
      }
   }
   acc = block_sum0<kKThreads>(acc);
   double tot;
   if (grid_total<kKThreads>(acc, part, ticket, &tot) && threadIdx.x == 0) *out = tot;
}

// ---- DCGS2 (delayed classical Gram-Schmidt with re-orthogonalisation; FGMRES ortho 2) ----------------------
// Sweep 1 of a step: S[k] = (v_k, a) and T[k] = (v_k, b) for the m basis columns (the last of them is a itself,
// the step's provisional column) -- the previous column's second pass and this column's first pass read the
// basis once together.  Partials: part[blk ldp + k] (S), part[blk ldp + m + k] (T); b may be null.
constexpr int kBD2 = 16;
__global__ __launch_bounds__(kBDThreads) void k_block_dots_ab(const double* __restrict__ a, const double* __restrict__ b,
                                                              const double* __restrict__ V, size_t n, int m,
                                                              double* __restrict__ part, int ldp)
{
   __shared__ double s[kBDThreads / 64][2 * kBD2];
   const int g0 = blockIdx.y * kBD2;
   const int cnt = min(kBD2, m - g0);
   double sa[kBD2], sb[kBD2];
#pragma unroll
   for (int j = 0; j < kBD2; j++) sa[j] = sb[j] = 0.0;
   const size_t stride = (size_t)gridDim.x * kBDThreads;
   for (size_t r = (size_t)blockIdx.x * kBDThreads + threadIdx.x; r < n; r += stride) {
      const double ar = a[r];
      const double br = b ? b[r] : 0.0;
      double v[kBD2];
#pragma unroll
      for (int j = 0; j < kBD2; j++) v[j] = j < cnt ? V[(size_t)(g0 + j) * n + r] : 0.0;
#pragma unroll
      for (int j = 0; j < kBD2; j++) {
         sa[j] = fma(v[j], ar, sa[j]);
         sb[j] = fma(v[j], br, sb[j]);
      }
   }
   const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
   for (int j = 0; j < kBD2; j++) {
      double x = sa[j], y = sb[j];
      for (int off = 32; off > 0; off >>= 1) {
         x += __shfl_down(x, off, 64);
         y += __shfl_down(y, off, 64);
      }
      if (lane == 0) {
         s[wave][j] = x;
         s[wave][kBD2 + j] = y;
      }
   }
   __syncthreads();
   if (threadIdx.x < 2 * kBD2) {
      const int j = threadIdx.x % kBD2, which = threadIdx.x / kBD2;
      if (j < cnt && (which == 0 || b)) {
         double t = 0.0;
#pragma unroll
         for (int q = 0; q < kBDThreads / 64; q++) t += s[q][threadIdx.x];
         part[(size_t)blockIdx.x * ldp + which * m + g0 + j] = t;
      }
   }
}

// Update of a step (row-parallel, basis columns read once): column j is finalised in place,
// v_j = (V[:, j] - sum_{k<j} s_k v_k) / alpha, and w becomes the next provisional column's numerator
// u = w / alpha - sum_{k<j} g_k v_k - g_j v_j; *out = ||u||^2.  coef = [s (j) | g (j + 1) | 1 / alpha].
__global__ __launch_bounds__(kKThreads) void k_dcgs2_update(double* __restrict__ V, double* __restrict__ w, size_t n,
                                                            int j, const double* __restrict__ coef,
                                                            double* __restrict__ part,
                                                            unsigned int* __restrict__ ticket,
                                                            double* __restrict__ out)
{
   extern __shared__ double s_c[];
   for (int k = threadIdx.x; k < 2 * j + 2; k += kKThreads) s_c[k] = coef[k];
   __syncthreads();
   const double* s_s = s_c;
   const double* s_g = s_c + j;
   const double ia = s_c[2 * j + 1];
   double acc = 0.0;
   const size_t stride = (size_t)gridDim.x * kKThreads * kKEPT;
   double* vjcol = V + (size_t)j * n;
   for (size_t i0 = (size_t)blockIdx.x * kKThreads * kKEPT + threadIdx.x; i0 < n; i0 += stride) {
      double v0[kKEPT], u[kKEPT];
      bool in[kKEPT];
#pragma unroll
      for (int e = 0; e < kKEPT; e++) {
         const size_t i = i0 + (size_t)e * kKThreads;
         in[e] = i < n;
         v0[e] = in[e] ? vjcol[i] : 0.0;
         u[e] = in[e] ? w[i] * ia : 0.0;
      }
      int k = 0;
      for (; k + 4 <= j; k += 4) {
         double z[4][kKEPT];
#pragma unroll
         for (int q = 0; q < 4; q++)
#pragma unroll
            for (int e = 0; e < kKEPT; e++) z[q][e] = in[e] ? V[(size_t)(k + q) * n + i0 + (size_t)e * kKThreads] : 0.0;
#pragma unroll
         for (int q = 0; q < 4; q++) {
            const double sk = s_s[k + q], gk = s_g[k + q];
#pragma unroll
            for (int e = 0; e < kKEPT; e++) {
               v0[e] = fma(-sk, z[q][e], v0[e]);
               u[e] = fma(-gk, z[q][e], u[e]);
            }
         }
      }
      for (; k < j; k++) {
         const double sk = s_s[k], gk = s_g[k];
#pragma unroll
         for (int e = 0; e < kKEPT; e++) {
            const double z = in[e] ? V[(size_t)k * n + i0 + (size_t)e * kKThreads] : 0.0;
            v0[e] = fma(-sk, z, v0[e]);
            u[e] = fma(-gk, z, u[e]);
         }
      }
      const double gj = s_g[j];
#pragma unroll
      for (int e = 0; e < kKEPT; e++) {
         const size_t i = i0 + (size_t)e * kKThreads;
         const double vj = v0[e] * ia;
         u[e] = fma(-gj, vj, u[e]);
         if (in[e]) {
            vjcol[i] = vj;
            w[i] = u[e];
         }
         acc = fma(u[e], u[e], acc);
      }
   }
   acc = block_sum0<kKThreads>(acc);
   double tot;
   if (grid_total<kKThreads>(acc, part, ticket, &tot) && threadIdx.x == 0) *out = tot;
}

// a *= 1 / sqrt(*nrm2) (the provisional column's normalisation, without a host round trip).  A lucky breakdown
// (u = 0 exactly, e.g. A = I) leaves the zero column as it is: 1 / sqrt(0) would fill it with NaN, and the host
// finishes the Hessenberg column with H(j, j-1) = 0 (convergence)
__global__ void k_scale_rnorm(double* __restrict__ a, size_t n, const double* __restrict__ nrm2)
{
   const double f = *nrm2 > 0.0 ? 1.0 / sqrt(*nrm2) : 0.0;
   for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] *= f;
}

int egrid(size_t n)
{
   size_t g = (n + 255) / 256;
   return (int)std::max<size_t>(1, std::min<size_t>(g, 4096));
}

// device scratch of the Krylov solvers: two reduction pairs, device scalars, pinned read-back
struct KScratch {
   static constexpr int kScal = 4096;
   double *part = nullptr, *part2 = nullptr, *scal = nullptr, *hscal = nullptr, *coef = nullptr;
   double* hcoef = nullptr;  // pinned staging of per-step coefficients (DCGS2)
   double* bpart = nullptr;  // block Gram-Schmidt partials [kBDMaxBlocks][kScal]
   unsigned int *ticket = nullptr, *ticket2 = nullptr;
   double* lz_part = nullptr;          // k_lanczos_local: 4 partial arrays
   unsigned int* lz_ticket = nullptr;  // k_lanczos_local: 3 ticket arrays
   int lz_occ = -1;                    // resident k_lanczos_local workgroups
   int* chain = nullptr;      // k_mgs_chain: [1] error word
   int* hchain_err = nullptr; // pinned read-back of the error word
   int chain_occ = -1;        // resident workgroups of k_mgs_chain per CU x CUs (0: unusable)
   int wide_occ[6] = {-1, -1, -1, -1, -1, -1};  // the same for k_mgs_wide<1024, kWideS[x]>
   // set once a one-launch sweep's wait has given up in this process: the sweeps then run as launch chains
   // (k_gs_step / block_gs), which cannot wait on other workgroups
   bool chain_off = false;
   // after a wait gave up: clear the error word and every ticket array the one-launch kernels count on, so
   // later reductions start from zero, and stop using those kernels (chain_off)
   void chain_reset()
   {
      (void)hipDeviceSynchronize();
      if (chain) (void)hipMemset(chain, 0, sizeof(int) * 2);
      if (ticket) (void)hipMemset(ticket, 0, sizeof(unsigned int) * kTicketWords);
      if (lz_ticket) (void)hipMemset(lz_ticket, 0, sizeof(unsigned int) * 3 * kTicketWords);
      if (hchain_err) *hchain_err = 0;
      chain_off = true;
   }
   unsigned int* bd_tickets = nullptr;  // k_block_dots<true>: one ticket array per column group
   int ensure_bpart()
   {
      if (!bpart) NFFT4GP_HIP_CHECK(hipMalloc((void**)&bpart, sizeof(double) * kBDMaxBlocks * kScal));
      if (!bd_tickets) {
         const size_t words = (size_t)(kScal / kBD + 1) * kTicketWords;
         NFFT4GP_HIP_CHECK(hipMalloc((void**)&bd_tickets, sizeof(unsigned int) * words));
         NFFT4GP_HIP_CHECK(hipMemset(bd_tickets, 0, sizeof(unsigned int) * words));
      }
      return 0;
   }
   int ensure()
   {
      if (part) return 0;
      NFFT4GP_HIP_CHECK(hipMalloc((void**)&part, sizeof(double) * kKMaxBlocks));
      NFFT4GP_HIP_CHECK(hipMalloc((void**)&part2, sizeof(double) * kKMaxBlocks));
      NFFT4GP_HIP_CHECK(hipMalloc((void**)&scal, sizeof(double) * kScal));
      NFFT4GP_HIP_CHECK(hipMalloc((void**)&coef, sizeof(double) * kScal));
      NFFT4GP_HIP_CHECK(hipMalloc((void**)&ticket, sizeof(unsigned int) * kTicketWords));
      NFFT4GP_HIP_CHECK(hipMalloc((void**)&ticket2, sizeof(unsigned int) * kTicketWords));
      NFFT4GP_HIP_CHECK(hipMemset(ticket, 0, sizeof(unsigned int) * kTicketWords));
      NFFT4GP_HIP_CHECK(hipMemset(ticket2, 0, sizeof(unsigned int) * kTicketWords));
      NFFT4GP_HIP_CHECK(hipHostMalloc((void**)&hscal, sizeof(double) * kScal));
      NFFT4GP_HIP_CHECK(hipHostMalloc((void**)&hcoef, sizeof(double) * kScal));
      return 0;
   }
   int ensure_chain()
   {
      if (ensure()) return -1;
      if (!chain) {
         NFFT4GP_HIP_CHECK(hipMalloc((void**)&chain, sizeof(int) * 2));
         NFFT4GP_HIP_CHECK(hipMemset(chain, 0, sizeof(int) * 2));
         NFFT4GP_HIP_CHECK(hipHostMalloc((void**)&hchain_err, sizeof(int)));
         *hchain_err = 0;
      }
      if (!lz_part) {
         NFFT4GP_HIP_CHECK(hipMalloc((void**)&lz_part, sizeof(double) * 4 * kKMaxBlocks));
         NFFT4GP_HIP_CHECK(hipMalloc((void**)&lz_ticket, sizeof(unsigned int) * 3 * kTicketWords));
         NFFT4GP_HIP_CHECK(hipMemset(lz_ticket, 0, sizeof(unsigned int) * 3 * kTicketWords));
      }
      if (lz_occ < 0) {
         int dev = 0, occ = 0;
         hipDeviceProp_t prop;
         lz_occ = 0;
         if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess &&
             hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_lanczos_local<1024, 4>, 1024, 0) == hipSuccess)
            lz_occ = occ * prop.multiProcessorCount;
      }
      if (chain_occ < 0) {
         int dev = 0, occ = 0;
         hipDeviceProp_t prop;
         chain_occ = 0;
         if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess &&
             hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_mgs_chain<1024, 4>, 1024, 0) == hipSuccess)
            chain_occ = occ * prop.multiProcessorCount;
         for (int x = 0; x < 6; x++) {
            wide_occ[x] = 0;
            occ = 0;
            if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess &&
                hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, mgs_wide_fn(kWideS[x]), 1024, 0) == hipSuccess)
               wide_occ[x] = occ * prop.multiProcessorCount;
         }
      }
      return 0;
   }
};
KScratch g_k;

struct Ctx {
   hipStream_t s;
   size_t n;
   // row-sharded vectors (a distributed operator's rows): every inner product is a local partial, summed
   // in place over the ranks on the stream before anything reads it; NULL for whole vectors
   Comm* comm = nullptr;
   bool lz_launched = false;  // the last lanczos_local call launched k_lanczos_local
   int red(double* d, int count)
   {
      return comm ? comm->allreduce(d, (size_t)count, s) : 0;
   }
   // the MGS sweep's form for this n (comm == NULL): 0 k_mgs_chain (one pass of 4 elements per thread covers n with
   // a resident grid), S > 0 k_mgs_wide<1024, S> on *grid workgroups (the smallest S of kWideS whose resident grid
   // covers n in S passes), -1 neither (the per-projection chain on its usual grid)
   int mgs_form(unsigned* grid)
   {
      *grid = (unsigned)std::max<size_t>(1, std::min<size_t>((n + 4095) / 4096, kKMaxBlocks));
      if (comm || g_k.ensure_chain()) return -1;
      if ((size_t)*grid * 4096 >= n && (int)*grid <= g_k.chain_occ) return 0;
      const char* e = getenv("NFFT4GP_AMD_MGS_WIDE");
      if (e && atoi(e) == 0) return -1;
      for (int x = 0; x < 6; x++) {
         const size_t per = (size_t)kWideS[x] * 4096;
         const size_t g = (n + per - 1) / per;
         if (g <= (size_t)g_k.wide_occ[x] && g <= (size_t)kKMaxBlocks) {
            *grid = (unsigned)g;
            return kWideS[x];
         }
      }
      return -1;
   }
   // w -= h u (u optional), *out = (w, v) or ||w||^2; grid 0: the usual grid, else that many workgroups
   // (grid-stride over n: the MGS sweep's grid when k_mgs_wide serves this n, so the two forms are bitwise equal)
   int gs(double* w, const double* u, const double* hprev, const double* v, double* out, unsigned grid_in = 0)
   {
      // 1024 threads x 4 elements: a quarter of the 256-thread partials for the last block to add (8.35 us per
      // projection at n = 1e6 against 9.16; 1024 x 8: 10.7, 512 x 4: 8.49 -- round 3, tools/ab_gs.sh, removed)
      const unsigned grid =
          grid_in ? grid_in : (unsigned)std::max<size_t>(1, std::min<size_t>((n + 4095) / 4096, kKMaxBlocks));
      hipLaunchKernelGGL((k_gs_step<1024, 4>), dim3(grid), dim3(1024), 0, s, w, u, hprev, v, n, g_k.part, g_k.ticket,
                         out);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return red(out, 1);
   }
   // the MGS sweep of an FGMRES step (w against V[0..i), then ||w||^2) into hd[0..i] in one launch when the grid
   // fits (k_mgs_chain); returns 1 when it does not (the caller runs the k_gs_step chain)
   int mgs_chain(double* w, const double* V, int i, double* hd)
   {
      if (comm || g_k.ensure_chain()) return comm ? 1 : -1;
      unsigned grid = 0;
      const int form = mgs_form(&grid);
      const char* e = getenv("NFFT4GP_AMD_MGS_CHAIN");
      const bool off = e && atoi(e) == 0;
      if (off || g_k.chain_off || form < 0) return 1;
      NFFT4GP_HIP_CHECK(hipMemsetAsync(hd, 0xFF, sizeof(double) * (i + 1), s));  // kChainUnset
      if (form > 0)
         hipLaunchKernelGGL(mgs_wide_fn(form), dim3(grid), dim3(1024), 0, s, w, V, n, i, hd, g_k.part, g_k.ticket,
                            g_k.chain + 1);
      else
         hipLaunchKernelGGL((k_mgs_chain<1024, 4>), dim3(grid), dim3(1024), 0, s, w, V, n, i, hd, g_k.part,
                            g_k.ticket, g_k.chain + 1);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      // the error word comes back with the step's scalars (the caller's read synchronises)
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(g_k.hchain_err, g_k.chain + 1, sizeof(int), hipMemcpyDeviceToHost, s));
      return 0;
   }
   // mgs2's local pass (block_gs(w, Vl, Zl, ml, h, 1)) in one launch where the grid fits (k_lanczos_local);
   // otherwise block_gs.  NFFT4GP_AMD_LANCZOS_LOCAL=0 keeps block_gs.
   int lanczos_local(double* w, const double* Vl, const double* Zl, int ml, double* h)
   {
      const unsigned grid = (unsigned)std::max<size_t>(1, std::min<size_t>((n + 4095) / 4096, kKMaxBlocks));
      const char* e = getenv("NFFT4GP_AMD_LANCZOS_LOCAL");
      lz_launched = false;
      if (comm || (e && atoi(e) == 0) || ml < 1 || ml > 2 || g_k.ensure_chain() || (size_t)grid * 4096 < n ||
          (int)grid > g_k.lz_occ || g_k.chain_off)
         return block_gs(w, Vl, Zl, ml, h, 1);
      lz_launched = true;
      NFFT4GP_HIP_CHECK(hipMemsetAsync(h, 0xFF, sizeof(double) * (ml + 2), s));  // kChainUnset
      hipLaunchKernelGGL((k_lanczos_local<1024, 4>), dim3(grid), dim3(1024), 0, s, w, Vl, Zl, Zl == Vl ? 1 : 0, n,
                         ml, h, g_k.lz_part, g_k.lz_ticket, g_k.chain + 1);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(g_k.hchain_err, g_k.chain + 1, sizeof(int), hipMemcpyDeviceToHost, s));
      return 0;
   }
   // after the read that follows mgs_chain: did a wait give up?  Then this solve fails, the error word and the
   // tickets are reset and later sweeps in this process run as k_gs_step chains (KScratch::chain_reset)
   int chain_failed()
   {
      if (*g_k.hchain_err) {
         fprintf(stderr, "nfft4gp_amd: FGMRES: the one-launch MGS sweep's wait gave up\n");
         g_k.chain_reset();
         return 1;
      }
      return 0;
   }
   // after the read that follows lanczos_local: did this step's launch give up waiting?  (same reset)
   int lanczos_local_failed()
   {
      if (lz_launched && *g_k.hchain_err) {
         fprintf(stderr, "nfft4gp_amd: Lanczos: the one-launch local pass's wait gave up\n");
         g_k.chain_reset();
         return 1;
      }
      return 0;
   }
   int read(const double* d, int count, double* h)
   {
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(g_k.hscal, d, sizeof(double) * count, hipMemcpyDeviceToHost, s));
      NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
      memcpy(h, g_k.hscal, sizeof(double) * count);
      return 0;
   }
   double dot(const double* a, const double* b)
   {
      if (gs(const_cast<double*>(a), nullptr, nullptr, b, g_k.scal + KScratch::kScal - 1)) return NAN;
      double v;
      if (read(g_k.scal + KScratch::kScal - 1, 1, &v)) return NAN;
      return v;
   }
   double norm(const double* a) { return std::sqrt(dot(a, a)); }
   // k_block_reduce folded into k_block_dots (NFFT4GP_AMD_BD_FOLD=0: two launches)
   static bool fold_reduce()
   {
      const char* e = getenv("NFFT4GP_AMD_BD_FOLD");
      return !(e && atoi(e) == 0);
   }
   // the block passes' 16-byte row pairs: n even and every vector 16-byte aligned (then so is every column);
   // NFFT4GP_AMD_BD_VEC=0 keeps one row per load
   bool bd_vec(const void* a, const void* b, const void* c2) const
   {
      const char* e = getenv("NFFT4GP_AMD_BD_VEC");
      if (e && atoi(e) == 0) return false;
      return n % 2 == 0 && (((uintptr_t)a | (uintptr_t)b | (uintptr_t)c2) & 15) == 0;
   }
   // h[0..mc) = V^T w (column m, when mc = m + 1, is w itself: h[m + 1]) in k_block_dots (+ k_block_reduce
   // unless folded); after / before: the DGKS gate of a second pass
   void block_dots(const double* w, const double* V, int m, int with_norm, double* h, bool vec,
                   const double* after = nullptr, const double* before = nullptr)
   {
      const int nb = bd_grid(n);
      const int mc = m + with_norm;
      const dim3 grid(nb, (mc + kBD - 1) / kBD);
      if (fold_reduce()) {
         if (vec)
            hipLaunchKernelGGL((k_block_dots<true, 2>), grid, dim3(kBDThreads), 0, s, w, V, n, m, with_norm, g_k.bpart,
                               KScratch::kScal, after, before, h, g_k.bd_tickets);
         else
            hipLaunchKernelGGL((k_block_dots<true, 1>), grid, dim3(kBDThreads), 0, s, w, V, n, m, with_norm, g_k.bpart,
                               KScratch::kScal, after, before, h, g_k.bd_tickets);
      } else {
         if (vec)
            hipLaunchKernelGGL((k_block_dots<false, 2>), grid, dim3(kBDThreads), 0, s, w, V, n, m, with_norm,
                               g_k.bpart, KScratch::kScal, after, before, (double*)nullptr, (unsigned int*)nullptr);
         else
            hipLaunchKernelGGL((k_block_dots<false, 1>), grid, dim3(kBDThreads), 0, s, w, V, n, m, with_norm,
                               g_k.bpart, KScratch::kScal, after, before, (double*)nullptr, (unsigned int*)nullptr);
         hipLaunchKernelGGL(k_block_reduce, dim3((mc + 63) / 64), dim3(1024), 0, s, g_k.bpart, nb, KScratch::kScal, mc,
                            m, h);
      }
   }
   // w -= Z h (m columns), *out = ||w||^2; after / before / flag: the DGKS gate of a second pass
   void block_update(double* w, const double* Z, int m, const double* h, double* out, bool vec,
                     const double* after = nullptr, const double* before = nullptr, double* flag = nullptr)
   {
      if (vec)
         hipLaunchKernelGGL(k_block_update<2>, dim3(kgrid(n)), dim3(kKThreads), sizeof(double) * m, s, w, Z, n, h, m,
                            g_k.part, g_k.ticket, out, after, before, flag);
      else
         hipLaunchKernelGGL(k_block_update<1>, dim3(kgrid(n)), dim3(kKThreads), sizeof(double) * m, s, w, Z, n, h, m,
                            g_k.part, g_k.ticket, out, after, before, flag);
   }
   // one classical Gram-Schmidt pass: h[0..m) = V^T w, w -= Z h, h[m] = ||w||^2 afterwards (device
   // scalars); with_norm: also h[m + 1] = ||w||^2 before the update (from the dot pass)
   int block_gs(double* w, const double* V, const double* Z, int m, double* h, int with_norm = 0)
   {
      if (m <= 0 || m + 2 > KScratch::kScal) return -1;
      if (g_k.ensure_bpart()) return -1;
      const bool vec = bd_vec(w, V, Z);
      // h[m], h[m + 1] take part in the all-reduce below even when this pass does not write them
      if (comm) NFFT4GP_HIP_CHECK(hipMemsetAsync(h + m, 0, sizeof(double) * 2, s));
      block_dots(w, V, m, with_norm, h, vec);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      if (red(h, m + 2)) return -1;  // the projections and the norm before them, summed over the row shards
      block_update(w, Z, m, h, h + m, vec);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return red(h + m, 1);
   }
   // CGS2 against the basis V (m columns) with one host read: pass 1 (dots with the norm before, update with
   // the norm after), then pass 2 with every launch gated on the device by the DGKS test on pass 1's norms, so
   // the host does not wait between the passes.  h: [0, m) pass-1 projections, h[m] ||w||^2 after pass 1,
   // h[m + 1] before it, [m + 2, 2m + 2) pass-2 projections, h[2m + 2] ||w||^2 after pass 2, h[2m + 3] the
   // decision (1 / 0); pass-2 entries are meaningful only when the decision is 1
   int block_cgs2(double* w, const double* V, int m, double* h)
   {
      if (m <= 0 || 2 * m + 4 > KScratch::kScal) return -1;
      if (block_gs(w, V, V, m, h, 1)) return -1;
      const bool vec = bd_vec(w, V, V);
      const double* after = h + m;
      const double* before = h + m + 1;
      block_dots(w, V, m, 0, h + m + 2, vec, after, before);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      if (red(h + m + 2, m)) return -1;
      block_update(w, V, m, h + m + 2, h + 2 * m + 2, vec, after, before, h + 2 * m + 3);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return red(h + 2 * m + 2, 1);
   }
   // DCGS2 sweep 1: out[0, m) = V(:, 0..m)^T a, out[m, 2m) = V(:, 0..m)^T b (b optional; column m - 1 is a)
   int dots_ab(const double* a, const double* b, const double* V, int m, double* out)
   {
      if (m <= 0 || 2 * m > KScratch::kScal) return -1;
      if (g_k.ensure_bpart()) return -1;
      const int nb = bd_grid(n);
      hipLaunchKernelGGL(k_block_dots_ab, dim3(nb, (m + kBD2 - 1) / kBD2), dim3(kBDThreads), 0, s, a, b, V, n, m,
                         g_k.bpart, KScratch::kScal);
      const int mc = b ? 2 * m : m;
      hipLaunchKernelGGL(k_block_reduce, dim3((mc + 63) / 64), dim3(1024), 0, s, g_k.bpart, nb, KScratch::kScal, mc,
                         mc, out);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return red(out, mc);
   }
   // DCGS2 update (k_dcgs2_update) with the host's coefficients [s | g | 1/alpha], then w /= ||w|| on the
   // device; *nrm2 = ||w||^2 before that scaling
   int dcgs2_update(double* V, double* w, int j, const std::vector<double>& coef, double* nrm2)
   {
      if (coef.size() > (size_t)KScratch::kScal) return -1;
      // pinned staging: the previous step's copy has run (the host read this step's sweep after it)
      memcpy(g_k.hcoef, coef.data(), sizeof(double) * coef.size());
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(g_k.coef, g_k.hcoef, sizeof(double) * coef.size(), hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(k_dcgs2_update, dim3(kgrid(n)), dim3(kKThreads), sizeof(double) * (2 * j + 2), s, V, w, n, j,
                         g_k.coef, g_k.part, g_k.ticket, nrm2);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      if (red(nrm2, 1)) return -1;
      hipLaunchKernelGGL(k_scale_rnorm, dim3(egrid(n)), dim3(256), 0, s, w, n, (const double*)nrm2);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return 0;
   }
   void scale(double* a, double* b, double f)
   {
      hipLaunchKernelGGL(k_scale2, dim3(egrid(n)), dim3(256), 0, s, a, b, n, f);
   }
   int combine(double* x, const double* B, int m, const double* c)
   {
      if (m <= 0) return 0;
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(g_k.coef, c, sizeof(double) * m, hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(k_combine, dim3(egrid(n)), dim3(256), 0, s, x, B, n, n, g_k.coef, m);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return 0;
   }
   int copy(double* dst, const double* src)
   {
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(dst, src, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
      return 0;
   }
};

double* rel_hist(int len)
{
   return (double*)calloc((size_t)std::max(1, len), sizeof(double));
}

template <class T>
int dmalloc(T** p, size_t count)
{
   NFFT4GP_HIP_CHECK(hipMalloc((void**)p, sizeof(T) * std::max<size_t>(1, count)));
   return 0;
}

// host tridiagonal eigensolve: dstev 'V' (ascending eigenvalues, eigenvectors in columns of TV)
int tridiag_eig(int m, const double* d, const double* e, std::vector<double>& w, std::vector<double>& V)
{
   std::vector<double> A((size_t)m * m, 0.0);
   for (int i = 0; i < m; i++) {
      A[(size_t)i * m + i] = d[i];
      if (i + 1 < m) {
         A[(size_t)i * m + i + 1] = e[i];
         A[(size_t)(i + 1) * m + i] = e[i];
      }
   }
   return sym_eig_host(A, m, w, V);
}

}  // namespace

namespace nfft4gp_amd {

// FGMRES orthogonalisation: 0 = the reference's modified Gram-Schmidt (Nfft4GPModifiedGS, one launch per
// basis vector), 1 = block classical Gram-Schmidt passes (the Lanczos re-orthogonalisation's kernels: two
// launches per pass whatever its length), a second pass when the DGKS test asks for it -- Nfft4GPAmdSetFgmresOrtho
int g_fgmres_ortho = -1;
long long g_fgmres_second_passes = 0;  // DGKS re-orthogonalisations taken (ortho 1), Nfft4GPAmdFgmresStats
int fgmres_ortho()
{
   if (g_fgmres_ortho < 0) {
      const char* e = getenv("NFFT4GP_AMD_FGMRES_ORTHO");
      g_fgmres_ortho = (e && (atoi(e) == 1 || atoi(e) == 2)) ? atoi(e) : 0;
   }
   return g_fgmres_ortho;
}

// ---- FGMRES with DCGS2 (ortho 2) ------------------------------------------------------------------------------
// The reference's FGMRES (fgmres.c:3-252: the same Givens recurrence, breakdown exit, restart and reporting)
// with the Arnoldi basis orthogonalised by delayed CGS2 (Swirydowicz, Langou, Ananthan, Yang, Thomas 2020):
// step j multiplies the provisional column v_j^0 = u_j / beta_j (once orthogonalised), then ONE sweep forms
// s = V^T v_j^0 (v_j's second pass, delayed) and t = V^T w (w = A v_j^0), and ONE update sweep finalises
// v_j = (v_j^0 - V s) / alpha, alpha^2 = (v_j^0, v_j^0) - |s|^2, and forms the next provisional column
// u = A v_j - V c through the Arnoldi relation A v_j = (w - V H s) / alpha, which gives
// u = (w - V_{<j} t) / alpha - ((v_j^0, w) - s.t) / alpha^2 v_j.  Column j - 1 of H becomes final at step j:
// H(<j, j-1) += beta_j s, H(j, j-1) = beta_j alpha, so the Givens rotation and the residual of iteration j are
// applied one step late (one extra operator application per cycle).  Mathematically CGS2 with a second pass at
// every step; the basis is read twice per step instead of up to four times.
// With a (flexible, right) preconditioner M (fgmres.c:140-146: z = M^-1 v, w = A z) the provisional column's
// z_j^0 = M^-1 v_j^0 is kept, w = A z_j^0, and the finalised direction z_j = (z_j^0 - sum_{k<j} s_k z_k) / alpha
// satisfies A z_j = (w - V H s) / alpha: the same Arnoldi relation, so V, H and the sweeps are unchanged.  z_j is
// never formed: x += Z y is applied as Z^0 c, c from y by the triangular recurrence of the s and alpha (combine).
int fgmres_dcgs2_dev(Callbacks& cb, double* x, const double* rhs, int kdim, int maxits, int atol, double tol,
                     double* prel_res, double** prel_res_v, int* piter, int print_level)
{
   const size_t n = cb.n;
   Ctx c{current_stream(), n, cb.comm};
   const double EPS = DBL_EPSILON;
   if (cb.n_global == 0) {
      *prel_res = 0.0;
      *piter = 0;
      *prel_res_v = rel_hist(1);
      return 0;
   }
   const double normb = c.norm(rhs);
   if (normb < EPS) {
      NFFT4GP_HIP_CHECK(hipMemsetAsync(x, 0, sizeof(double) * n, c.s));
      *prel_res = 0.0;
      *piter = 0;
      *prel_res_v = rel_hist(1);
      return 0;
   }
   const int kmax = KScratch::kScal / 2 - 2;
   if (kdim > kmax) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPSolverFgmres: restart dimension %d above %d\n", kdim, kmax);
      return -1;
   }
   double *V = nullptr, *Z = nullptr;  // Z: the provisional directions z_j^0 = M^-1 v_j^0 (preconditioned only)
   double* rel = nullptr;
   auto cleanup = [&]() {
      (void)hipStreamSynchronize(c.s);
      (void)hipFree(V);
      (void)hipFree(Z);
   };
   // every error exit: the basis, Z and the history are released
   auto fail = [&]() -> int {
      free(rel);
      rel = nullptr;
      cleanup();
      return -1;
   };
   if (dmalloc(&V, n * (size_t)(kdim + 1)) || (cb.prec && dmalloc(&Z, n * (size_t)(kdim + 1)))) return fail();
   // Hr: the unrotated Hessenberg (the Arnoldi relation), H: the rotated one (fgmres.c's H)
   std::vector<double> Hr((size_t)kdim * (kdim + 1), 0.0), H((size_t)kdim * (kdim + 1), 0.0), cs(kdim), sn(kdim),
       rs(kdim + 1);
   // the delayed second pass of each column (s_j, alpha_j): the recurrence from y to Z^0's coefficients
   std::vector<std::vector<double>> spass(kdim + 1);
   std::vector<double> alph(kdim + 1, 1.0), ccoef;
   double* v = V;
   c.copy(v, rhs);
   if (cb.apply(-1.0, x, 1.0, v)) return fail();
   double normr = c.norm(v);
   if (normr < EPS) {
      *prel_res = 0.0;
      *piter = 0;
      *prel_res_v = rel_hist(1);
      cleanup();
      return 0;
   }
   const double tolr = atol ? tol : tol * normb;
   rel = rel_hist(maxits + 1);
   rel[0] = normr / normb;
   int iter = 0, i = 0;
   if (print_level > 0) {
      printf("--------------------------------------------------------------------------------\n");
      printf("Start FlexGMRES(%d)\n", kdim);
      printf("Residual Tol: %e\nMax number of inner iterations: %d\n", tolr, maxits);
      printf("--------------------------------------------------------------------------------\n");
      printf("Step    Residual norm  Relative res.  Convergence Rate\n");
      printf("%5d   %8e   %8e   N/A\n", 0, normr, rel[0]);
   }
   double* dsc = g_k.scal;  // device scalars of step j (m = j + 1): [0, 2m) the sweep, [2m] ||u_j||^2
   std::vector<double> hh, coef;
   bool broke = false, converged = false;
   if (2 * (kdim + 1) + 1 > KScratch::kScal) return fail();
   while (iter < maxits) {
      rs[0] = normr;
      c.scale(V, nullptr, 1.0 / normr);
      i = 0;                 // final columns of H in this cycle
      double beta = 0.0;     // ||u_j|| of the provisional column j (j >= 1)
      for (int j = 0;; j++) {
         // step j: column j of V is provisional (j >= 1); column j - 1 of H is completed here
         const bool more = j < kdim && iter + (j > 0 ? 1 : 0) < maxits;  // will column j get a first pass?
         double* vj = V + (size_t)j * n;
         double* w = V + (size_t)(j + 1) * n;
         if (more) {
            if (cb.prec) {
               double* zj = Z + (size_t)j * n;  // z_j^0 = M^-1 v_j^0, w = A z_j^0
               if (cb.solve(zj, vj) || cb.apply(1.0, zj, 0.0, w)) return fail();
            } else if (cb.apply(1.0, vj, 0.0, w)) {
               return fail();
            }
         }
         const int m = j + 1;
         hh.assign(2 * m + 1, 0.0);
         if (c.dots_ab(vj, more ? w : nullptr, V, m, dsc)) return fail();
         if (c.read(dsc, 2 * m + 1, hh.data())) return fail();  // (T is stale when !more)
         if (j > 0) beta = std::sqrt(hh[2 * m]);
         // the delayed second pass of column j: s = hh[0, j), omega = hh[j]
         double alpha = 1.0, ss = 0.0;
         if (j > 0) {
            for (int k = 0; k < j; k++) ss += hh[k] * hh[k];
            const double a2 = hh[j] - ss;
            alpha = a2 > 0.0 ? std::sqrt(a2) : std::sqrt(hh[j]);
            spass[j].assign(hh.begin(), hh.begin() + j);
            alph[j] = alpha;
            // column j - 1 of H is final: H(<j, j-1) += beta s, H(j, j-1) = beta alpha
            double* Hrc = Hr.data() + (size_t)(j - 1) * (kdim + 1);
            for (int k = 0; k < j; k++) Hrc[k] += beta * hh[k];
            Hrc[j] = beta * alpha;
            // fgmres.c:160-200 on that column: the previous rotations, a new one, the residual estimate
            i = j;
            iter++;
            double* Hc = H.data() + (size_t)(i - 1) * (kdim + 1);
            for (int k = 0; k <= i; k++) Hc[k] = Hrc[k];
            for (int k = 1; k < i; k++) {
               const double hii = Hc[k - 1];
               Hc[k - 1] = cs[k - 1] * hii + sn[k - 1] * Hc[k];
               Hc[k] = -sn[k - 1] * hii + cs[k - 1] * Hc[k];
            }
            const double hii = Hc[i - 1], hii1 = Hc[i];
            const double gam = std::sqrt(hii * hii + hii1 * hii1);
            if (std::fabs(gam) < EPS) {
               broke = true;
               break;
            }
            cs[i - 1] = hii / gam;
            sn[i - 1] = hii1 / gam;
            rs[i] = -sn[i - 1] * rs[i - 1];
            rs[i - 1] = cs[i - 1] * rs[i - 1];
            Hc[i - 1] = cs[i - 1] * hii + sn[i - 1] * hii1;
            normr = std::fabs(rs[i]);
            rel[iter] = normr / normb;
            if (print_level > 0)
               printf("%5d   %8e   %8e   %8.6f\n", iter, normr, rel[iter], rel[iter] / rel[iter - 1]);
            if (normr <= tolr) {
               converged = true;
               break;
            }
         }
         if (!more) break;
         // first pass of A v_j: H(<j, j) = (t - (H s))/alpha, H(j, j) = ((v_j^0, w) - s.t)/alpha - (H s)_j)/alpha
         const double* t = hh.data() + m;
         double st = 0.0;
         for (int k = 0; k < j; k++) st += hh[k] * t[k];
         const double vjw = (t[j] - st) / alpha;
         std::vector<double> Hs(m, 0.0);
         for (int q = 0; q < j; q++) {
            const double* Hrq = Hr.data() + (size_t)q * (kdim + 1);
            for (int k = 0; k <= q + 1 && k < m; k++) Hs[k] += Hrq[k] * hh[q];
         }
         double* Hrj = Hr.data() + (size_t)j * (kdim + 1);
         for (int k = 0; k < j; k++) Hrj[k] = (t[k] - Hs[k]) / alpha;
         Hrj[j] = (vjw - Hs[j]) / alpha;
         // update: v_j final, u = w / alpha - sum_{k<j} (t_k / alpha) v_k - (vjw / alpha) v_j
         coef.assign(2 * j + 2, 0.0);
         for (int k = 0; k < j; k++) {
            coef[k] = j > 0 ? hh[k] : 0.0;
            coef[j + k] = t[k] / alpha;
         }
         coef[2 * j] = vjw / alpha;
         coef[2 * j + 1] = 1.0 / alpha;
         if (c.dcgs2_update(V, w, j, coef, dsc + 2 * (m + 1))) return fail();  // ||u_{j+1}||^2 where step j + 1 reads it
      }
      if (broke) break;
      if (print_level == 0)
         printf("Rel. residual at the end of current cycle (# of steps per cycle/total its: %d/%d): %e \n", kdim,
                iter, rel[iter]);
      if (i > 0) {
         rs[i - 1] /= H[(size_t)(i - 1) * (kdim + 1) + i - 1];
         for (int k = i - 2; k >= 0; k--) {
            for (int q = k + 1; q < i; q++) rs[k] -= H[(size_t)q * (kdim + 1) + k] * rs[q];
            rs[k] /= H[(size_t)k * (kdim + 1) + k];
         }
         if (!cb.prec) {
            if (c.combine(x, V, i, rs.data())) return fail();
         } else {
            // x += sum_j y_j z_j with z_j = (z_j^0 - sum_{k<j} s_jk z_k) / alpha_j: from the last column down,
            // c_j = y_j / alpha_j moves -c_j s_jk onto z_k's coefficient
            ccoef.assign(rs.begin(), rs.begin() + i);
            for (int q = i - 1; q >= 0; q--) {
               ccoef[q] /= alph[q];
               for (int k = 0; k < q && k < (int)spass[q].size(); k++) ccoef[k] -= ccoef[q] * spass[q][k];
            }
            if (c.combine(x, Z, i, ccoef.data())) return fail();
         }
      }
      if (converged || normr <= tolr) break;
      // restart (fgmres.c:236-243): v = rhs - A x through w.  The reference keeps the Givens estimate as the
      // new cycle's norm, so its first basis vector is not of unit length; MGS tolerates that, but the block
      // orthogonalisations assume an orthonormal basis, so they restart from the true norm (one dot)
      double* w = V + n;
      c.copy(V, rhs);
      if (cb.apply(1.0, x, 0.0, w)) return fail();
      hipLaunchKernelGGL(k_sub, dim3(egrid(n)), dim3(256), 0, c.s, V, V, w, n);
      normr = c.norm(V);
   }
   *prel_res = normr / normb;
   *piter = iter;
   *prel_res_v = rel;
   cleanup();
   return 0;
}

// ---- FGMRES (fgmres.c:3-252) on device vectors ----------------------------------------------------
int fgmres_dev(Callbacks& cb, double* x, const double* rhs, int kdim, int maxits, int atol, double tol,
               double* prel_res, double** prel_res_v, int* piter, int print_level)
{
   const size_t n = cb.n;
   Ctx c{current_stream(), n, cb.comm};
   const double EPS = DBL_EPSILON;
   if (cb.n_global == 0) {  // (a row shard may hold no rows: it still takes part in every all-reduce)
      *prel_res = 0.0;
      *piter = 0;
      *prel_res_v = rel_hist(1);
      return 0;
   }
   const double normb = c.norm(rhs);
   if (normb < EPS) {
      NFFT4GP_HIP_CHECK(hipMemsetAsync(x, 0, sizeof(double) * n, c.s));
      *prel_res = 0.0;
      *piter = 0;
      *prel_res_v = rel_hist(1);
      return 0;
   }
   const int ortho = fgmres_ortho();
   if (ortho == 2)
      return fgmres_dcgs2_dev(cb, x, rhs, kdim, maxits, atol, tol, prel_res, prel_res_v, piter, print_level);
   const int kmax = ortho ? KScratch::kScal / 2 - 2 : KScratch::kScal - 2;
   if (kdim > kmax) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPSolverFgmres: restart dimension %d above %d\n", kdim, kmax);
      return -1;
   }
   double *V = nullptr, *Z = nullptr;
   // without a preconditioner z_i = v_i: the combination reads V and no Z is kept
   if (dmalloc(&V, n * (size_t)(kdim + 1)) || (cb.prec && dmalloc(&Z, n * (size_t)(kdim + 1)))) return -1;
   auto cleanup = [&]() {
      (void)hipStreamSynchronize(c.s);
      (void)hipFree(V);
      (void)hipFree(Z);
   };
   double* rel = nullptr;
   // every error exit: the bases and the history are released
   auto fail = [&]() -> int {
      free(rel);
      rel = nullptr;
      cleanup();
      return -1;
   };
   std::vector<double> H((size_t)kdim * (kdim + 1), 0.0), cs(kdim), sn(kdim), rs(kdim + 1);
   double* v = V;
   c.copy(v, rhs);
   if (cb.apply(-1.0, x, 1.0, v)) return fail();
   double normr = c.norm(v);
   if (normr < EPS) {
      *prel_res = 0.0;
      *piter = 0;
      *prel_res_v = rel_hist(1);
      cleanup();
      return 0;
   }
   const double tolr = atol ? tol : tol * normb;
   rel = rel_hist(maxits + 1);
   rel[0] = normr / normb;
   int iter = 0, i = 0;
   double* w = V;
   if (print_level > 0) {
      printf("--------------------------------------------------------------------------------\n");
      printf("Start FlexGMRES(%d)\n", kdim);
      printf("Residual Tol: %e\nMax number of inner iterations: %d\n", tolr, maxits);
      printf("--------------------------------------------------------------------------------\n");
      printf("Step    Residual norm  Relative res.  Convergence Rate\n");
      printf("%5d   %8e   %8e   N/A\n", 0, normr, rel[0]);
   }
   bool broke = false;
   while (iter < maxits) {
      rs[0] = normr;
      c.scale(v, nullptr, 1.0 / normr);
      i = 0;
      while (i < kdim && iter < maxits) {
         i++;
         iter++;
         v = V + (size_t)(i - 1) * n;
         w = V + (size_t)i * n;
         if (cb.prec) {
            double* z = Z + (size_t)(i - 1) * n;
            if (cb.solve(z, v) || cb.apply(1.0, z, 0.0, w)) return fail();
         } else {
            if (cb.apply(1.0, v, 0.0, w)) return fail();
         }
         double* hd = g_k.scal;
         std::vector<double> hcol(i + 1);
         if (ortho == 0) {
            // Nfft4GPModifiedGS (matops.c:274-346) with k = i-1, no re-orthogonalisation: one launch for the
            // sweep where the grid fits (k_mgs_chain), else one per projection
            const int rc = c.mgs_chain(w, V, i, hd);
            if (rc < 0) return fail();
            if (rc > 0) {
               // the per-projection chain, on the grid of the one-launch form this n would take (bitwise equal)
               unsigned mg = 0;
               if (c.mgs_form(&mg) < 0) mg = 0;
               for (int j = 0; j < i; j++)
                  if (c.gs(w, j ? V + (size_t)(j - 1) * n : nullptr, j ? hd + j - 1 : nullptr, V + (size_t)j * n,
                           hd + j, mg))
                     return fail();
               if (c.gs(w, V + (size_t)(i - 1) * n, hd + i - 1, nullptr, hd + i, mg)) return fail();
            }
            if (c.read(hd, i + 1, hcol.data())) return fail();
            if (rc == 0 && c.chain_failed()) return fail();
         } else {
            // classical passes h = V^T w, w -= V h; a second one only when the first dropped ||w|| below 0.7071
            // of its value before it (the DGKS test of the reference's MGS2, matops.c:348-440); H(:, i) = the
            // sum of the passes' projections, ||w|| after the last
            std::vector<double> hh(2 * i + 4);
            if (c.block_cgs2(w, V, i, hd) || c.read(hd, 2 * i + 4, hh.data())) return fail();
            for (int j = 0; j < i; j++) hcol[j] = hh[j];
            hcol[i] = hh[i];
            if (hh[2 * i + 3] != 0.0) {
               for (int j = 0; j < i; j++) hcol[j] += hh[i + 2 + j];
               hcol[i] = hh[2 * i + 2];
               g_fgmres_second_passes++;
            }
         }
         const double t = std::sqrt(hcol[i]);
         double* Hc = H.data() + (size_t)(i - 1) * (kdim + 1);
         for (int j = 0; j < i; j++) Hc[j] = hcol[j];
         Hc[i] = t;
         c.scale(w, nullptr, 1.0 / t);
         for (int j = 1; j < i; j++) {
            const double hii = Hc[j - 1];
            Hc[j - 1] = cs[j - 1] * hii + sn[j - 1] * Hc[j];
            Hc[j] = -sn[j - 1] * hii + cs[j - 1] * Hc[j];
         }
         const double hii = Hc[i - 1], hii1 = Hc[i];
         const double gam = std::sqrt(hii * hii + hii1 * hii1);
         if (std::fabs(gam) < EPS) {
            broke = true;  // fgmres.c:179-182: leave without updating x
            break;
         }
         cs[i - 1] = hii / gam;
         sn[i - 1] = hii1 / gam;
         rs[i] = -sn[i - 1] * rs[i - 1];
         rs[i - 1] = cs[i - 1] * rs[i - 1];
         Hc[i - 1] = cs[i - 1] * hii + sn[i - 1] * hii1;
         normr = std::fabs(rs[i]);
         rel[iter] = normr / normb;
         if (print_level > 0)
            printf("%5d   %8e   %8e   %8.6f\n", iter, normr, rel[iter], rel[iter] / rel[iter - 1]);
         if (normr <= tolr) break;
      }
      if (broke) break;
      if (print_level == 0)
         printf("Rel. residual at the end of current cycle (# of steps per cycle/total its: %d/%d): %e \n", kdim,
                iter, rel[iter]);
      rs[i - 1] /= H[(size_t)(i - 1) * (kdim + 1) + i - 1];
      for (int k = i - 2; k >= 0; k--) {
         for (int j = k + 1; j < i; j++) rs[k] -= H[(size_t)j * (kdim + 1) + k] * rs[j];
         rs[k] /= H[(size_t)k * (kdim + 1) + k];
      }
      if (c.combine(x, cb.prec ? Z : V, i, rs.data())) return fail();
      if (normr <= tolr) break;
      // restart (fgmres.c:236-243): v = rhs - A x through w; normr keeps the Givens estimate
      v = V;
      c.copy(v, rhs);
      if (cb.apply(1.0, x, 0.0, w)) return fail();
      hipLaunchKernelGGL(k_sub, dim3(egrid(n)), dim3(256), 0, c.s, v, v, w, n);
      if (ortho) normr = c.norm(v);  // block CGS2: restart from the true norm (see fgmres_dcgs2_dev)
   }
   *prel_res = normr / normb;
   *piter = iter;
   *prel_res_v = rel;
   cleanup();
   return 0;
}

// ---- FGMRES on a batch of right-hand sides (the predict's std solves) ---------------------------------------
// fgmres_dev's MGS iteration (fgmres.c:3-252, ortho 0) for m systems A x_s = b_s at once, in lockstep: every
// running system is at the same step, so each projection is ONE launch over all of them (k_gs_batch, grid.y =
// running systems), the step's Hessenberg entries of every system come back in ONE read, and the operator
// applications go out together (two vectors per pass on this library's additive operator,
// additive_matvec_multi).  Per system the Givens recurrence, breakdown exit, restart and tolerance are
// fgmres_dev's, and so is the arithmetic of every vector kernel (the same bodies and grids): with one system
// the results are fgmres_dev's.  A system leaves the batch when it converges or breaks down, the others go on.
// x0 = 0 (the predict's initial guess, nfft_interface.c:1030-1036), so v_0 = b without an operator application.
// The basis grows in groups of columns as the steps need them (nfft_interface.c:1044 asks for a restart
// dimension of n: no n x n basis is reserved).  x_s = X + s ldx, b_s = B + s ldb.  Lines that fgmres_dev
// would print are kept per system and printed in system order at the end.
struct BatchOut {
   std::vector<int> iters;
   std::vector<double> rel_res;
};

int fgmres_batch_dev(Callbacks& cb, int m, double* X, size_t ldx, const double* B, size_t ldb, int kdim, int maxits,
                     int atol, double tol, int print_level, BatchOut& res)
{
   const size_t n = cb.n;
   hipStream_t st = current_stream();
   const double EPS = DBL_EPSILON;
   res.iters.assign(m, 0);
   res.rel_res.assign(m, 0.0);
   if (m <= 0) return 0;
   if (cb.comm || cb.n_global != cb.n) return -1;
   const bool multi = cb.mv_dev && cb.matvec == (func_symmatvec)&Nfft4GPAdditiveNFFTMatSymv;
   const unsigned ggrid = (unsigned)std::max<size_t>(1, std::min<size_t>((n + 4095) / 4096, kKMaxBlocks));
   // device scratch: partials / tickets per slot, the step's scalars [j][s], factors, the running list
   double *part = nullptr, *hd = nullptr, *dfac = nullptr, *dcoef = nullptr;
   const double** dcols = nullptr;
   unsigned int* ticket = nullptr;
   int* dact = nullptr;
   double* pin = nullptr;  // pinned: [0, m) factors, then the combine's coefficients and column pointers
   int* pact = nullptr;    // pinned: the running list
   // the one-launch MGS sweep (k_mgs_chain<.., true>): device column table, error word
   const double** dvcols = nullptr;
   const double** pvcols = nullptr;  // pinned staging of new column pointers
   int *derr = nullptr, *herr = nullptr;
   int vcols_up = 0;
   hipEvent_t pin_ev = nullptr;  // the last copy out of pin / pact
   std::vector<double*> groups;  // basis column groups (V, then Z when preconditioned)
   std::vector<double*> Vc, Zc;  // column j of every system: Vc[j] + s n
   int hcap = 0;                 // columns of hd
   auto cleanup = [&]() {
      (void)hipStreamSynchronize(st);
      for (double* g : groups) (void)hipFree(g);
      (void)hipFree(part);
      (void)hipFree(hd);
      (void)hipFree(dfac);
      (void)hipFree(dcoef);
      (void)hipFree(dcols);
      (void)hipFree(ticket);
      (void)hipFree(dact);
      if (pin) (void)hipHostFree(pin);
      if (pact) (void)hipHostFree(pact);
      (void)hipFree(dvcols);
      (void)hipFree(derr);
      if (pvcols) (void)hipHostFree(pvcols);
      if (herr) (void)hipHostFree(herr);
      if (pin_ev) (void)hipEventDestroy(pin_ev);
   };
   auto fail = [&]() -> int {
      cleanup();
      return -1;
   };
   const int kcyc = std::min(kdim, maxits) + 1;  // columns a cycle can combine
   const int kpin = 4 * m + 2 * kcyc + 16;
   if (dmalloc(&part, (size_t)m * kKMaxBlocks) || dmalloc(&ticket, (size_t)m * kTicketWords) || dmalloc(&dfac, m) ||
       dmalloc(&dact, m) || dmalloc(&dcoef, (size_t)kcyc) || dmalloc(&dcols, (size_t)kcyc))
      return fail();
   if (hipHostMalloc((void**)&pin, sizeof(double) * kpin) != hipSuccess) {
      pin = nullptr;
      return fail();
   }
   if (hipHostMalloc((void**)&pact, sizeof(int) * m) != hipSuccess) {
      pact = nullptr;
      return fail();
   }
   const int colcap = std::min(kdim, maxits) + 2;
   if (dmalloc(&dvcols, (size_t)colcap) || dmalloc(&derr, 1)) return fail();
   if (hipHostMalloc((void**)&pvcols, sizeof(double*) * 64) != hipSuccess ||
       hipHostMalloc((void**)&herr, sizeof(int)) != hipSuccess) {
      pvcols = nullptr;
      herr = nullptr;
      return fail();
   }
   *herr = 0;
   NFFT4GP_HIP_CHECK(hipMemsetAsync(derr, 0, sizeof(int), st));
   static int occ_batch = -1;  // resident k_mgs_chain<1024, 4, true> workgroups on the device
   if (occ_batch < 0) {
      int dev = 0, occ = 0;
      hipDeviceProp_t prop;
      occ_batch = 0;
      if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess &&
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_mgs_chain<1024, 4, true>, 1024, 0) == hipSuccess)
         occ_batch = occ * prop.multiProcessorCount;
   }
   NFFT4GP_HIP_CHECK(hipEventCreateWithFlags(&pin_ev, hipEventDisableTiming));
   NFFT4GP_HIP_CHECK(hipEventRecord(pin_ev, st));
   // the staging buffers are rewritten only after the copies out of them have run
   auto pin_wait = [&]() -> int {
      NFFT4GP_HIP_CHECK(hipEventSynchronize(pin_ev));
      return 0;
   };
   auto pin_done = [&]() -> int {
      NFFT4GP_HIP_CHECK(hipEventRecord(pin_ev, st));
      return 0;
   };
   NFFT4GP_HIP_CHECK(hipMemsetAsync(ticket, 0, sizeof(unsigned int) * (size_t)m * kTicketWords, st));
   // columns [0, need) of the basis (and of Z) allocated, in groups of 16 columns
   auto ensure_cols = [&](int need) -> int {
      constexpr int kG = 16;
      while ((int)Vc.size() < need) {
         const int g = std::min(kG, std::max(1, need + kG - 1 - (int)Vc.size()));
         for (int pass = 0; pass < (cb.prec ? 2 : 1); pass++) {
            double* base = nullptr;
            if (hipMalloc((void**)&base, sizeof(double) * n * m * g) != hipSuccess) {
               fprintf(stderr, "nfft4gp_amd: FGMRES batch of %d: no memory for %zu basis columns of %zu\n", m,
                       Vc.size() + g, n);
               return -1;
            }
            groups.push_back(base);
            for (int k = 0; k < g; k++) (pass ? Zc : Vc).push_back(base + (size_t)k * n * m);
         }
      }
      return 0;
   };
   auto ensure_h = [&](int cols) -> int {
      if (cols <= hcap) return 0;
      const int nc = std::max(cols, 2 * hcap);
      double* nh = nullptr;
      if (dmalloc(&nh, (size_t)nc * m)) return -1;
      NFFT4GP_HIP_CHECK(hipStreamSynchronize(st));
      (void)hipFree(hd);
      hd = nh;
      hcap = nc;
      return 0;
   };
   std::vector<int> act;
   auto upload_act = [&]() -> int {  // stream-ordered: launches already queued still read the old list
      if (pin_wait()) return -1;
      memcpy(pact, act.data(), sizeof(int) * act.size());
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(dact, pact, sizeof(int) * act.size(), hipMemcpyHostToDevice, st));
      return pin_done();
   };
   auto read = [&](const double* d, size_t count, std::vector<double>& h) -> int {
      h.resize(count);
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(h.data(), d, sizeof(double) * count, hipMemcpyDeviceToHost, st));
      NFFT4GP_HIP_CHECK(hipStreamSynchronize(st));
      return 0;
   };
   // w_s -= hprev[s] u_s (u optional), out[s] = (w_s, v_s) or ||w_s||^2, for the running systems
   auto gs = [&](double* w, size_t ldw, const double* u, size_t ldu, const double* hprev, const double* v, size_t ldv,
                 double* out) -> int {
      hipLaunchKernelGGL((k_gs_batch<1024, 4>), dim3(ggrid, (unsigned)act.size()), dim3(1024), 0, st, w, ldw, u, ldu,
                         hprev, v, ldv, n, (const int*)dact, part, ticket, out);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return 0;
   };
   auto scale = [&](double* a, const std::vector<double>& fac) -> int {
      if (pin_wait()) return -1;
      memcpy(pin, fac.data(), sizeof(double) * m);
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(dfac, pin, sizeof(double) * m, hipMemcpyHostToDevice, st));
      if (pin_done()) return -1;
      hipLaunchKernelGGL(k_scale_batch, dim3(std::max(1, egrid(n) / std::max(1, (int)act.size())), (unsigned)act.size()),
                         dim3(256), 0, st, a, n, n, (const int*)dact, (const double*)dfac);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return 0;
   };
   // y_s = A x_s for the running systems
   auto apply = [&](const std::vector<const double*>& xs, const std::vector<double*>& ys) -> int {
      if (multi) return additive_matvec_multi(cb.mat, (int)xs.size(), 1.0, xs.data(), 0.0, ys.data());
      for (size_t k = 0; k < xs.size(); k++)
         if (cb.apply(1.0, const_cast<double*>(xs[k]), 0.0, ys[k])) return -1;
      return 0;
   };
   // x_s += sum_j c[j] cols[j] + s n
   auto combine = [&](int s, const std::vector<double*>& cols, int cnt, const double* c) -> int {
      if (cnt <= 0) return 0;
      if (pin_wait()) return -1;
      double* pc = pin + m;
      const double** pp = (const double**)(pin + m + cnt);
      for (int j = 0; j < cnt; j++) {
         pc[j] = c[j];
         pp[j] = cols[j] + (size_t)s * n;
      }
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(dcoef, pc, sizeof(double) * cnt, hipMemcpyHostToDevice, st));
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(dcols, pp, sizeof(double*) * cnt, hipMemcpyHostToDevice, st));
      if (pin_done()) return -1;
      hipLaunchKernelGGL(k_combine_cols, dim3(egrid(n)), dim3(256), 0, st, X + (size_t)s * ldx, (const double* const*)dcols,
                         n, (const double*)dcoef, cnt);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return 0;
   };
   if (2 * kcyc + 2 * m > kpin) return fail();

   struct Sys {
      double normb = 0, normr = 0, tolr = 0, rel_prev = 0;
      std::vector<std::vector<double>> H;  // H[i - 1]: column i - 1 (i + 1 entries)
      std::vector<double> cs, sn, rs;
      std::string log;
      bool done = false;
   };
   std::vector<Sys> S(m);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wformat-security"
   auto logf = [&](int s, const char* fmt, auto... a) {  // (fmt: the literals below)
      char buf[256];
      snprintf(buf, sizeof(buf), fmt, a...);
      S[s].log += buf;
   };
#pragma clang diagnostic pop
   for (int s = 0; s < m; s++) NFFT4GP_HIP_CHECK(hipMemsetAsync(X + (size_t)s * ldx, 0, sizeof(double) * n, st));
   if (ensure_cols(2) || ensure_h(2)) return fail();
   act.resize(m);
   for (int s = 0; s < m; s++) act[s] = s;
   if (upload_act()) return fail();
   // ||b_s|| (c.norm: the dot of b with itself), then v_0 = b - A 0 = b
   std::vector<double> hh;
   if (gs(const_cast<double*>(B), ldb, nullptr, 0, nullptr, B, ldb, hd) || read(hd, m, hh)) return fail();
   for (int s = 0; s < m; s++) {
      S[s].normb = std::sqrt(hh[s]);
      S[s].normr = S[s].normb;  // ||v_0|| = ||b||: the same vector
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(Vc[0] + (size_t)s * n, B + (size_t)s * ldb, sizeof(double) * n,
                                       hipMemcpyDeviceToDevice, st));
   }
   act.clear();
   for (int s = 0; s < m; s++) {
      Sys& y = S[s];
      if (y.normb < EPS) {  // x = 0 (set above), rel_res 0, 0 iterations
         y.done = true;
         continue;
      }
      y.tolr = atol ? tol : tol * y.normb;
      y.rel_prev = y.normr / y.normb;
      if (print_level > 0) {
         logf(s, "--------------------------------------------------------------------------------\n");
         logf(s, "Start FlexGMRES(%d)\n", kdim);
         logf(s, "Residual Tol: %e\nMax number of inner iterations: %d\n", y.tolr, maxits);
         logf(s, "--------------------------------------------------------------------------------\n");
         logf(s, "Step    Residual norm  Relative res.  Convergence Rate\n");
         logf(s, "%5d   %8e   %8e   N/A\n", 0, y.normr, y.rel_prev);
      }
      act.push_back(s);
   }
   if (upload_act()) return fail();
   // the end of a cycle of system s after i steps (fgmres.c:221-235): back substitution, x += Z y
   auto finish_cycle = [&](int s, int i) -> int {
      Sys& y = S[s];
      if (i <= 0) return 0;
      std::vector<double>& rs = y.rs;
      rs[i - 1] /= y.H[i - 1][i - 1];
      for (int k = i - 2; k >= 0; k--) {
         for (int j = k + 1; j < i; j++) rs[k] -= y.H[j][k] * rs[j];
         rs[k] /= y.H[k][k];
      }
      return combine(s, cb.prec ? Zc : Vc, i, rs.data());
   };
   int iter = 0;
   std::vector<double> fac(m, 0.0);
   while (!act.empty() && iter < maxits) {
      for (int s : act) {
         S[s].rs.assign(1, S[s].normr);
         S[s].H.clear();
         S[s].cs.clear();
         S[s].sn.clear();
         fac[s] = 1.0 / S[s].normr;
      }
      if (scale(Vc[0], fac)) return fail();
      int i = 0;
      while (!act.empty() && i < kdim && iter < maxits) {
         i++;
         iter++;
         if (ensure_cols(i + 1) || ensure_h(i + 1)) return fail();
         std::vector<const double*> xs;
         std::vector<double*> ys;
         for (int s : act) {
            double* v = Vc[i - 1] + (size_t)s * n;
            if (cb.prec) {
               double* z = Zc[i - 1] + (size_t)s * n;
               if (cb.solve(z, v)) return fail();
               xs.push_back(z);
            } else {
               xs.push_back(v);
            }
            ys.push_back(Vc[i] + (size_t)s * n);
         }
         if (apply(xs, ys)) return fail();
         // Nfft4GPModifiedGS (matops.c:274-346) with k = i - 1: the whole sweep of every running system in one
         // launch where the grid fits (k_mgs_chain), else one launch per projection for all of them
         const char* ce = getenv("NFFT4GP_AMD_MGS_CHAIN");
         const bool chain = !(ce && atoi(ce) == 0) && (size_t)ggrid * 4096 >= n &&
                            (long)ggrid * (long)act.size() <= (long)occ_batch && i + 1 <= colcap && !*herr;
         if (chain) {
            while (vcols_up <= i) {  // the column table: pointers of columns not uploaded yet
               if (pin_wait()) return fail();
               const int cnt = std::min(64, i + 1 - vcols_up);
               for (int k = 0; k < cnt; k++) pvcols[k] = Vc[vcols_up + k];
               NFFT4GP_HIP_CHECK(hipMemcpyAsync(dvcols + vcols_up, pvcols, sizeof(double*) * cnt,
                                                hipMemcpyHostToDevice, st));
               if (pin_done()) return fail();
               vcols_up += cnt;
            }
            NFFT4GP_HIP_CHECK(hipMemsetAsync(hd, 0xFF, sizeof(double) * (size_t)(i + 1) * m, st));  // kChainUnset
            hipLaunchKernelGGL((k_mgs_chain<1024, 4, true>), dim3(ggrid, (unsigned)act.size()), dim3(1024), 0, st,
                               (double*)nullptr, (const double*)nullptr, n, i, hd, part, ticket, derr,
                               (const double* const*)dvcols, (const int*)dact, m);
            NFFT4GP_HIP_CHECK(hipGetLastError());
            NFFT4GP_HIP_CHECK(hipMemcpyAsync(herr, derr, sizeof(int), hipMemcpyDeviceToHost, st));
         } else {
            for (int j = 0; j < i; j++)
               if (gs(Vc[i], n, j ? Vc[j - 1] : nullptr, n, j ? hd + (size_t)(j - 1) * m : nullptr, Vc[j], n,
                      hd + (size_t)j * m))
                  return fail();
            if (gs(Vc[i], n, Vc[i - 1], n, hd + (size_t)(i - 1) * m, nullptr, 0, hd + (size_t)i * m)) return fail();
         }
         if (read(hd, (size_t)(i + 1) * m, hh)) return fail();
         if (chain && *herr) {
            fprintf(stderr, "nfft4gp_amd: FGMRES batch: the one-launch MGS sweep's wait gave up\n");
            return fail();
         }
         std::vector<int> keep, conv;
         for (int s : act) {
            Sys& y = S[s];
            const double t = std::sqrt(hh[(size_t)i * m + s]);
            std::vector<double> Hc(i + 1);
            for (int j = 0; j < i; j++) Hc[j] = hh[(size_t)j * m + s];
            Hc[i] = t;
            fac[s] = 1.0 / t;
            for (int j = 1; j < i; j++) {
               const double hii = Hc[j - 1];
               Hc[j - 1] = y.cs[j - 1] * hii + y.sn[j - 1] * Hc[j];
               Hc[j] = -y.sn[j - 1] * hii + y.cs[j - 1] * Hc[j];
            }
            const double hii = Hc[i - 1], hii1 = Hc[i];
            const double gam = std::sqrt(hii * hii + hii1 * hii1);
            if (std::fabs(gam) < EPS) {  // fgmres.c:179-182: leave without updating x
               y.done = true;
               res.iters[s] = iter;
               res.rel_res[s] = y.normr / y.normb;
               continue;
            }
            y.cs.push_back(hii / gam);
            y.sn.push_back(hii1 / gam);
            y.rs.push_back(-y.sn[i - 1] * y.rs[i - 1]);
            y.rs[i - 1] = y.cs[i - 1] * y.rs[i - 1];
            Hc[i - 1] = y.cs[i - 1] * hii + y.sn[i - 1] * hii1;
            y.H.push_back(std::move(Hc));
            y.normr = std::fabs(y.rs[i]);
            const double rel = y.normr / y.normb;
            if (print_level > 0) logf(s, "%5d   %8e   %8e   %8.6f\n", iter, y.normr, rel, rel / y.rel_prev);
            y.rel_prev = rel;
            (y.normr <= y.tolr ? conv : keep).push_back(s);
         }
         if (scale(Vc[i], fac)) return fail();
         for (int s : conv) {  // converged in this cycle: its end (fgmres.c:212-235)
            if (print_level == 0)
               logf(s, "Rel. residual at the end of current cycle (# of steps per cycle/total its: %d/%d): %e \n", kdim,
                    iter, S[s].rel_prev);
            if (finish_cycle(s, i)) return fail();
            S[s].done = true;
            res.iters[s] = iter;
            res.rel_res[s] = S[s].normr / S[s].normb;
         }
         if (keep.size() != act.size()) {
            act = keep;
            if (!act.empty() && upload_act()) return fail();
         }
      }
      if (act.empty()) break;
      // the cycle ends for every running system together (restart dimension or maxits reached)
      for (int s : act) {
         if (print_level == 0)
            logf(s, "Rel. residual at the end of current cycle (# of steps per cycle/total its: %d/%d): %e \n", kdim,
                 iter, S[s].rel_prev);
         if (finish_cycle(s, i)) return fail();
      }
      if (iter >= maxits) break;
      // restart (fgmres.c:236-243): v = b - A x; normr keeps the Givens estimate
      std::vector<const double*> xs;
      std::vector<double*> ys;
      for (int s : act) {
         xs.push_back(X + (size_t)s * ldx);
         ys.push_back(Vc[1] + (size_t)s * n);
      }
      if (apply(xs, ys)) return fail();
      for (int s : act)
         hipLaunchKernelGGL(k_sub, dim3(egrid(n)), dim3(256), 0, st, Vc[0] + (size_t)s * n, B + (size_t)s * ldb,
                            (const double*)(Vc[1] + (size_t)s * n), n);
      NFFT4GP_HIP_CHECK(hipGetLastError());
   }
   for (int s : act) {
      res.iters[s] = iter;
      res.rel_res[s] = S[s].normr / S[s].normb;
   }
   bool printed = false;
   for (int s = 0; s < m; s++)
      if (!S[s].log.empty()) {
         fputs(S[s].log.c_str(), stdout);
         printed = true;
      }
   if (printed) fflush(stdout);
   cleanup();
   return 0;
}

// ---- Lanczos (lanczos.c:3-419) on device vectors ----------------------------------------------------
// Re-orthogonalisation of w against V[0..k] (dots) / Z[0..k] (updates), adding the projections on v_{k-1}
// and v_k to te / td (Nfft4GPModifiedGS2, matops.c:348-440: MGS over the whole basis, repeated while ||w||
// drops below 0.7071 of its previous value).  Here:
//   1. a local classical pass against the last one or two basis vectors (v_{k-1}, v_k: the three-term
//      recurrence, where the large projections of a Lanczos step are), with ||w|| before it;
//   2. classical passes over the whole basis (Ctx::block_gs: one launch for all the dots, one for the update),
//      repeated while ||w|| drops below 0.7071 of its value before the pass (the DGKS / "twice is enough"
//      test the reference applies), at least one.
// After the local pass the whole-basis projections are at rounding level, so one whole pass normally ends the
// step: the basis is read twice per step instead of four times (two whole passes, the round-3 scheme).  In
// exact arithmetic the projections equal MGS's; in floating point they differ by rounding.
static int mgs2(Ctx& c, double* w, const double* V, const double* Z, int k, double* td, double* te, double* t)
{
   double* hd = g_k.scal;
   const size_t n = c.n;
   const int j0 = k >= 1 ? k - 1 : 0;
   const int ml = k + 1 - j0;  // 1 or 2 basis vectors in the local pass
   if (c.block_gs(w, V + (size_t)j0 * n, Z + (size_t)j0 * n, ml, hd, 1)) return -1;
   double hl[4];
   if (c.read(hd, ml + 2, hl)) return -1;
   if (k >= 1 && te) *te = hl[0];
   if (td) *td = hl[ml - 1];
   double normw = std::sqrt(hl[ml]);  // ||w|| after the local pass
   *t = normw;
   if (normw < DBL_EPSILON) return 0;  // w lies in span(v_{k-1}, v_k): the reference's loop stops here too
   std::vector<double> h(k + 2);
   for (;;) {
      if (c.block_gs(w, V, Z, k + 1, hd, 0)) return -1;
      if (c.read(hd, k + 2, h.data())) return -1;
      if (k >= 1 && te) *te += h[k - 1];
      if (td) *td += h[k];
      *t = std::sqrt(h[k + 1]);
      if (!(*t < normw * 0.7071 && *t >= DBL_EPSILON)) break;
      normw = *t;
   }
   return 0;
}

// One Lanczos run as a resumable object, so that two probes of the quadrature can share their matvecs
// (lanczos_pair_dev).  lanczos_dev drives one run the way lanczos.c does.
struct LanczosRun {
   Callbacks& cb;
   Ctx c;
   size_t n;
   double* x;
   int wsize, maxits, print_level;
   double tol;
   int atol;
   bool alias = false;
   double *V = nullptr, *Z = nullptr, *z = nullptr, *v = nullptr, *wv = nullptr;
   double *TD = nullptr, *TE = nullptr, *rel = nullptr;
   double **TDp, **TEp;
   std::vector<double> TLD, TLE, y;
   double normb = 0.0, beta = 0.0, tolr = 0.0, normr = 0.0, ls = 0.0, t = 0.0, dotvz = 0.0;
   int iter = 0, chol_size = 0;
   bool done_early = false;  // the run ended in init (n == 0, b == 0, beta == 0): outputs already set
   static constexpr double EPS = DBL_EPSILON;

   LanczosRun(Callbacks& cb_, double* x_, int wsize_, int maxits_, int atol_, double tol_, int print_level_,
              double** TDp_, double** TEp_)
       : cb(cb_), c{current_stream(), cb_.n, cb_.comm}, n(cb_.n), x(x_), wsize(wsize_), maxits(maxits_),
         print_level(print_level_), tol(tol_), atol(atol_), TDp(TDp_), TEp(TEp_)
   {
      if (wsize <= 0) wsize = maxits;
      wsize = std::min(wsize, maxits);
   }
   ~LanczosRun()
   {
      if (V || Z) (void)hipStreamSynchronize(c.s);
      (void)hipFree(V);
      if (!alias) (void)hipFree(Z);
      if (TD && TD != *TDp) free(TD);
      if (TE && TE != *TEp) free(TE);
      free(rel);
   }
   // everything before the first step; returns -1 on error, 1 when the run is already complete
   int init(const double* rhs, double* prel_res, double** prel_res_v, int* piter)
   {
      if (cb.n_global == 0) {
         *prel_res = 0.0;
         *piter = 0;
         *prel_res_v = rel_hist(1);
         done_early = true;
         return 1;
      }
      normb = c.norm(rhs);
      if (normb < EPS) {
         NFFT4GP_HIP_CHECK(hipMemsetAsync(x, 0, sizeof(double) * n, c.s));
         *prel_res = 0.0;
         *piter = 0;
         *prel_res_v = rel_hist(1);
         done_early = true;
         return 1;
      }
      if (maxits + 2 > KScratch::kScal) {
         fprintf(stderr, "nfft4gp_amd: Nfft4GPSolverLanczos: maxits %d above %d\n", maxits, KScratch::kScal - 2);
         return -1;
      }
      // without a preconditioner v = z at every step (the same copy, scaled by the same factor), so the
      // basis is stored once and is its own update basis
      alias = !cb.prec;
      if (dmalloc(&V, n * (size_t)(maxits + 1))) return -1;
      if (alias)
         Z = V;
      else if (dmalloc(&Z, n * (size_t)(maxits + 1)))
         return -1;
      TLD.assign(maxits + 1, 0.0);
      TLE.assign(maxits + 1, 0.0);
      y.assign(maxits + 1, 0.0);
      TD = *TDp ? *TDp : (double*)calloc((size_t)maxits + 1, sizeof(double));
      TE = *TEp ? *TEp : (double*)calloc((size_t)std::max(1, maxits), sizeof(double));
      z = Z;
      v = V;
      c.copy(z, rhs);
      if (cb.apply(-1.0, x, 1.0, z)) return -1;
      if (cb.prec) {
         if (cb.solve(v, z)) return -1;
      } else if (!alias) {
         c.copy(v, z);
      }
      normr = c.norm(z);
      beta = std::sqrt(c.dot(v, z));
      if (beta < EPS) {
         *prel_res = 0.0;
         *piter = 0;
         *prel_res_v = rel_hist(1);
         done_early = true;
         return 1;
      }
      tolr = atol ? tol / beta : tol;
      rel = rel_hist(maxits + 1);
      rel[0] = normr / normb;
      if (print_level > 0) {
         printf("--------------------------------------------------------------------------------\n");
         printf("Start Lanczos(%d)\n", maxits);
         printf("Residual Tol: %e\nMax number of inner iterations: %d\n", tolr, maxits);
         printf("--------------------------------------------------------------------------------\n");
         printf("Step    Residual norm  Relative res.  Convergence Rate\n");
         printf("%5d   %8e   %8e   N/A\n", 0, normr, rel[0]);
      }
      c.scale(v, alias ? nullptr : z, 1.0 / beta);
      return 0;
   }
   // a step up to its matvec: z_iter = A v_{iter-1} is the caller's
   void step_begin()
   {
      iter++;
      z = Z + (size_t)iter * n;
      wv = V + (size_t)(iter - 1) * n;
      v = V + (size_t)iter * n;
   }
   // the rest of the step; 1 ends the loop (breakdown, or convergence in the first loop)
   // the fast step (one host read): k of this step, and whether its scalars fit a region of kRegion doubles
   static constexpr int kB0 = 8;
   static constexpr int kRegion = KScratch::kScal / 2;
   int step_k(bool first_loop) const { return first_loop ? std::min(iter - 1, wsize) : iter - 1; }
   bool fast_ok(bool first_loop) const { return kB0 + step_k(first_loop) + 1 + 4 <= kRegion; }
   int region_len(bool first_loop) const { return kB0 + step_k(first_loop) + 1 + 4; }
   // mgs2's local pass and first whole-basis pass, then (speculatively) the preconditioner and k_dot2 of the
   // step, scalars into hd[0, region_len): the host needs mgs2's scalars only to decide whether a further pass
   // is due (rare after the local pass) or w broke down, and in both cases the speculative results are
   // dropped (a further pass recomputes them; a breakdown restarts v and z).  Same kernels, same order, same
   // values as mgs2 followed by the solve and the dot.
   int step_enqueue(bool first_loop, double* hd)
   {
      const int k = step_k(first_loop);
      const int m = k + 1;
      const int j0 = k >= 1 ? k - 1 : 0;
      const int ml = k + 1 - j0;
      double* o = hd + kB0 + m + 2;
      if (c.lanczos_local(z, V + (size_t)j0 * n, Z + (size_t)j0 * n, ml, hd)) return -1;
      if (c.block_gs(z, V, Z, m, hd + kB0, 0)) return -1;
      if (cb.prec && cb.solve(v, z)) return -1;
      hipLaunchKernelGGL(k_dot2, dim3(kgrid(n)), dim3(kKThreads), 0, c.s, v, z, n, g_k.part, g_k.ticket, g_k.part2,
                         g_k.ticket2, o);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return c.red(o, 2);
   }
   // the host side of step_enqueue's scalars hh (read back): mgs2's bookkeeping and repeat rule, then the step's
   // tail; 1 ends the loop
   int step_after(bool first_loop, const double* hh)
   {
      if (c.lanczos_local_failed()) return -1;
      const int k = step_k(first_loop);
      const int m = k + 1;
      const int j0 = k >= 1 ? k - 1 : 0;
      const int ml = k + 1 - j0;
      double te_dummy;
      double* tdp = TD + iter - 1;
      double* tep = iter >= 2 ? TE + iter - 2 : &te_dummy;
      if (k >= 1) *tep = hh[0];
      *tdp = hh[ml - 1];
      double normw = std::sqrt(hh[ml]);  // ||w|| after the local pass
      if (normw < DBL_EPSILON) {          // mgs2 stops after the local pass
         t = normw;
         return 1;
      }
      const double* h = hh + kB0;
      if (k >= 1) *tep += h[k - 1];
      *tdp += h[k];
      t = std::sqrt(h[k + 1]);
      bool again = t < normw * 0.7071 && t >= DBL_EPSILON;
      double vz[2] = {hh[kB0 + m + 2], hh[kB0 + m + 3]};
      if (again) {
         double* hd = g_k.scal;
         std::vector<double> h2(k + 2);
         while (again) {  // mgs2's repeat rule, then the solve and the dot of the final w
            normw = t;
            if (c.block_gs(z, V, Z, m, hd, 0) || c.read(hd, k + 2, h2.data())) return -1;
            if (k >= 1) *tep += h2[k - 1];
            *tdp += h2[k];
            t = std::sqrt(h2[k + 1]);
            again = t < normw * 0.7071 && t >= DBL_EPSILON;
         }
         if (t < EPS) return 1;
         if (cb.prec && cb.solve(v, z)) return -1;
         double* o2 = g_k.scal + KScratch::kScal - 2;
         hipLaunchKernelGGL(k_dot2, dim3(kgrid(n)), dim3(kKThreads), 0, c.s, v, z, n, g_k.part, g_k.ticket,
                            g_k.part2, g_k.ticket2, o2);
         if (c.red(o2, 2) || c.read(o2, 2, vz)) return -1;
      } else if (t < EPS) {
         return 1;
      }
      return step_tail(first_loop, vz);
   }
   int step_end(bool first_loop)
   {
      if (fast_ok(first_loop)) {
         const int len = region_len(first_loop);
         std::vector<double> hh(len);
         if (step_enqueue(first_loop, g_k.scal) || c.read(g_k.scal, len, hh.data())) return -1;
         return step_after(first_loop, hh.data());
      }
      const int k = step_k(first_loop);
      double te_dummy;
      if (mgs2(c, z, V, Z, k, TD + iter - 1, iter >= 2 ? TE + iter - 2 : &te_dummy, &t)) return -1;
      if (t < EPS) return 1;
      if (cb.prec) {
         if (cb.solve(v, z)) return -1;
      }
      double* o = g_k.scal + KScratch::kScal - 2;
      hipLaunchKernelGGL(k_dot2, dim3(kgrid(n)), dim3(kKThreads), 0, c.s, v, z, n, g_k.part, g_k.ticket, g_k.part2,
                         g_k.ticket2, o);
      double vz[2];
      if (c.red(o, 2) || c.read(o, 2, vz)) return -1;
      return step_tail(first_loop, vz);
   }
   // the rest of a step from (v, z) and ||z||^2 (the scaling, the Cholesky of T, the residual estimate)
   int step_tail(bool first_loop, const double* vz)
   {
      dotvz = std::sqrt(vz[0]);
      if (dotvz < EPS) return 1;
      c.scale(v, alias ? nullptr : z, 1.0 / dotvz);
      if (first_loop) {
         const double normz = std::sqrt(vz[1]) / dotvz;
         if (iter != 1) {
            TLE[iter - 2] = TE[iter - 2] / TLD[iter - 2];
            TLD[iter - 1] = std::sqrt(TD[iter - 1] - TLE[iter - 2] * TLE[iter - 2]);
            const double le = 1.0 / TLD[iter - 1];
            ls = -ls * TLE[iter - 2] * le;
            normr = std::fabs(le * ls) * dotvz * beta * normz;
         } else {
            TLD[0] = std::sqrt(TD[0]);
            ls = 1.0 / TLD[0];
            normr = dotvz / TD[0] * beta * normz;
         }
         chol_size++;
         rel[iter] = normr / normb;
         if (print_level > 0)
            printf("%5d   %8e   %8e   %8.6f\n", iter, normr, rel[iter], rel[iter] / rel[iter - 1]);
         if (normr <= tolr) return 1;
      } else if (print_level > 0) {
         printf("%5d   Building T\n", iter);
      }
      return 0;
   }
   int step(bool first_loop)
   {
      step_begin();
      if (cb.apply(1.0, wv, 0.0, z)) return -1;
      return step_end(first_loop);
   }
   // after the first loop: the solution from the Cholesky factor of T (lanczos.c:258-273), then the second
   // loop that completes T up to wsize, restarting from a random vector after a breakdown
   int finish(double* prel_res, double** prel_res_v, int* piter, int* tsize)
   {
      if (print_level == 0)
         printf("Rel. residual at the end of the iteration (# of its: %d): %e \n", iter, rel[iter]);
      if (chol_size > 0) {
         y[0] = beta / TLD[0];
         for (int k = 1; k < chol_size; k++) y[k] = (-y[k - 1] * TLE[k - 1]) / TLD[k];
         y[chol_size - 1] /= TLD[chol_size - 1];
         for (int k = chol_size - 2; k >= 0; k--) y[k] = (y[k] - TLE[k] * y[k + 1]) / TLD[k];
         if (c.combine(x, V, chol_size, y.data())) return -1;
      }
      *prel_res = normr / normb;
      *piter = iter;
      *prel_res_v = rel;
      rel = nullptr;
      while (iter < wsize) {
         if (t < EPS || dotvz < EPS) {
            z = Z + (size_t)iter * n;
            v = V + (size_t)iter * n;
            // Nfft4GPVecRand of the whole vector (every rank draws the same n_global numbers; a row shard
            // keeps its rows)
            std::vector<double> rnd(cb.n_global);
            {
               CallerRandBatch caller;
               for (size_t i = 0; i < cb.n_global; i++) rnd[i] = (double)rand() / (double)RAND_MAX;
            }
            NFFT4GP_HIP_CHECK(hipMemcpy(z, rnd.data() + cb.row_begin, sizeof(double) * n, hipMemcpyHostToDevice));
            double td, te;
            if (mgs2(c, z, V, Z, iter - 1, &td, &te, &t)) return -1;
            if (t < EPS) break;
            if (cb.prec) {
               if (cb.solve(v, z)) return -1;
            }
            dotvz = std::sqrt(c.dot(v, z));
            if (dotvz < EPS) break;
            c.scale(v, alias ? nullptr : z, 1.0 / dotvz);
         }
         while (iter < wsize) {
            const int r = step(false);
            if (r < 0) return -1;
            if (r) break;
         }
      }
      *tsize = iter;
      *TDp = TD;
      *TEp = TE;
      return 0;
   }
};

int lanczos_dev(Callbacks& cb, double* x, const double* rhs, int wsize, int maxits, int atol, double tol,
                double* prel_res, double** prel_res_v, int* piter, int* tsize, double** TDp, double** TEp,
                int print_level)
{
   LanczosRun L(cb, x, wsize, maxits, atol, tol, print_level, TDp, TEp);
   const int r0 = L.init(rhs, prel_res, prel_res_v, piter);
   if (r0) return r0 < 0 ? -1 : 0;
   while (L.iter < L.maxits) {
      const int r = L.step(true);
      if (r < 0) return -1;
      if (r) break;
   }
   return L.finish(prel_res, prel_res_v, piter, tsize);
}

// Two quadrature probes' Lanczos runs in lockstep through their first loops: while both run, each step's
// two matvecs are one two-vector matvec (launch pair, Nfft4GPAmdAdditiveMatSymvMulti).  Each run computes
// what lanczos_dev computes (the two-vector kernels sum in a different order: rounding-level
// differences); run 0's finish (and any rand() draws of its restarts) comes before run 1's, as in the
// reference's probe order.
int lanczos_pair_dev(Callbacks& cb, double* const* x, const double* const* rhs, int maxits, int print_level,
                     double* prel_res, int* tsize, double** TD, double** TE)
{
   LanczosRun L0(cb, x[0], maxits, maxits, 0, DBL_EPSILON, print_level, &TD[0], &TE[0]);
   LanczosRun L1(cb, x[1], maxits, maxits, 0, DBL_EPSILON, print_level, &TD[1], &TE[1]);
   LanczosRun* R[2] = {&L0, &L1};
   double* relv[2] = {nullptr, nullptr};
   int piter[2] = {0, 0};
   int st[2];  // 0 running the first loop, 1 first loop over, 2 complete in init
   for (int k = 0; k < 2; k++) {
      const int r = R[k]->init(rhs[k], &prel_res[k], &relv[k], &piter[k]);
      if (r < 0) return -1;
      st[k] = r ? 2 : 0;
      if (r) tsize[k] = 0;
   }
   while (st[0] == 0 || st[1] == 0) {
      bool run[2];
      for (int k = 0; k < 2; k++) run[k] = st[k] == 0 && R[k]->iter < R[k]->maxits;
      for (int k = 0; k < 2; k++)
         if (st[k] == 0 && !run[k]) st[k] = 1;
      if (!run[0] && !run[1]) break;
      for (int k = 0; k < 2; k++)
         if (run[k]) R[k]->step_begin();
      if (run[0] && run[1]) {
         const double* xs[2] = {R[0]->wv, R[1]->wv};
         double* ys[2] = {R[0]->z, R[1]->z};
         if (additive_matvec_multi(cb.mat, 2, 1.0, xs, 0.0, ys)) return -1;
      } else {
         LanczosRun* Q = run[0] ? R[0] : R[1];
         if (cb.apply(1.0, Q->wv, 0.0, Q->z)) return -1;
      }
      if (run[0] && run[1] && R[0]->fast_ok(true) && R[1]->fast_ok(true)) {
         // both runs' scalars behind one read (each in its half of the scalar buffer)
         constexpr int kR = LanczosRun::kRegion;
         if (R[0]->step_enqueue(true, g_k.scal) || R[1]->step_enqueue(true, g_k.scal + kR)) return -1;
         std::vector<double> hh(kR + R[1]->region_len(true));
         if (R[0]->c.read(g_k.scal, (int)hh.size(), hh.data())) return -1;
         for (int k = 0; k < 2; k++) {
            const int r = R[k]->step_after(true, hh.data() + k * kR);
            if (r < 0) return -1;
            if (r) st[k] = 1;
         }
      } else {
         for (int k = 0; k < 2; k++) {
            if (!run[k]) continue;
            const int r = R[k]->step_end(true);
            if (r < 0) return -1;
            if (r) st[k] = 1;
         }
      }
   }
   for (int k = 0; k < 2; k++) {
      if (st[k] == 2) {
         free(relv[k]);
         continue;
      }
      if (R[k]->finish(&prel_res[k], &relv[k], &piter[k], &tsize[k])) return -1;
      free(relv[k]);
   }
   return 0;
}

// ---- stochastic Lanczos quadrature (lanczos.c:421-610) --------------------------------------------
int lanczos_logdet_dev(Callbacks& cb, Callbacks& dcb, func_trace tracefunc, func_logdet logdetfunc,
                       func_dvp dvpfunc, int maxits, int nvecs, const double* radamacher, int print_level,
                       double* logdet, double** dlogdetp)
{
   const size_t n = cb.n;
   const double nall = (double)cb.n_global;  // the 1/n normalisations use the whole problem's n
   Ctx c{current_stream(), n, cb.comm};
   void* prec_data = cb.prec ? cb.pdata : nullptr;
   double* dval = *dlogdetp ? *dlogdetp : (double*)calloc(3, sizeof(double));
   double traces_precond[3] = {0.0, 0.0, 0.0}, logdet_precond = 0.0;
   if (prec_data) {
      double* tp = traces_precond;
      if (tracefunc(prec_data, &tp)) return -1;
      for (int i = 0; i < 3; i++) traces_precond[i] /= nall;
      logdet_precond = logdetfunc(prec_data) / nall;
   }
   const bool dvp_dev = g_cb_mode == 1 || (g_cb_mode == -1 && library_operator((const void*)dvpfunc));
   double *z = nullptr, *x = nullptr, *dAz = nullptr, *px = nullptr;
   std::vector<double> hz, hpx;
   if (dmalloc(&z, n) || dmalloc(&x, n) || dmalloc(&dAz, 3 * n) || dmalloc(&px, 3 * n)) return -1;
   auto cleanup = [&]() {
      (void)hipStreamSynchronize(c.s);
      for (double* p : {z, x, dAz, px}) (void)hipFree(p);
   };
   const bool rad_dev = radamacher && is_device_ptr(radamacher);
   double val = 0.0;
   for (int j = 0; j < 3; j++) dval[j] = 0.0;
   // probe i's contribution from its Lanczos run (lanczos.c:525-567); 1: the reference's early return
   auto post = [&](int i, const double* zc, const double* xc, double* TD, double* TE, int tsize) -> int {
      if (dcb.apply(1.0, const_cast<double*>(zc), 0.0, dAz)) return -1;
      while (tsize > 0 && std::isnan(TD[tsize - 1])) tsize--;
      if (tsize == 0) {
         printf("Warning: empty tridiagonal matrix\n");  // lanczos.c:525-529 returns without a result
         return 1;
      }
      std::vector<double> w, TV;
      if (tridiag_eig(tsize, TD, TE, w, TV)) {
         printf("Warning: DSTEV failed at iteration %d/%d\n", i, nvecs);
         return -1;
      }
      // sum_j TV(0, j)^2 log|lambda_j|  (TV column-major, eigenvector j in column j)
      for (int j = 0; j < tsize; j++) val += TV[(size_t)j * tsize] * TV[(size_t)j * tsize] * std::log(std::fabs(w[j]));
      if (prec_data) {
         if (dvp_dev) {
            double* pp = px;
            if (dvpfunc(prec_data, (int)n, nullptr, const_cast<double*>(zc), &pp)) return -1;
         } else {
            hz.resize(n);
            hpx.assign(3 * n, 0.0);
            NFFT4GP_HIP_CHECK(hipMemcpy(hz.data(), zc, sizeof(double) * n, hipMemcpyDeviceToHost));
            double* pp = hpx.data();
            if (dvpfunc(prec_data, (int)n, nullptr, hz.data(), &pp)) return -1;
            NFFT4GP_HIP_CHECK(hipMemcpy(px, hpx.data(), sizeof(double) * 3 * n, hipMemcpyHostToDevice));
         }
      }
      for (int j = 0; j < 3; j++) {
         dval[j] += c.dot(dAz + (size_t)j * n, xc);
         if (prec_data) dval[j] -= c.dot(px + (size_t)j * n, zc);
      }
      return 0;
   };
   // two probes share their matvecs (lanczos_pair_dev) on this library's additive operator when the probes
   // are given (no rand() draws between them) and the runs print nothing per step
   const bool pairs = radamacher && print_level <= 0 && cb.mv_dev &&
                      cb.matvec == (func_symmatvec)&Nfft4GPAdditiveNFFTMatSymv;
   double *z2 = nullptr, *x2 = nullptr;
   if (pairs && nvecs > 1 && (dmalloc(&z2, n) || dmalloc(&x2, n))) {
      cleanup();
      return -1;
   }
   auto done = [&](int rc) {
      (void)hipStreamSynchronize(c.s);
      (void)hipFree(z2);
      (void)hipFree(x2);
      cleanup();
      return rc;
   };
   for (int i = 0; i < nvecs;) {
      if (pairs && i + 1 < nvecs) {
         double* zz[2] = {z, z2};
         double* xx[2] = {x, x2};
         for (int k = 0; k < 2; k++) {
            NFFT4GP_HIP_CHECK(hipMemcpyAsync(zz[k], radamacher + (size_t)(i + k) * n, sizeof(double) * n,
                                             rad_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c.s));
            NFFT4GP_HIP_CHECK(hipMemsetAsync(xx[k], 0, sizeof(double) * n, c.s));
         }
         double rel_res[2];
         int tsize[2] = {0, 0};
         double* TD[2] = {nullptr, nullptr};
         double* TE[2] = {nullptr, nullptr};
         const double* zc[2] = {z, z2};
         const int rc = lanczos_pair_dev(cb, xx, zc, maxits, print_level, rel_res, tsize, TD, TE);
         int pr = rc ? -1 : 0;
         for (int k = 0; k < 2 && pr == 0; k++) pr = post(i + k, zz[k], xx[k], TD[k], TE[k], tsize[k]);
         for (int k = 0; k < 2; k++) {
            free(TD[k]);
            free(TE[k]);
         }
         if (pr) return done(pr < 0 ? -1 : 0);
         i += 2;
         continue;
      }
      if (radamacher) {
         NFFT4GP_HIP_CHECK(hipMemcpyAsync(z, radamacher + (size_t)i * n, sizeof(double) * n,
                                          rad_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c.s));
      } else {
         // every rank draws the whole probe (the same libc sequence); a row shard keeps its rows
         hz.resize(cb.n_global);
         Nfft4GPVecRadamacher(hz.data(), (int)cb.n_global);
         NFFT4GP_HIP_CHECK(hipMemcpy(z, hz.data() + cb.row_begin, sizeof(double) * n, hipMemcpyHostToDevice));
      }
      NFFT4GP_HIP_CHECK(hipMemsetAsync(x, 0, sizeof(double) * n, c.s));
      double rel_res, *rel_res_v = nullptr, *TD = nullptr, *TE = nullptr;
      int niter = 0, tsize = 0;
      if (lanczos_dev(cb, x, z, maxits, maxits, 0, DBL_EPSILON, &rel_res, &rel_res_v, &niter, &tsize, &TD, &TE,
                      print_level))
         return done(-1);
      free(rel_res_v);
      const int pr = post(i, z, x, TD, TE, tsize);
      free(TD);
      free(TE);
      if (pr) return done(pr < 0 ? -1 : 0);
      i++;
   }
   (void)hipFree(z2);
   (void)hipFree(x2);
   cleanup();
   double scale = 1.0 / (double)nvecs;
   val *= scale;
   scale /= nall;
   for (int j = 0; j < 3; j++) dval[j] *= scale;
   val += logdet_precond;
   for (int j = 0; j < 3; j++) dval[j] += traces_precond[j];
   *logdet = val;
   if (!*dlogdetp) *dlogdetp = dval;
   return 0;
}

}  // namespace nfft4gp_amd

// ---------------------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------------------
namespace {

bool make_callbacks(Callbacks& cb, int n, func_symmatvec matvec, void* mat, func_solve prec, void* pdata)
{
   cb.matvec = matvec;
   cb.mat = mat;
   cb.prec = pdata ? prec : nullptr;  // the reference tests prec_data, not the function (fgmres.c:148)
   cb.pdata = pdata;
   cb.n = (size_t)n;
   cb.mv_dev = g_cb_mode == 1 || (g_cb_mode == -1 && library_operator((const void*)matvec));
   cb.pc_dev = g_cb_mode == 1 || (g_cb_mode == -1 && library_operator((const void*)prec));
   if (bind_dist(cb)) return false;
   return g_k.ensure() == 0;
}

}  // namespace

// Fault injection for tests/test_gpu_krylov.py: mode 1 sets the one-launch kernels' error word (the state a
// wait that gave up leaves) and re-enables them; mode 0 clears it and re-enables them.  Returns whether the
// one-launch sweeps were off (a wait had given up) before the call.
extern "C" int Nfft4GPAmdDebugChainFault(int mode)
{
   if (g_k.ensure_chain()) return -1;
   const int was_off = g_k.chain_off ? 1 : 0;
   (void)hipDeviceSynchronize();
   const int v = mode ? 1 : 0;
   NFFT4GP_HIP_CHECK(hipMemcpy(g_k.chain + 1, &v, sizeof(int), hipMemcpyHostToDevice));
   *g_k.hchain_err = 0;
   g_k.chain_off = false;
   return was_off;
}

// Timing probe for tools/reorth_probe.py: `reps` classical Gram-Schmidt passes (Ctx::block_gs, the Lanczos
// re-orthogonalisation's pass) of the device vector w against m device columns V (dots) / Z (updates) on the
// library's stream; *ms = average pass time (hipEvents), h_out (m + 2 doubles, optional) = the last pass's scalars
extern "C" int Nfft4GPAmdDebugBlockGs(double* w, const double* V, const double* Z, long long n, int m, int with_norm,
                                      int reps, float* ms, double* h_out)
{
   if (!need_device("Nfft4GPAmdDebugBlockGs") || n <= 0 || m <= 0 || reps <= 0 || g_k.ensure()) return -1;
   Ctx c{current_stream(), (size_t)n, nullptr};
   hipEvent_t e0, e1;
   NFFT4GP_HIP_CHECK(hipEventCreate(&e0));
   NFFT4GP_HIP_CHECK(hipEventCreate(&e1));
   int rc = c.block_gs(w, V, Z, m, g_k.scal, with_norm);  // warm-up
   NFFT4GP_HIP_CHECK(hipEventRecord(e0, c.s));
   for (int r = 0; r < reps && rc == 0; r++) rc = c.block_gs(w, V, Z, m, g_k.scal, with_norm);
   NFFT4GP_HIP_CHECK(hipEventRecord(e1, c.s));
   NFFT4GP_HIP_CHECK(hipEventSynchronize(e1));
   float t = 0.f;
   NFFT4GP_HIP_CHECK(hipEventElapsedTime(&t, e0, e1));
   if (ms) *ms = t / reps;
   (void)hipEventDestroy(e0);
   (void)hipEventDestroy(e1);
   if (rc == 0 && h_out) rc = c.read(g_k.scal, m + 2, h_out);
   return rc;
}

extern "C" {

void Nfft4GPAmdSetFgmresOrtho(int ortho) { g_fgmres_ortho = (ortho == 1 || ortho == 2) ? ortho : 0; }

// the second classical passes FGMRES (ortho 1) has taken since the last call (its DGKS test), then reset
long long Nfft4GPAmdFgmresSecondPasses(void)
{
   const long long v = g_fgmres_second_passes;
   g_fgmres_second_passes = 0;
   return v;
}

int Nfft4GPSolverFgmres(void* mat_data, int n, func_symmatvec matvec, void* prec_data, func_solve precondfunc,
                        double* x, double* rhs, int kdim, int maxits, int atol, double tol, double* prel_res,
                        double** prel_res_v, int* piter, int print_level)
{
   if (!need_device("Nfft4GPSolverFgmres")) return -1;
   Callbacks cb;
   if (!make_callbacks(cb, n, matvec, mat_data, precondfunc, prec_data)) return -1;
   Vec vx, vb;
   if (vx.open(x, n, true) || vb.open(rhs, n, true)) return -1;
   int rc = fgmres_dev(cb, vx.d, vb.d, kdim, maxits, atol, tol, prel_res, prel_res_v, piter, print_level);
   if (rc == 0 && dist_final_check(cb)) rc = -1;
   vb.close(false);
   vx.close(rc == 0);
   return rc;
}

int Nfft4GPSolverLanczos(void* mat_data, int n, func_symmatvec matvec, void* prec_data, func_solve precondfunc,
                         double* x, double* rhs, int wsize, int maxits, int atol, double tol, double* prel_res,
                         double** prel_res_v, int* piter, int* tsize, double** TDp, double** TEp, int print_level)
{
   RandScope rand_scope;  // libc rand() as the reference draws it (internal.h)
   if (!need_device("Nfft4GPSolverLanczos")) return -1;
   Callbacks cb;
   if (!make_callbacks(cb, n, matvec, mat_data, precondfunc, prec_data)) return -1;
   Vec vx, vb;
   if (vx.open(x, n, true) || vb.open(rhs, n, true)) return -1;
   int rc = lanczos_dev(cb, vx.d, vb.d, wsize, maxits, atol, tol, prel_res, prel_res_v, piter, tsize, TDp, TEp,
                        print_level);
   if (rc == 0 && dist_final_check(cb)) rc = -1;
   vb.close(false);
   vx.close(rc == 0);
   return rc;
}

int Nfft4GPLanczosQuadratureLogdet(void* mat_data, void* dmat_data, int n, func_symmatvec matvec,
                                   func_symmatvec dmatvec, void* prec_data, func_solve precondfunc,
                                   func_trace tracefunc, func_logdet logdetfunc, func_dvp dvpfunc, int maxits,
                                   int nvecs, double* radamacher, int print_level, double* logdet, double** dlogdetp)
{
   RandScope rand_scope;  // libc rand() as the reference draws it (internal.h)
   if (!need_device("Nfft4GPLanczosQuadratureLogdet")) return -1;
   Callbacks cb, dcb;
   if (!make_callbacks(cb, n, matvec, mat_data, precondfunc, prec_data) ||
       !make_callbacks(dcb, n, dmatvec, dmat_data, nullptr, nullptr))
      return -1;
   dcb.out_mult = 3;
   const int rc = lanczos_logdet_dev(cb, dcb, tracefunc, logdetfunc, dvpfunc, maxits, nvecs, radamacher, print_level,
                                     logdet, dlogdetp);
   return rc == 0 && dist_final_check(cb) ? -1 : rc;
}

int Nfft4GPTransform(nfft4gp_transform_type type, double val, int inverse, double* tvalp, double* dtvalp)
{
   switch (type) {
   case 1:  // NFFT4GP_TRANSFORM_SIGMOID
      if (!inverse) {
         *tvalp = 1.0 / (exp(-val) + 1.0);
         *dtvalp = *tvalp * (1 - *tvalp);
      } else {
         *tvalp = log(val / (1.0 - val));
      }
      break;
   case 0:  // NFFT4GP_TRANSFORM_SOFTPLUS
      if (!inverse) {
         if (val > 20.0) {
            *tvalp = val;
            *dtvalp = 1.0;
         } else if (val < -20.0) {
            *tvalp = exp(val);
            *dtvalp = exp(val);
         } else {
            *tvalp = log(1.0 + exp(val));
            *dtvalp = exp(val) / (1.0 + exp(val));
         }
      } else {
         if (val > 20.0)
            *tvalp = val;
         else if (val < 2.06115362243856e-09)
            *tvalp = log(val);
         else
            *tvalp = log(exp(val) - 1.0);
      }
      break;
   case 2:  // NFFT4GP_TRANSFORM_EXP
      if (!inverse) {
         *tvalp = exp(val);
         *dtvalp = exp(val);
      } else {
         *tvalp = log(val);
      }
      break;
   case 3:  // NFFT4GP_TRANSFORM_IDENTITY
      *tvalp = val;
      if (!inverse) *dtvalp = 1.0;
      break;
   default:
      printf("Error: unknown transform type.\n");
      return -1;
   }
   return 0;
}

int Nfft4GPGpLoss(double* x, double* data, double* label, int n, int ldim, int d, func_kernel fkernel,
                  void* vfkernel_data, func_free kernel_data_free, func_symmatvec matvec, func_symmatvec dmatvec,
                  func_kernel precond_fkernel, void* precond_vfkernel_data, func_free precond_vfkernel_data_free,
                  precond_kernel_setup precond_setup, func_solve precond_solve, func_trace precond_trace,
                  func_logdet precond_logdet, func_dvp precond_dvp, func_free precond_reset, void* precond_data,
                  int atol, double tol, int wsize, int maxits, int nvecs, double* radamacher,
                  nfft4gp_transform_type transform,
                  int* mask, int print_level, double* dwork, double* loss, double* grad)
{
   RandScope rand_scope;  // libc rand() as the reference draws it (internal.h)
   (void)precond_vfkernel_data_free;
   (void)wsize;
   if (!need_device("Nfft4GPGpLoss")) return -1;
   double tvals[3], dtvals[3];
   for (int i = 0; i < 3; i++)
      if (Nfft4GPTransform(transform, x[i], 0, tvals + i, dtvals + i)) return -1;
   printf("Transform %e %e %e into %e %e %e with grad %e %e %e\n", x[0], x[1], x[2], tvals[0], tvals[1], tvals[2],
          dtvals[0], dtvals[1], dtvals[2]);
   nfft4gp_kernel* kd = (nfft4gp_kernel*)vfkernel_data;
   nfft4gp_kernel* pkd = (nfft4gp_kernel*)precond_vfkernel_data;
   kd->_params[0] = tvals[0];
   kd->_params[1] = tvals[1];
   kd->_noise_level = tvals[2];
   if (pkd) {
      pkd->_params[0] = tvals[0];
      pkd->_params[1] = tvals[1];
      pkd->_noise_level = tvals[2];
   }
   double* kernel_mat = nullptr;
   double* dkernel_mat = nullptr;
   if (dwork) {
      kernel_mat = dwork;
      dkernel_mat = dwork + (size_t)n * n;
   }
   if (fkernel(vfkernel_data, data, n, ldim, d, nullptr, 0, nullptr, 0, &kernel_mat, &dkernel_mat)) return -1;
   if (precond_setup)
      precond_setup(data, n, ldim, d, precond_fkernel, precond_vfkernel_data, 1, precond_data);
   else
      precond_data = nullptr;

   Callbacks cb, dcb;
   if (!make_callbacks(cb, n, matvec, kernel_mat, precond_solve, precond_data) ||
       !make_callbacks(dcb, n, dmatvec, dkernel_mat, nullptr, nullptr))
      return -1;
   dcb.out_mult = 3;
   if (cb.comm != dcb.comm || cb.n_global != dcb.n_global) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPGpLoss: matvec and dmatvec must be split the same way\n");
      return -1;
   }
   const int nall = (int)cb.n_global;  // n of the whole problem (a row shard holds n of its rows)
   hipStream_t s = current_stream();
   Ctx c{s, (size_t)n, cb.comm};
   double *iKY = nullptr, *dKiKY = nullptr;
   Vec vl;
   if (dmalloc(&iKY, (size_t)n) || dmalloc(&dKiKY, 3 * (size_t)n) || vl.open(label, n, true)) return -1;
   NFFT4GP_HIP_CHECK(hipMemsetAsync(iKY, 0, sizeof(double) * n, s));
   const int solve_kdim = std::min(nall, maxits * 2), solve_maxits = std::min(nall, maxits * 2);
   double rel_res, *rel_res_v = nullptr;
   int niter = 0;
   if (fgmres_dev(cb, iKY, vl.d, solve_kdim, solve_maxits, atol, tol, &rel_res, &rel_res_v, &niter, print_level))
      return -1;
   if (rel_res > 1e10) {
      printf("Warning: FGMRES unstable, rel_res = %f\n", rel_res);
      printf("Current parameters (after transform): f = %f, l = %f, mu = %f\n", tvals[0], tvals[1], tvals[2]);
   }
   free(rel_res_v);
   const double L1 = c.dot(vl.d, iKY) / (double)nall;
   if (dcb.apply(1.0, iKY, 0.0, dKiKY)) return -1;
   double L1_grad[3];
   for (int i = 0; i < 3; i++) L1_grad[i] = c.dot(dKiKY + (size_t)i * n, iKY) / (double)nall * dtvals[i];
   double L2 = 0.0, *L2_grad = nullptr;
   const int qits = std::min(nall, maxits);
   const int err = lanczos_logdet_dev(cb, dcb, precond_trace, precond_logdet, precond_dvp, qits, nvecs, radamacher,
                                      print_level, &L2, &L2_grad);
   (void)hipStreamSynchronize(s);
   (void)hipFree(iKY);
   (void)hipFree(dKiKY);
   vl.close(false);
   if (err != 0) {
      printf("Error in Nfft4GPLanczosQuadratureLogdet\n");
      return err;
   }
   if (dist_final_check(cb)) {
      free(L2_grad);
      return -1;
   }
   loss[0] = 0.5 * (L1 + L2 + log(2.0 * 3.1415926535897932384626));
   for (int i = 0; i < 3; i++) {
      const double g = L2_grad ? 0.5 * (-L1_grad[i] + L2_grad[i] * dtvals[i]) : 0.0;
      grad[i] = (mask && !mask[i]) ? 0.0 : g;
   }
   free(L2_grad);
   if (!dwork && kernel_data_free) {
      kernel_data_free(kernel_mat);
      kernel_data_free(dkernel_mat);
   }
   if (precond_data && precond_reset) precond_reset(precond_data);
   return 0;
}

int Nfft4GPAdditiveNFFTGpPredict(double* x, double* data, double* label, int n, int ldim, int d,
                                 double* data_predict, int n_predict, int ldim_predict, double* data_all,
                                 func_kernel fkernel, void* vfkernel_data, void* vfkernel_data_l,
                                 func_free kernel_data_free, func_symmatvec matvec, func_kernel precond_fkernel,
                                 void* precond_vfkernel_data, func_free precond_kernel_data_free,
                                 precond_kernel_setup precond_setup, func_solve precond_solve, void* precond_data,
                                 int atol, double tol, int maxits, nfft4gp_transform_type transform,
                                 int print_level, double* dwork, double** label_predictp, double** std_predictp)
{
   (void)data_predict, (void)ldim_predict, (void)kernel_data_free, (void)precond_kernel_data_free, (void)dwork;
   if (!need_device("Nfft4GPAdditiveNFFTGpPredict")) return -1;
   double tvals[3], dtvals[3];
   for (int i = 0; i < 3; i++)
      if (Nfft4GPTransform(transform, x[i], 0, tvals + i, dtvals + i)) return -1;
   nfft4gp_kernel* kd = (nfft4gp_kernel*)vfkernel_data;
   nfft4gp_kernel* kl = (nfft4gp_kernel*)vfkernel_data_l;
   for (nfft4gp_kernel* k : {kd, kl}) {
      k->_params[0] = tvals[0];
      k->_params[1] = tvals[1];
      k->_noise_level = tvals[2];
   }
   double *K11 = nullptr, *dK11 = nullptr, *K = nullptr, *dK = nullptr;
   const int na = n + n_predict;
   if (fkernel(vfkernel_data, data, n, ldim, d, nullptr, 0, nullptr, 0, &K11, &dK11) ||
       fkernel(vfkernel_data_l, data_all, na, na, d, nullptr, 0, nullptr, 0, &K, &dK))
      return -1;
   if (precond_setup)
      precond_setup(data, n, ldim, d, precond_fkernel, precond_vfkernel_data, 1, precond_data);
   else
      precond_data = nullptr;
   Callbacks cb11, cba;
   if (!make_callbacks(cb11, n, matvec, K11, precond_solve, precond_data) ||
       !make_callbacks(cba, na, matvec, K, nullptr, nullptr))
      return -1;
   if (cb11.n_global != cb11.n || cb11.comm) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAdditiveNFFTGpPredict takes a one-GPU operator\n");
      return -1;
   }
   hipStream_t s = current_stream();
   Ctx c{s, (size_t)n};
   double *iKY = nullptr, *helper = nullptr;
   Vec vl;
   if (dmalloc(&iKY, (size_t)na) || dmalloc(&helper, (size_t)na) || vl.open(label, n, true)) return -1;
   auto cleanup = [&]() {
      (void)hipStreamSynchronize(s);
      (void)hipFree(iKY);
      (void)hipFree(helper);
      vl.close(false);
   };
   NFFT4GP_HIP_CHECK(hipMemsetAsync(iKY, 0, sizeof(double) * na, s));
   double rel_res, *rel_res_v = nullptr;
   int niter = 0;
   if (fgmres_dev(cb11, iKY, vl.d, maxits, maxits, atol, tol, &rel_res, &rel_res_v, &niter, print_level)) {
      cleanup();
      return -1;
   }
   free(rel_res_v);
   // label_predict = (K_all [iKY; 0])[n:]  (nfft_interface.c:973-979)
   if (cba.apply(1.0, iKY, 0.0, helper)) {
      cleanup();
      return -1;
   }
   double* lp = *label_predictp ? *label_predictp : (double*)malloc(sizeof(double) * std::max(1, n_predict));
   const bool lp_dev = is_device_ptr(lp);
   NFFT4GP_HIP_CHECK(hipMemcpyAsync(lp, helper + n, sizeof(double) * n_predict,
                                    lp_dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
   NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
   if (!*label_predictp) *label_predictp = lp;
   if (std_predictp) {
      // diag of K22 - K21 K11^{-1} K12 (nfft_interface.c:993-1060), a batch of prediction points at a time:
      // the K12 columns and K22 diagonal entries of the batch by one operator application to its unit vectors
      // (two per pass on this library's operator), then its solves K11 x = K12(:, i) in lockstep
      // (fgmres_batch_dev: restart dimension and iteration limit n as the reference), then the dots
      double* sp = *std_predictp ? *std_predictp : (double*)malloc(sizeof(double) * std::max(1, n_predict));
      std::vector<double> hs(n_predict);
      // 32 points per batch up to n = 2^18 (0.077 against 0.108 s for 16 at n = 20 000, 0.366 against 0.417 s at
      // n = 200 000: profiles/r05_predict_std_batch.txt), 16 above (each basis column holds batch x n doubles)
      int bm = n <= (1 << 18) ? 32 : 16;
      if (const char* e = getenv("NFFT4GP_AMD_PREDICT_BATCH")) bm = std::max(1, std::min(256, atoi(e)));
      bm = std::max(1, std::min(bm, n_predict));
      double *E = nullptr, *Y = nullptr, *Xs = nullptr, *dsc = nullptr;
      int* dall = nullptr;
      auto bfree = [&]() {
         (void)hipStreamSynchronize(s);
         (void)hipFree(E);
         (void)hipFree(Y);
         (void)hipFree(Xs);
         (void)hipFree(dsc);
         (void)hipFree(dall);
      };
      if (dmalloc(&E, (size_t)na * bm) || dmalloc(&Y, (size_t)na * bm) || dmalloc(&Xs, (size_t)n * bm) ||
          dmalloc(&dsc, 2 * (size_t)bm) || dmalloc(&dall, bm)) {
         bfree();
         cleanup();
         return -1;
      }
      const bool multi = cba.mv_dev && cba.matvec == (func_symmatvec)&Nfft4GPAdditiveNFFTMatSymv;
      {
         std::vector<int> ids(bm);
         for (int k = 0; k < bm; k++) ids[k] = k;
         NFFT4GP_HIP_CHECK(hipMemcpy(dall, ids.data(), sizeof(int) * bm, hipMemcpyHostToDevice));
      }
      double* gpart = nullptr;
      unsigned int* gtick = nullptr;
      if (dmalloc(&gpart, (size_t)bm * kKMaxBlocks) || dmalloc(&gtick, (size_t)bm * kTicketWords)) {
         (void)hipFree(gpart);
         bfree();
         cleanup();
         return -1;
      }
      NFFT4GP_HIP_CHECK(hipMemsetAsync(gtick, 0, sizeof(unsigned int) * (size_t)bm * kTicketWords, s));
      int rc = 0;
      for (int i0 = 0; i0 < n_predict && !rc; i0 += bm) {
         const int mb = std::min(bm, n_predict - i0);
         NFFT4GP_HIP_CHECK(hipMemsetAsync(E, 0, sizeof(double) * (size_t)na * mb, s));
         hipLaunchKernelGGL(k_set_units, dim3((mb + 255) / 256), dim3(256), 0, s, E, (size_t)na, (size_t)(n + i0), mb);
         std::vector<const double*> xs(mb);
         std::vector<double*> ys(mb);
         for (int k = 0; k < mb; k++) {
            xs[k] = E + (size_t)k * na;
            ys[k] = Y + (size_t)k * na;
         }
         if (multi) {
            rc = additive_matvec_multi(cba.mat, mb, 1.0, xs.data(), 0.0, ys.data());
         } else {
            for (int k = 0; k < mb && !rc; k++) rc = cba.apply(1.0, const_cast<double*>(xs[k]), 0.0, ys[k]);
         }
         if (rc) break;
         hipLaunchKernelGGL(k_pick_diag, dim3((mb + 255) / 256), dim3(256), 0, s, dsc, (const double*)Y, (size_t)na,
                            (size_t)(n + i0), mb);
         BatchOut bo;
         if ((rc = fgmres_batch_dev(cb11, mb, Xs, (size_t)n, Y, (size_t)na, n, n, atol, tol, print_level, bo))) break;
         // (K12(:, i), x_i) per point: k_gs_step's dot, batched
         const unsigned gg = (unsigned)std::max<size_t>(1, std::min<size_t>(((size_t)n + 4095) / 4096, kKMaxBlocks));
         hipLaunchKernelGGL((k_gs_batch<1024, 4>), dim3(gg, (unsigned)mb), dim3(1024), 0, s, Y, (size_t)na,
                            (const double*)nullptr, (size_t)0, (const double*)nullptr, (const double*)Xs, (size_t)n,
                            (size_t)n, (const int*)dall, gpart, gtick, dsc + bm);
         NFFT4GP_HIP_CHECK(hipGetLastError());
         std::vector<double> h2(2 * (size_t)bm);
         if ((rc = c.read(dsc, 2 * bm, h2.data()))) break;
         for (int k = 0; k < mb; k++) hs[i0 + k] = std::sqrt(std::fabs(h2[k] - h2[bm + k]));
      }
      (void)hipStreamSynchronize(s);
      (void)hipFree(gpart);
      (void)hipFree(gtick);
      bfree();
      if (rc) {
         if (!*std_predictp) free(sp);
         cleanup();
         return -1;
      }
      if (is_device_ptr(sp))
         NFFT4GP_HIP_CHECK(hipMemcpy(sp, hs.data(), sizeof(double) * n_predict, hipMemcpyHostToDevice));
      else
         memcpy(sp, hs.data(), sizeof(double) * n_predict);
      if (!*std_predictp) *std_predictp = sp;
   }
   cleanup();
   return 0;
}

}  // extern "C"
