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
#include "callbacks.hpp"
#include "reduce.hpp"

using namespace nfft4gp_amd;

namespace nfft4gp_amd {
void nys_free(NysDev* N)
{
   if (!N) return;
   (void)hipStreamSynchronize(current_stream());
   for (double* p : {N->U, N->s, N->w, N->part, N->Kall, N->dU, N->G, N->Gt, N->GdKG, N->D, N->vk, N->vn})
      (void)hipFree(p);
   (void)hipFree(N->Uf);
   delete N;
}

int nys_alloc_scratch(NysDev* N)
{
   N->nblk = (N->n + kNysRows - 1) / kNysRows;
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&N->w, sizeof(double) * std::max(1, N->k)));
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&N->part, sizeof(double) * (size_t)N->nblk * std::max(1, N->k)));
   return 0;
}
}  // namespace nfft4gp_amd

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

// ---------------------------------------------------------------------------------------------
// Device-controlled PCG (pcg.c:3-206).  The iteration's scalars (rho, pq, ||r||) and its control
// decisions (the rho/beta/pq breakdown tests and the convergence test) live on the device, so the
// host enqueues iterations back to back and only polls a status slot in pinned host memory a few
// iterations behind.  Once a kernel flags a stop, every later PCG kernel of the launched-ahead
// iterations is a no-op, so the state the host finds is exactly the state at the flagged iteration.
// ---------------------------------------------------------------------------------------------
struct PcgState {
   double normb, tolb, pq, normr2;
   int status;     // 0 running, 1 converged candidate, 2 rho == 0, 3 beta == 0, 4 pq <= 0, 5 k_pcg_xr's
                   // in-kernel wait gave up (an error)
   int flag_iter;  // iteration that set status
   double loc[2];  // distributed PCG: this rank's partial dot (0) / ||r||^2 (1), all-reduced in place
   double beta_next;  // FUSEP k_pcg_xr: the next iteration's beta, handed from the last workgroup to the others
   int bar;           // FUSEP k_pcg_xr: +ii (apply beta) / -ii (no update) once beta_next is stored
   int pad;
};

struct PcgSlot {   // pinned host memory, written by the last kernel of each iteration
   double normr;
   int status, flag_iter, seq, pad;
};

// PCG vector kernels: kEPT independent elements per thread (all loads issued before use), so each
// lane keeps several HBM requests in flight; grid = ceil(n / (kVecThreads * kEPT)) <= kPcgMaxBlocks.
constexpr int kEPT = 4;
constexpr int kPcgMaxBlocks = 2048;  // <= kRedMaxBlocks (reduce.hpp)

int pcg_grid(size_t n)
{
   size_t g = (n + (size_t)kVecThreads * kEPT - 1) / ((size_t)kVecThreads * kEPT);
   if (g > (size_t)kPcgMaxBlocks) g = kPcgMaxBlocks;
   return (int)(g == 0 ? 1 : g);
}

// which = 0: rhos[ii] = (z, r) with the rho == 0 test;  which = 1: pq = (q, p) with the pq <= 0 test
__device__ void pcg_dot_store(double tot, PcgState* st, double* __restrict__ rhos, int ii, int which)
{
   if (which == 0) {
      rhos[ii] = tot;
      if (tot == 0.0) { st->status = 2; st->flag_iter = ii; }
   } else {
      st->pq = tot;
      if (tot <= 0.0) { st->status = 4; st->flag_iter = ii; }
   }
}

// loc != NULL (distributed PCG): only this rank's partial is written there; k_pcg_dot_fin applies it after
// the all-reduce
__global__ __launch_bounds__(kVecThreads) void k_pcg_dot(const double* __restrict__ a, const double* __restrict__ b,
                                                         size_t n, double* __restrict__ part,
                                                         unsigned int* __restrict__ ticket, PcgState* st,
                                                         double* __restrict__ rhos, int ii, int which,
                                                         double* __restrict__ loc)
{
   if (st->status) return;
   double acc = 0.0;
   const size_t stride = (size_t)gridDim.x * kVecThreads * kEPT;
   for (size_t i0 = (size_t)blockIdx.x * kVecThreads * kEPT + threadIdx.x; i0 < n; i0 += stride) {
      double av[kEPT], bv[kEPT];
#pragma unroll
      for (int u = 0; u < kEPT; u++) {
         const size_t i = i0 + (size_t)u * kVecThreads;
         av[u] = i < n ? a[i] : 0.0;
         bv[u] = i < n ? b[i] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < kEPT; u++) acc = fma(av[u], bv[u], acc);
   }
   acc = block_sum0<kVecThreads>(acc);
   double tot;
   if (!grid_total<kVecThreads>(acc, part, ticket, &tot) || threadIdx.x != 0) return;
   if (loc) {
      *loc = tot;
      return;
   }
   pcg_dot_store(tot, st, rhos, ii, which);
}

__global__ void k_pcg_dot_fin(PcgState* st, double* __restrict__ rhos, int ii, int which, const double* __restrict__ loc)
{
   if (threadIdx.x == 0 && !st->status) pcg_dot_store(*loc, st, rhos, ii, which);
}

// p = z (ii == 1) or p = beta p + z, beta = rhos[ii]/rhos[ii-1] (pcg.c:131-147: Scale then Axpy)
__global__ __launch_bounds__(kVecThreads) void k_pcg_pupdate(double* __restrict__ p, const double* __restrict__ z,
                                                             size_t n, PcgState* st, const double* __restrict__ rhos,
                                                             int ii)
{
   if (st->status) return;
   const double rho = rhos[ii];
   if (rho == 0.0) {  // no-preconditioner path: rho came from the previous iteration's norm
      if (blockIdx.x == 0 && threadIdx.x == 0) { st->status = 2; st->flag_iter = ii; }
      return;
   }
   double beta = 0.0;
   if (ii > 1) {
      beta = rho / rhos[ii - 1];
      if (beta == 0.0) {
         if (blockIdx.x == 0 && threadIdx.x == 0) { st->status = 3; st->flag_iter = ii; }
         return;
      }
   }
   const size_t stride = (size_t)gridDim.x * kVecThreads * kEPT;
   for (size_t i0 = (size_t)blockIdx.x * kVecThreads * kEPT + threadIdx.x; i0 < n; i0 += stride) {
      double pv[kEPT], zv[kEPT];
#pragma unroll
      for (int u = 0; u < kEPT; u++) {
         const size_t i = i0 + (size_t)u * kVecThreads;
         zv[u] = i < n ? z[i] : 0.0;
         pv[u] = (ii > 1 && i < n) ? p[i] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < kEPT; u++) {
         const size_t i = i0 + (size_t)u * kVecThreads;
         if (i < n) p[i] = (ii > 1) ? beta * pv[u] + zv[u] : zv[u];
      }
   }
}

__device__ void pcg_slot_write(const PcgState* st, PcgSlot* slot, double normr, int ii)
{
   slot->normr = normr;
   slot->status = st->status;
   slot->flag_iter = st->flag_iter;
   __hip_atomic_store(&slot->seq, ii, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ||r||^2 = tot of iteration ii: history, next rho (no preconditioner), convergence test, status slot
__device__ void pcg_xr_tail(double tot, PcgState* st, double* __restrict__ rhos, double* __restrict__ hist, int ii,
                            int rho_from_norm, PcgSlot* slot)
{
   const double normr = sqrt(tot);
   st->normr2 = normr;
   hist[ii] = normr / st->normb;
   if (rho_from_norm) rhos[ii + 1] = tot;  // z = r next iteration: rho = (r, r)
   if (normr <= st->tolb) { st->status = 1; st->flag_iter = ii; }
   pcg_slot_write(st, slot, normr, ii);
}

// x += alpha p ; r -= alpha q ; ||r|| ; convergence test ; status slot  (pcg.c:168-182).  T = 1024: a
// quarter of the block partials for the last block (the MGS step's measurement, krylov.hip)
// FUSEP (no preconditioner, one GPU, every element in the first pass of a grid that is resident at once): also
// the next iteration's direction update p = beta p + r (k_pcg_pupdate of ii + 1, with its rho == 0 / beta == 0
// tests) from the p and r values still in registers.  The last workgroup, which has ||r||^2, hands beta to
// the others through st (agent-scope stores and loads, as reduce.hpp's partials); they wait for it, boundedly.
template <int T, bool FUSEP = false>
__global__ __launch_bounds__(T) void k_pcg_xr(double* __restrict__ x, double* __restrict__ r,
                                                        double* __restrict__ p, const double* __restrict__ q,
                                                        size_t n, double* __restrict__ part,
                                                        unsigned int* __restrict__ ticket, PcgState* st,
                                                        double* __restrict__ rhos, double* __restrict__ hist, int ii,
                                                        int rho_from_norm, int check_pq, PcgSlot* slot,
                                                        double* __restrict__ loc, int do_p = 0)
{
   // loc != NULL (distributed PCG): the local ||r||^2 goes to *loc and k_pcg_xr_fin, after the all-reduce,
   // makes the convergence test and writes the status slot
   // check_pq: (q, p) came from the fused matvec-dot, so the pq <= 0 breakdown test (pcg.c:158) is here
   const int status = st->status ? st->status : ((check_pq && st->pq <= 0.0) ? 4 : 0);
   if (status) {
      if (blockIdx.x == 0 && threadIdx.x == 0) {
         if (!st->status) {
            st->status = status;
            st->flag_iter = ii;
         }
         if (!loc) pcg_slot_write(st, slot, st->normr2, ii);
      }
      return;
   }
   const double a = rhos[ii] / st->pq;
   double acc = 0.0;
   double p_keep[kEPT], r_keep[kEPT];  // FUSEP: this thread's (single pass) p and new r
   const size_t stride = (size_t)gridDim.x * T * kEPT;
   for (size_t i0 = (size_t)blockIdx.x * T * kEPT + threadIdx.x; i0 < n; i0 += stride) {
      double xv[kEPT], rv[kEPT], pv[kEPT], qv[kEPT];
#pragma unroll
      for (int u = 0; u < kEPT; u++) {
         const size_t i = i0 + (size_t)u * T;
         const bool ok = i < n;
         xv[u] = ok ? x[i] : 0.0;
         rv[u] = ok ? r[i] : 0.0;
         pv[u] = ok ? p[i] : 0.0;
         qv[u] = ok ? q[i] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < kEPT; u++) {
         const size_t i = i0 + (size_t)u * T;
         const double xi = xv[u] + a * pv[u];
         const double ri = rv[u] + (-a) * qv[u];
         acc = fma(ri, ri, acc);
         if (FUSEP) {
            p_keep[u] = pv[u];
            r_keep[u] = ri;
         }
         if (i < n) {
            x[i] = xi;
            r[i] = ri;
         }
      }
   }
   acc = block_sum0<T>(acc);
   double tot;
   if constexpr (!FUSEP) {
      if (!grid_total<T>(acc, part, ticket, &tot) || threadIdx.x != 0) return;
      if (loc) {
         *loc = tot;
         return;
      }
      pcg_xr_tail(tot, st, rhos, hist, ii, rho_from_norm, slot);
   } else {
      __shared__ double s_beta;
      __shared__ int s_go;
      if (grid_total<T>(acc, part, ticket, &tot)) {
         if (threadIdx.x == 0) {
            // pcg_xr_tail's bookkeeping, with the status slot (a system-scope release: an L2 write-back) written
            // after the others are released, and the next iteration's tests (k_pcg_pupdate's) in between
            const double normr = sqrt(tot);
            st->normr2 = normr;
            hist[ii] = normr / st->normb;
            rhos[ii + 1] = tot;  // z = r next iteration: rho = (r, r)
            const int stat_ii = normr <= st->tolb ? 1 : 0;
            if (stat_ii) {
               st->status = 1;
               st->flag_iter = ii;
            }
            int go = 0;
            double beta = 0.0;
            if (do_p && !stat_ii) {
               const double rho = tot;
               beta = rho / rhos[ii];
               if (rho == 0.0) {
                  st->status = 2;
                  st->flag_iter = ii + 1;
               } else if (beta == 0.0) {
                  st->status = 3;
                  st->flag_iter = ii + 1;
               } else {
                  go = 1;
               }
            }
            __hip_atomic_store(&st->beta_next, beta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(&st->bar, go ? ii : -ii, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_beta = beta;
            s_go = go;
            // slot ii as pcg_slot_write leaves it (status of iteration ii; 2 / 3 belong to ii + 1's slot)
            slot->normr = normr;
            slot->status = stat_ii;
            slot->flag_iter = ii;
            __hip_atomic_store(&slot->seq, ii, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
         }
      } else if (threadIdx.x == 0) {
         int b = 0;
         for (long spin = 0; spin < (1l << 22); spin++) {
            b = __hip_atomic_load(&st->bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (b == ii || b == -ii) break;
            __builtin_amdgcn_s_sleep(2);
         }
         if (b == ii) {
            s_beta = __hip_atomic_load(&st->beta_next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_go = 1;
         } else {
            s_go = 0;
            if (b != -ii) {  // the last workgroup never arrived: fail loudly (host: status 5)
               __hip_atomic_store(&st->status, 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
               __hip_atomic_store(&st->flag_iter, ii, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
         }
      }
      __syncthreads();
      if (!s_go) return;
      const double beta = s_beta;
      // k_pcg_pupdate's update for this thread's elements (the grid covers n in one pass: i0 < T kEPT gridDim.x)
      const size_t i0 = (size_t)blockIdx.x * T * kEPT + threadIdx.x;
#pragma unroll
      for (int u = 0; u < kEPT; u++) {
         const size_t i = i0 + (size_t)u * T;
         if (i < n) p[i] = beta * p_keep[u] + r_keep[u];
      }
   }
}

__global__ void k_pcg_xr_fin(PcgState* st, double* __restrict__ rhos, double* __restrict__ hist, int ii,
                             int rho_from_norm, PcgSlot* slot, const double* __restrict__ loc)
{
   if (threadIdx.x != 0) return;
   if (st->status)
      pcg_slot_write(st, slot, st->normr2, ii);
   else
      pcg_xr_tail(*loc, st, rhos, hist, ii, rho_from_norm, slot);
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

// comm != NULL: the local dot summed over the ranks (row-sharded vectors)
int dev_dot(const double* x, const double* y, size_t n, double* out, Comm* comm = nullptr)
{
   if (g_red.ensure()) return -1;
   hipStream_t s = current_stream();
   const int g = grid_for(n);
   hipLaunchKernelGGL(k_dot_partial, dim3(g), dim3(kVecThreads), 0, s, x, y, n, g_red.part);
   hipLaunchKernelGGL(k_sum_final, dim3(1), dim3(kVecThreads), 0, s, g_red.part, g, g_red.res);
   if (comm && comm->allreduce(g_red.res, 1, s)) return -1;
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


// ---------------------------------------------------------------------------------------------
// Nystrom apply kernels
// ---------------------------------------------------------------------------------------------
constexpr int kNysThreads = 256;

// partial[blk][j] = sum_{i in blk rows} U[i, j] r[i].  The block's r segment is staged in LDS; each
// wave walks its columns four at a time with 32 loads per lane in flight, row indices clamped to
// n - 1 (and r zero-padded) so the loads need no predication.
// T = float: the fp32 copy of U (Nfft4GPAmdNysSetStorage), widened to fp64 before the fp64 accumulation
constexpr int kNysUtCols = 4;
template <class T>
__global__ __launch_bounds__(kNysThreads) void k_nys_ut(const T* __restrict__ U, size_t ldu, int n, int k,
                                                       const double* __restrict__ r, double* __restrict__ part)
{
   constexpr int kPer = kNysRows / 64;
   constexpr int kChunk = 8;
   __shared__ double s_r[kNysRows];
   const int lane = threadIdx.x & 63;
   const int wave = threadIdx.x >> 6;
   const int nwv = kNysThreads / 64;
   const size_t r0 = (size_t)blockIdx.x * kNysRows;
   for (int t = threadIdx.x; t < kNysRows; t += kNysThreads) {
      const size_t i = r0 + t;
      s_r[t] = (i < (size_t)n) ? r[i] : 0.0;
   }
   __syncthreads();
   const size_t last = (size_t)n - 1;
   for (int j0 = wave * kNysUtCols; j0 < k; j0 += nwv * kNysUtCols) {
      const T* col[kNysUtCols];
#pragma unroll
      for (int c = 0; c < kNysUtCols; c++) col[c] = U + (size_t)min(j0 + c, k - 1) * ldu;
      double acc[kNysUtCols] = {};
#pragma unroll
      for (int t = 0; t < kPer; t += kChunk) {
         double v[kNysUtCols][kChunk];
#pragma unroll
         for (int c = 0; c < kNysUtCols; c++)
#pragma unroll
            for (int u = 0; u < kChunk; u++) {
               const size_t i = r0 + (size_t)(t + u) * 64 + lane;
               v[c][u] = (double)__builtin_nontemporal_load(col[c] + (i < last ? i : last));
            }
#pragma unroll
         for (int u = 0; u < kChunk; u++) {
            const double rr = s_r[(t + u) * 64 + lane];
#pragma unroll
            for (int c = 0; c < kNysUtCols; c++) acc[c] = fma(v[c][u], rr, acc[c]);
         }
      }
#pragma unroll
      for (int c = 0; c < kNysUtCols; c++) {
         double a = acc[c];
         for (int off = 32; off > 0; off >>= 1) a += __shfl_down(a, off, 64);
         if (lane == 0 && j0 + c < k) part[(size_t)blockIdx.x * k + j0 + c] = a;
      }
   }
}

// w[j] = (s[j] - 1/eta) * sum_blk part[blk][j].  A workgroup owns 64 columns; its 16 wave-rows
// each sum every 16th block (coalesced over j), then one fixed-order pass over the 16 sums.
constexpr int kNysWRows = 16;
__global__ __launch_bounds__(64 * kNysWRows) void k_nys_w(const double* __restrict__ part, int nblk, int k,
                                                          const double* __restrict__ s, double eta,
                                                          double* __restrict__ w)
{
   __shared__ double s_sum[kNysWRows][64];
   const int lane = threadIdx.x & 63;
   const int g = threadIdx.x >> 6;
   const int j = blockIdx.x * 64 + lane;
   const int jj = j < k ? j : k - 1;
   double z[4] = {};
   int b = g, u = 0;
   for (; b < nblk; b += kNysWRows, u = (u + 1) & 3) z[u] += part[(size_t)b * k + jj];
   s_sum[g][lane] = (z[0] + z[1]) + (z[2] + z[3]);
   __syncthreads();
   if (g == 0 && j < k) {
      double t = 0.0;
#pragma unroll
      for (int q = 0; q < kNysWRows; q++) t += s_sum[q][lane];
      w[j] = s ? s[j] * t - t / eta : t;  // s == NULL: the plain column sums (A^T x)
   }
}

// x[i] = r[i]/eta + sum_j U[i, j] w[j]
template <class T>
__global__ __launch_bounds__(kNysThreads) void k_nys_u(const T* __restrict__ U, size_t ldu, int n, int k,
                                                      const double* __restrict__ w, const double* __restrict__ r,
                                                      double eta, double* __restrict__ x)
{
   extern __shared__ double s_w[];
   for (int j = threadIdx.x; j < k; j += blockDim.x) s_w[j] = w[j];
   __syncthreads();
   const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
   if (i >= (size_t)n) return;
   double acc = 0.0;
   for (int j = 0; j < k; j++) acc = fma((double)U[(size_t)j * ldu + i], s_w[j], acc);
   x[i] = r[i] / eta + acc;
}

// PCG scratch: reduction partials + arrival ticket (device), status slots (pinned host, mapped)
struct PcgScratch {
   static constexpr int kSlots = 4;
   double* part = nullptr;
   unsigned int* ticket = nullptr;
   PcgSlot* slots_h = nullptr;
   PcgSlot* slots_d = nullptr;
   int ensure()
   {
      if (!part) {
         NFFT4GP_HIP_CHECK(hipMalloc((void**)&part, sizeof(double) * kPcgMaxBlocks));
         const size_t tb = sizeof(unsigned int) * kTicketWords;
         NFFT4GP_HIP_CHECK(hipMalloc((void**)&ticket, tb));
         NFFT4GP_HIP_CHECK(hipMemset(ticket, 0, tb));
         NFFT4GP_HIP_CHECK(hipHostMalloc((void**)&slots_h, sizeof(PcgSlot) * kSlots,
                                         hipHostMallocMapped | hipHostMallocCoherent));
         NFFT4GP_HIP_CHECK(hipHostGetDevicePointer((void**)&slots_d, slots_h, 0));
         memset(slots_h, 0, sizeof(PcgSlot) * kSlots);
      }
      return 0;
   }
};
PcgScratch g_pcg;


int g_last_hist_len = 0;

}  // namespace

namespace nfft4gp_amd {
// out[0..k) = A^T x for A n x k column-major (lda), fixed-order reduction over kNysRows row blocks;
// part holds ceil(n / kNysRows) * k doubles
int nys_gemv_t(const double* A, size_t lda, int n, int k, const double* x, double* out, double* part, hipStream_t s)
{
   const int nblk = (n + kNysRows - 1) / kNysRows;
   hipLaunchKernelGGL(k_nys_ut<double>, dim3(nblk), dim3(kNysThreads), 0, s, A, lda, n, k, x, part);
   hipLaunchKernelGGL(k_nys_w, dim3((k + 63) / 64), dim3(64 * kNysWRows), 0, s, part, nblk, k, (const double*)nullptr,
                      1.0, out);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

// x = M^{-1} rhs on device vectors (nys.c:115-173 in natural row order)
int nys_apply_dev(NysDev* N, double* x, const double* rhs, hipStream_t s)
{
   const int n = N->n;
   if (N->Uf)
      hipLaunchKernelGGL(k_nys_ut<float>, dim3(N->nblk), dim3(kNysThreads), 0, s, N->Uf, (size_t)n, n, N->k, rhs,
                         N->part);
   else
      hipLaunchKernelGGL(k_nys_ut<double>, dim3(N->nblk), dim3(kNysThreads), 0, s, N->U, (size_t)n, n, N->k, rhs,
                         N->part);
   hipLaunchKernelGGL(k_nys_w, dim3((N->k + 63) / 64), dim3(64 * kNysWRows), 0, s, N->part, N->nblk, N->k, N->s, N->eta,
                      N->w);
   if (N->Uf)
      hipLaunchKernelGGL(k_nys_u<float>, dim3((n + kNysThreads - 1) / kNysThreads), dim3(kNysThreads),
                         sizeof(double) * N->k, s, N->Uf, (size_t)n, n, N->k, N->w, rhs, N->eta, x);
   else
      hipLaunchKernelGGL(k_nys_u<double>, dim3((n + kNysThreads - 1) / kNysThreads), dim3(kNysThreads),
                         sizeof(double) * N->k, s, N->U, (size_t)n, n, N->k, N->w, rhs, N->eta, x);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

// the two U passes of the apply on this rank's rows, for the row-sharded apply (dist.hip): w = U^T r
// (column sums, not yet scaled) and x = U w + r / eta
int nys_ut_local(NysDev* N, const double* rhs, double* w, hipStream_t s)
{
   if (N->n == 0) {
      NFFT4GP_HIP_CHECK(hipMemsetAsync(w, 0, sizeof(double) * N->k, s));
      return 0;
   }
   hipLaunchKernelGGL(k_nys_ut<double>, dim3(N->nblk), dim3(kNysThreads), 0, s, (const double*)N->U, (size_t)N->n,
                      N->n, N->k, rhs, N->part);
   hipLaunchKernelGGL(k_nys_w, dim3((N->k + 63) / 64), dim3(64 * kNysWRows), 0, s, (const double*)N->part, N->nblk,
                      N->k, (const double*)nullptr, N->eta, w);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int nys_u_local(NysDev* N, const double* w, const double* rhs, double* x, hipStream_t s)
{
   if (N->n == 0) return 0;
   hipLaunchKernelGGL(k_nys_u<double>, dim3((N->n + kNysThreads - 1) / kNysThreads), dim3(kNysThreads),
                      sizeof(double) * N->k, s, (const double*)N->U, (size_t)N->n, N->n, N->k, w, rhs, N->eta, x);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

__global__ void k_to_f32(const double* __restrict__ a, size_t count, float* __restrict__ b)
{
   for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x)
      b[i] = (float)a[i];
}
}  // namespace nfft4gp_amd

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

// vecops.c:15-46: serial libc rand() (the reference's sequence for a given srand seed); device vectors
// get the same host-generated values
static void vec_random(double* x, int n, bool rademacher)
{
   std::vector<double> h(std::max(0, n));
   {
      CallerRandBatch caller;
      for (int i = 0; i < n; i++) {
         h[i] = (double)rand() / (double)RAND_MAX;
         if (rademacher) h[i] = h[i] < 0.5 ? -1.0 : 1.0;
      }
   }
   if (n > 0 && is_device_ptr(x))
      (void)hipMemcpy(x, h.data(), sizeof(double) * n, hipMemcpyHostToDevice);
   else if (n > 0)
      memcpy(x, h.data(), sizeof(double) * n);
}

void Nfft4GPVecRand(double* x, int n) { vec_random(x, n, false); }
void Nfft4GPVecRadamacher(double* x, int n) { vec_random(x, n, true); }

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
   Callbacks cb;
   cb.matvec = matvec;
   cb.mat = mat_data;
   cb.prec = precondfunc;
   cb.pdata = prec_data;
   cb.n = N;
   cb.mv_dev = g_cb_mode == 1 || (g_cb_mode == -1 && library_operator((const void*)matvec));
   cb.pc_dev = g_cb_mode == 1 || (g_cb_mode == -1 && library_operator((const void*)precondfunc));
   Vec vx, vb;
   if (vx.open(x, N, true) || vb.open(rhs, N, true)) return -1;
   double *r = nullptr, *z = nullptr, *p = nullptr, *q = nullptr;
   double *rhos = nullptr, *hist_d = nullptr;
   PcgState* st = nullptr;
   PcgSlot* slots_h = nullptr;  // pinned, device-visible
   PcgSlot* slots_d = nullptr;
   int iter = 0;
   double normb, normr, normr2, tolb;
   double* rel_res_v = nullptr;
   const double EPSILON = DBL_EPSILON;
   if (g_red.ensure() || g_pcg.ensure()) return -1;

   auto cleanup = [&](bool copy_x) {
      if (r) (void)hipFree(r);
      if (z) (void)hipFree(z);
      if (p) (void)hipFree(p);
      if (q) (void)hipFree(q);
      if (rhos) (void)hipFree(rhos);
      if (hist_d) (void)hipFree(hist_d);
      if (st) (void)hipFree(st);
      vx.close(copy_x);
      vb.close(false);
   };

   // a distributed operator (dist.hip): row-sharded vectors sum every dot over its communicator (red), and
   // maxits is clamped to the global n; component-sharded (replicated) vectors need neither
   const bool is_dist = cb.mv_dev && matvec == &Nfft4GPAmdDistMatSymv;
   DistPcgInfo dinfo;
   if (is_dist && dist_pcg_info(mat_data, dinfo)) return -1;
   Comm* red = is_dist ? dinfo.dot_comm : nullptr;
   const int n_all = is_dist ? dinfo.n_global : n;
   if (dev_dot(vb.d, vb.d, N, &normb, red)) return -1;
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
   if (maxits > n_all) maxits = n_all;

   NFFT4GP_HIP_CHECK(hipMalloc((void**)&r, sizeof(double) * N));
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&p, sizeof(double) * N));
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&q, sizeof(double) * N));
   if (prec_data) NFFT4GP_HIP_CHECK(hipMalloc((void**)&z, sizeof(double) * N));

   NFFT4GP_HIP_CHECK(hipMemcpyAsync(r, vb.d, sizeof(double) * N, hipMemcpyDeviceToDevice, s));
   if (cb.apply(-1.0, vx.d, 1.0, r)) {
      cleanup(false);
      return -1;
   }
   double rr0;
   if (dev_dot(r, r, N, &rr0, red)) return -1;
   normr = std::sqrt(rr0);
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

   // device state
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&rhos, sizeof(double) * ((size_t)maxits + 2)));
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&hist_d, sizeof(double) * ((size_t)maxits + 1)));
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&st, sizeof(PcgState)));
   NFFT4GP_HIP_CHECK(hipMemsetAsync(hist_d, 0, sizeof(double) * ((size_t)maxits + 1), s));
   {
      PcgState h{};
      h.normb = normb;
      h.tolb = tolb;
      h.normr2 = normr;
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(st, &h, sizeof(h), hipMemcpyHostToDevice, s));
      // no preconditioner: z = r, so iteration 1's rho is (r, r)  (pcg.c:103-119)
      if (!prec_data) NFFT4GP_HIP_CHECK(hipMemcpyAsync(rhos + 1, &rr0, sizeof(double), hipMemcpyHostToDevice, s));
      NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
   }
   slots_h = g_pcg.slots_h;
   slots_d = g_pcg.slots_d;
   for (int i = 0; i < PcgScratch::kSlots; i++) __atomic_store_n(&slots_h[i].seq, 0, __ATOMIC_RELAXED);

   const int g = pcg_grid(N);
   const int ge = g;
   const int g_xr = (int)std::max<size_t>(1, std::min<size_t>((N + 1024 * kEPT - 1) / (1024 * kEPT), kPcgMaxBlocks));
   // this library's additive operator forms (q, p) in its own interpolation launch
   const bool fused_dot = cb.mv_dev && ((matvec == &Nfft4GPAdditiveNFFTMatSymv && additive_fused_dot_ok(mat_data)) ||
                                        (is_dist && dinfo.fused_dot));
   double* loc0 = red ? &st->loc[0] : nullptr;  // device addresses inside st
   double* loc1 = red ? &st->loc[1] : nullptr;
   // the direction update folded into k_pcg_xr (FUSEP): no preconditioner, one GPU, n covered by one pass of a
   // grid that fits the chip at once (its workgroups wait for the last one); NFFT4GP_AMD_PCG_FUSEP=0 disables
   bool fusep = !prec_data && !red && (size_t)g_xr * 1024 * kEPT >= N;
   if (fusep) {
      static int occ = -1, ncu = 0;
      if (occ < 0) {
         int dev = 0;
         hipDeviceProp_t prop;
         if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess ||
             hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_pcg_xr<1024, true>, 1024, 0) != hipSuccess)
            occ = 0;
         else
            ncu = prop.multiProcessorCount;
      }
      const char* e = getenv("NFFT4GP_AMD_PCG_FUSEP");
      fusep = occ > 0 && g_xr <= occ * ncu && !(e && atoi(e) == 0);
   }
   bool need_p = true;  // the next iteration's p update is not done yet (first iteration, after a resume)
   // iterations in flight ahead of the host's status check (1 when printing every step)
   const int lag = print_level > 0 ? 1 : PcgScratch::kSlots;
   double prev_rel = rel_res_v[0];
   int next_check = 1;   // next iteration whose slot the host reads
   int ii = 1;
   bool stop = false;
   int rc = 0;
   while (!stop) {
      // enqueue iterations until `lag` are unchecked or maxits is reached
      while (ii <= maxits && ii - next_check < lag) {
         double* zz = r;
         if (prec_data) {
            if (cb.solve(z, r)) { rc = -1; break; }
            hipLaunchKernelGGL(k_pcg_dot, dim3(g), dim3(kVecThreads), 0, s, z, r, N, g_pcg.part, g_pcg.ticket, st,
                               rhos, ii, 0, loc0);
            if (red) {
               if (red->allreduce(loc0, 1, s)) { rc = -1; break; }
               hipLaunchKernelGGL(k_pcg_dot_fin, dim3(1), dim3(64), 0, s, st, rhos, ii, 0, (const double*)loc0);
            }
            zz = z;
         }
         if (need_p || !fusep)
            hipLaunchKernelGGL(k_pcg_pupdate, dim3(ge), dim3(kVecThreads), 0, s, p, zz, N, st, rhos, ii);
         if (fused_dot) {
            // q = A p with (q, p) formed inside the interpolation kernel's epilogue
            if (is_dist) {
               if (dist_matvec_dot(mat_data, p, q, &st->pq) || (red && red->allreduce(&st->pq, 1, s))) {
                  rc = -1;
                  break;
               }
            } else if (additive_matvec_dot(mat_data, p, q, &st->pq)) {
               rc = -1;
               break;
            }
         } else {
            if (cb.apply(1.0, p, 0.0, q)) { rc = -1; break; }
            hipLaunchKernelGGL(k_pcg_dot, dim3(g), dim3(kVecThreads), 0, s, q, p, N, g_pcg.part, g_pcg.ticket, st,
                               rhos, ii, 1, loc0);
            if (red) {
               if (red->allreduce(loc0, 1, s)) { rc = -1; break; }
               hipLaunchKernelGGL(k_pcg_dot_fin, dim3(1), dim3(64), 0, s, st, rhos, ii, 1, (const double*)loc0);
            }
         }
         PcgSlot* slot = slots_d + (ii % PcgScratch::kSlots);
         if (fusep) {
            hipLaunchKernelGGL((k_pcg_xr<1024, true>), dim3(g_xr), dim3(1024), 0, s, vx.d, r, p, q, N, g_pcg.part,
                               g_pcg.ticket, st, rhos, hist_d, ii, 1, fused_dot ? 1 : 0, slot, (double*)nullptr,
                               ii < maxits ? 1 : 0);
            need_p = false;
         } else {
            hipLaunchKernelGGL(k_pcg_xr<1024>, dim3(g_xr), dim3(1024), 0, s, vx.d, r, p, q, N, g_pcg.part,
                               g_pcg.ticket, st, rhos, hist_d, ii, prec_data ? 0 : 1, fused_dot ? 1 : 0, slot, loc1);
         }
         if (red) {
            if (red->allreduce(loc1, 1, s)) { rc = -1; break; }
            hipLaunchKernelGGL(k_pcg_xr_fin, dim3(1), dim3(64), 0, s, st, rhos, hist_d, ii, prec_data ? 0 : 1, slot,
                               (const double*)loc1);
         }
         ii++;
      }
      if (rc) break;
      NFFT4GP_HIP_CHECK(hipGetLastError());
      if (next_check >= ii) break;  // nothing in flight: maxits reached
      // wait for iteration next_check's status slot
      PcgSlot* sl = slots_h + (next_check % PcgScratch::kSlots);
      long spins = 0;
      while (__atomic_load_n(&sl->seq, __ATOMIC_ACQUIRE) != next_check) {
         if ((++spins & 0xFFFF) == 0) {
            const hipError_t qe = hipStreamQuery(s);
            if (qe == hipSuccess && __atomic_load_n(&sl->seq, __ATOMIC_ACQUIRE) != next_check) {
               fprintf(stderr, "nfft4gp_amd: PCG status slot %d never arrived\n", next_check);
               rc = -1;
               break;
            }
            if (qe != hipSuccess && qe != hipErrorNotReady) {
               fprintf(stderr, "nfft4gp_amd: PCG stream error %s\n", hipGetErrorString(qe));
               rc = -1;
               break;
            }
         }
      }
      if (rc) break;
      const int status = sl->status;
      const int fi = sl->flag_iter;
      if (print_level > 0 && (status == 0 || status == 1) && (status == 0 || fi == next_check)) {
         const double rel = sl->normr / normb;
         printf("%5d   %8e   %8e   %8.6f\n", next_check, sl->normr, rel, rel / prev_rel);
         prev_rel = rel;
      }
      if (status == 0) {
         next_check++;
         continue;
      }
      // a kernel stopped the iteration at fi <= next_check: drain the no-op'd tail, then act as pcg.c
      NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
      PcgState h;
      NFFT4GP_HIP_CHECK(hipMemcpy(&h, st, sizeof(h), hipMemcpyDeviceToHost));
      NFFT4GP_HIP_CHECK(hipMemcpy(rel_res_v + 1, hist_d + 1, sizeof(double) * (size_t)fi, hipMemcpyDeviceToHost));
      normr2 = h.normr2;
      if (status == 5) {
         fprintf(stderr, "nfft4gp_amd: PCG iteration %d: the fused update's wait for its last workgroup gave up\n", fi);
         rc = -1;
         break;
      }
      if (status != 1) {
         if (print_level > 1) {
            if (status == 2) printf("rho = %.16e\n", 0.0);
            if (status == 3) printf("beta = %.16e\n", 0.0);
            if (status == 4) printf("pq = %.16e\n", h.pq);
         }
         break;
      }
      // pcg.c:181-193: recompute the true residual
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(r, vb.d, sizeof(double) * N, hipMemcpyDeviceToDevice, s));
      if (cb.apply(-1.0, vx.d, 1.0, r)) { rc = -1; break; }
      double rr;
      if (dev_dot(r, r, N, &rr, red)) { rc = -1; break; }
      normr2 = std::sqrt(rr);
      rel_res_v[fi] = normr2;
      if (normr2 <= tolb) {
         iter = fi;
         break;
      }
      // keep iterating from fi + 1 with the true residual
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(hist_d + fi, &rel_res_v[fi], sizeof(double), hipMemcpyHostToDevice, s));
      if (!prec_data) NFFT4GP_HIP_CHECK(hipMemcpyAsync(rhos + fi + 1, &rr, sizeof(double), hipMemcpyHostToDevice, s));
      h.status = 0;
      h.normr2 = normr2;
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(st, &h, sizeof(h), hipMemcpyHostToDevice, s));
      NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
      for (int i = 0; i < PcgScratch::kSlots; i++) __atomic_store_n(&slots_h[i].seq, 0, __ATOMIC_RELAXED);
      prev_rel = rel_res_v[fi];
      ii = fi + 1;
      next_check = fi + 1;
      need_p = true;  // iteration fi's fused update saw its status and skipped p
   }
   if (!rc && iter == 0) {
      // not converged (maxits or breakdown): the history of the completed iterations
      (void)hipStreamSynchronize(s);
      PcgState h;
      if (hipMemcpy(&h, st, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess) {
         normr2 = h.normr2;
         const int last = h.status ? h.flag_iter : std::min(ii - 1, maxits);
         if (last > 0) (void)hipMemcpy(rel_res_v + 1, hist_d + 1, sizeof(double) * (size_t)last, hipMemcpyDeviceToHost);
         if (h.status == 1) rel_res_v[h.flag_iter] = normr2;
      }
   }
   if (rc) {
      (void)hipStreamSynchronize(s);
      free(rel_res_v);
      cleanup(false);
      return -1;
   }
   if (dist_final_check(cb)) {
      free(rel_res_v);
      cleanup(false);
      return -1;
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
   if (hipMalloc((void**)&N->U, sizeof(double) * hU.size()) != hipSuccess ||
       hipMalloc((void**)&N->s, sizeof(double) * k) != hipSuccess || nys_alloc_scratch(N)) {
      fprintf(stderr, "nfft4gp_amd: Nystrom allocation failed\n");
      return nullptr;
   }
   (void)hipMemcpy(N->U, hU.data(), sizeof(double) * hU.size(), hipMemcpyHostToDevice);
   (void)hipMemcpy(N->s, hs.data(), sizeof(double) * k, hipMemcpyHostToDevice);
   return N;
}


int Nfft4GPAmdNysSetStorage(void* nys, int bits)
{
   NysDev* N = (NysDev*)nys;
   if (!N || (bits != 32 && bits != 64)) return -1;
   hipStream_t s = current_stream();
   if (bits == 64) {
      if (N->Uf) {
         NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
         NFFT4GP_HIP_CHECK(hipFree(N->Uf));
         N->Uf = nullptr;
      }
      return 0;
   }
   if (N->Uf) return 0;
   const size_t count = (size_t)N->n * N->k;
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&N->Uf, sizeof(float) * std::max<size_t>(1, count)));
   hipLaunchKernelGGL(k_to_f32, dim3(4096), dim3(256), 0, s, N->U, count, N->Uf);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int Nfft4GPAmdNysSolve(void* nys, int n, double* x, double* rhs)
{
   NysDev* N = (NysDev*)nys;
   if (!N || n != N->n) return -1;
   hipStream_t s = current_stream();
   Vec vx, vr;
   if (vx.open(x, n, false) || vr.open(rhs, n, true)) return -1;
   if (nys_apply_dev(N, vx.d, vr.d, s)) return -1;
   vr.close(false);
   vx.close(true);
   return 0;
}

void Nfft4GPAmdNysFree(void* nys) { nys_free((NysDev*)nys); }

}  // extern "C"

namespace nfft4gp_amd {
int g_cb_mode = -1;
bool library_operator(const void* fn)
{
   return fn == (const void*)&Nfft4GPAdditiveNFFTMatSymv || fn == (const void*)&Nfft4GPNFFTMatSymv ||
          fn == (const void*)&Nfft4GPAdditiveNFFTGradMatSymv || fn == (const void*)&Nfft4GPNFFTGradMatSymv ||
          fn == (const void*)&Nfft4GPAmdNysSolve || fn == (const void*)&Nfft4GPAmdFsaiSolve ||
          fn == (const void*)&Nfft4GPAmdAfnSolve || fn == (const void*)&Nfft4GPAmdPrecondNysSolve ||
          fn == (const void*)&Nfft4GPAmdPrecondNysDvp || fn == (const void*)&Nfft4GPAmdPrecondFsaiSolve ||
          fn == (const void*)&Nfft4GPAmdPrecondFsaiDvp || fn == (const void*)&Nfft4GPAmdDistMatSymv ||
          fn == (const void*)&Nfft4GPAmdDistGradMatSymv || fn == (const void*)&Nfft4GPAmdDistNysSolve ||
          fn == (const void*)&Nfft4GPAmdDistAfnSolve || fn == (const void*)&Nfft4GPPrecondNysSolve ||
          fn == (const void*)&Nfft4GPAmdPrecondAFNSolve || fn == (const void*)&Nfft4GPAmdPrecondAFNDvp;
}
}  // namespace nfft4gp_amd

extern "C" void Nfft4GPAmdSetCallbackPointerMode(int mode) { g_cb_mode = (mode < -1 || mode > 1) ? -1 : mode; }
