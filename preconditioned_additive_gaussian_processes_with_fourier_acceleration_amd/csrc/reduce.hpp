// reduce.hpp -- deterministic grid-wide sums inside one launch (device code, included by the .hip files).
//
// Every block stores its partial with an agent-scope (sc1, memory-side) store, drains it with
// s_waitcnt vmcnt(0) and takes an arrival ticket; the LAST arriving block reads all partials back with
// agent-scope loads and sums them in block order (bitwise reproducible for a fixed grid).  No L2
// write-back fence is needed (a release fence here writes back every dirty line the kernel produced:
// measured +15-20 us per launch), and arrivals are counted per XCD first (block b runs on XCD b % 8)
// and then once per XCD on a top counter, because a single counter taking ~1000 RMWs serialises at
// one memory channel (~13 us).  MI355X_MICROARCH.md 'handoff-flag' is the pattern.
#pragma once

#include <hip/hip_runtime.h>

namespace nfft4gp_amd {

constexpr int kRedXcds = 8;
constexpr int kTicketStride = 64;                              // unsigned ints: 256 B between counters
constexpr int kTicketWords = (kRedXcds + 1) * kTicketStride;   // size of a ticket array
constexpr int kRedMaxBlocks = 4096;                            // partials a last arriver can sum

// block-wide sum of `acc`; the result is valid in thread 0.  s: THREADS / 64 doubles of LDS scratch
template <int THREADS>
__device__ __forceinline__ double block_sum0_s(double acc, double* s)
{
   for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
   if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
   __syncthreads();
   double v = 0.0;
   if (threadIdx.x == 0)
      for (int w = 0; w < THREADS / 64; w++) v += s[w];
   return v;
}
template <int THREADS>
__device__ __forceinline__ double block_sum0(double acc)
{
   __shared__ double s[THREADS / 64];
   return block_sum0_s<THREADS>(acc, s);
}

// thread 0 holds the block's partial `v`; returns true in every thread of the last arriving block,
// with the fixed-order total in *total.  gridDim.x <= kRedMaxBlocks.  Leaves the tickets at zero.
// s_last, s_red (THREADS / 64 doubles): LDS scratch
template <int THREADS>
__device__ bool grid_total_s(double v, double* __restrict__ part, unsigned int* __restrict__ ticket, double* total,
                             int* s_last_p, double* s_red)
{
   int& s_last = *s_last_p;
   if (threadIdx.x == 0) {
      __hip_atomic_store(part + blockIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
   if (!s_last) return false;
   constexpr int kPer = (kRedMaxBlocks + THREADS - 1) / THREADS;
   double pv[kPer];
#pragma unroll
   for (int u = 0; u < kPer; u++) {
      const unsigned i = threadIdx.x + u * THREADS;
      pv[u] = i < gridDim.x ? __hip_atomic_load(part + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
   }
   double acc = 0.0;
#pragma unroll
   for (int u = 0; u < kPer; u++) acc += pv[u];
   for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
   if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = acc;
   __syncthreads();
   double t = 0.0;
   for (int w = 0; w < THREADS / 64; w++) t += s_red[w];
   *total = t;
   if (threadIdx.x <= (unsigned)kRedXcds)
      __hip_atomic_store(ticket + threadIdx.x * kTicketStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
   return true;
}
template <int THREADS>
__device__ bool grid_total(double v, double* __restrict__ part, unsigned int* __restrict__ ticket, double* total)
{
   __shared__ int s_last;
   __shared__ double s_red[THREADS / 64];
   return grid_total_s<THREADS>(v, part, ticket, total, &s_last, s_red);
}

}  // namespace nfft4gp_amd
