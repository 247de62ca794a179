// nfft_kernels.hip -- CDNA4 (gfx950) kernels of the additive NFFT matvec.
//
// Per matvec three launches on one stream (see internal.h for the algebra):
//   k_spread  one workgroup per (block of B points, group of CG windows).  The workgroup stages the
//             block's alpha slice (B doubles) in LDS once for its windows; each lane walks one R-point
//             run of a single (window, cell), accumulates the 12 moments alpha*u^d in registers and
//             flushes them with ds_add_f64 into an LDS moment table; the workgroup finally folds the
//             moments into 64-cell partial grids (taps = C * M) and writes them to part[comp][block].
//             HBM: 6 B per (point, window) -- u16 local index + u32 fixed-point coordinate -- + alpha.
//   k_grid    one workgroup per window: sum of the partial grids (fixed order, deterministic), the
//             64x64 real circulant (= FFT . diag(bhat/phihut^2) . IFFT restricted to Re), and the
//             per-cell interpolation polynomials H = C^T h.
//   k_interp  one workgroup per block: lanes walk the same runs, load H[comp][cell] once per run,
//             Horner per point, ds_add_f64 into an LDS y-block; the epilogue applies
//             y = beta*y + alpha*ff*(sum + mu*x) (grad: the three outputs of nfft_interface.c:547-549)
//             in one coalesced pass.
// Kernel shapes (threads per workgroup, occupancy hint, next-run prefetch) are template parameters;
// the launchers pick a variant from AdditivePlan (env NFFT4GP_AMD_SPREAD_VARIANT / _INTERP_VARIANT).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>

#include "internal.h"

namespace nfft4gp_amd {

constexpr int kGridThreads = 1024;
// LDS row stride of the moment table: 13 doubles (26 banks) so rows of different cells spread over
// the 64 banks instead of repeating every 8 cells (stride 12 -> 24 banks)
constexpr int kMomStride = kNC + 1;

__device__ __forceinline__ double q_to_u(uint32_t q)
{
   // offset inside the cell minus one half: exact in fp64
   return (double)(q & 0x3FFFFFFu) * 0x1p-26 - 0.5;
}

// tap polynomial coefficients C[t][d] in constant memory: wave-uniform reads become scalar loads
__constant__ double c_taps[kTaps * kNC];

// diagnostic timeline (ABL == 5 builds only): per workgroup 4 s_memrealtime stamps (100 MHz)
constexpr int kMaxStampWG = 16384;
__device__ unsigned long long g_stamps[kMaxStampWG * 4];

template <int ABL>
__device__ __forceinline__ void stamp(int slot)
{
   if (ABL == 5 && threadIdx.x == 0 && blockIdx.x < kMaxStampWG)
      g_stamps[blockIdx.x * 4 + slot] = __builtin_amdgcn_s_memrealtime();
}

struct TileRegs {
   uint32_t mt;
   uint32_t pp[kR / 2];
   uint32_t qq[kR];
};

__device__ __forceinline__ void load_tile(TileRegs& T, const uint16_t* __restrict__ meta,
                                          const uint32_t* __restrict__ perm2, const uint32_t* __restrict__ qarr,
                                          int t, int lane)
{
   // 16 B per lane per load: perm2 quads [t][2][lane], q quads [t][4][lane] (layout.cpp)
   T.mt = meta[(size_t)t * 64 + lane];
   const uint4* p4 = reinterpret_cast<const uint4*>(perm2) + (size_t)t * (kR / 8) * 64 + lane;
   const uint4* q4 = reinterpret_cast<const uint4*>(qarr) + (size_t)t * (kR / 4) * 64 + lane;
#pragma unroll
   for (int k = 0; k < kR / 8; k++) {
      const uint4 v = p4[k * 64];
      T.pp[4 * k + 0] = v.x;
      T.pp[4 * k + 1] = v.y;
      T.pp[4 * k + 2] = v.z;
      T.pp[4 * k + 3] = v.w;
   }
#pragma unroll
   for (int k = 0; k < kR / 4; k++) {
      const uint4 v = q4[k * 64];
      T.qq[4 * k + 0] = v.x;
      T.qq[4 * k + 1] = v.y;
      T.qq[4 * k + 2] = v.z;
      T.qq[4 * k + 3] = v.w;
   }
}

// ------------------------------------------------------------------------------------------------
// spread
// ------------------------------------------------------------------------------------------------
template <int THREADS, int MINW, bool PREFETCH, int ABL = 0, bool CONTIG = false>
__global__ __launch_bounds__(THREADS, MINW) void k_spread(
    const uint16_t* __restrict__ meta, const uint32_t* __restrict__ perm2, const uint32_t* __restrict__ qarr,
    const int* __restrict__ tile_off, const double* __restrict__ x, int n, int B, int nblocks, int ngroups, int CG,
    int nw, double* __restrict__ part)
{
   extern __shared__ __attribute__((aligned(16))) double smem[];
   const int Bp = (B + 2) & ~1;
   double* s_alpha = smem;     // Bp
   double* s_mom = smem + Bp;  // CG*64*kMomStride per-cell moments

   // XCD-aware decode: the ngroups workgroups of one block land on one XCD (blockIdx % 8), so its
   // alpha slice is fetched into one L2.  Speed only; correctness does not depend on placement.
   const int xcd = blockIdx.x & 7;
   const int rest = blockIdx.x >> 3;
   const int g = rest % ngroups;
   const int b = (rest / ngroups) * 8 + xcd;
   if (b >= nblocks) return;
   stamp<ABL>(0);

   const int tid = threadIdx.x;
   const int lane = tid & 63;
   const int wave = tid >> 6;
   constexpr int nwaves = THREADS / 64;
   const int c0 = g * CG;
   const int t0 = tile_off[b * ngroups + g];
   const int t1 = tile_off[b * ngroups + g + 1];

   if (CONTIG) {
      // each wave takes a contiguous range of the group's tiles; with the column-dealt layout a lane
      // then walks CONSECUTIVE chunks of the sorted (window, cell) list, keeps its moments in registers
      // while the key stays the same and flushes to LDS only when the key changes
      const int T = t1 - t0;
      const int ta = t0 + (int)(((long long)wave * T) / nwaves);
      const int tb = t0 + (int)(((long long)(wave + 1) * T) / nwaves);
      TileRegs cur;
      if (ta < tb) load_tile(cur, meta, perm2, qarr, ta, lane);
      const int base = b * B;
      const int nloc = min(B, n - base);
      for (int i = tid; i < Bp; i += THREADS) s_alpha[i] = (i < nloc) ? x[base + i] : 0.0;
      for (int i = tid; i < CG * kNos * kMomStride; i += THREADS) s_mom[i] = 0.0;
      __syncthreads();
      double acc[kNC];
#pragma unroll
      for (int d = 0; d < kNC; d++) acc[d] = 0.0;
      uint32_t key = (ta < tb) ? cur.mt : 0u;
      for (int t = ta; t < tb; t++) {
         TileRegs nxt;
         if (t + 1 < tb) load_tile(nxt, meta, perm2, qarr, t + 1, lane);  // prefetch the next run
         if (cur.mt != key) {  // divergent: only lanes whose (window, cell) changed flush
            double* dst = s_mom + ((int)(key >> 6) - c0) * kNos * kMomStride + (int)(key & 63u) * kMomStride;
#pragma unroll
            for (int d = 0; d < kNC; d++) {
               atomicAdd(dst + d, acc[d]);
               acc[d] = 0.0;
            }
            key = cur.mt;
         }
#pragma unroll
         for (int r = 0; r < kR; r++) {
            const uint32_t loc = (r & 1) ? (cur.pp[r >> 1] >> 16) : (cur.pp[r >> 1] & 0xFFFFu);
            const double u = q_to_u(cur.qq[r]);
            double tpow = s_alpha[loc];
            acc[0] += tpow;
#pragma unroll
            for (int d = 1; d < kNC; d++) {
               tpow *= u;
               acc[d] += tpow;
            }
         }
         if (t + 1 < tb) cur = nxt;
      }
      if (ta < tb) {
         double* dst = s_mom + ((int)(key >> 6) - c0) * kNos * kMomStride + (int)(key & 63u) * kMomStride;
#pragma unroll
         for (int d = 0; d < kNC; d++) atomicAdd(dst + d, acc[d]);
      }
      __syncthreads();
   } else {
   // issue the first run's loads before the alpha staging so both are in flight together
   TileRegs cur;
   int t = t0 + wave;
   if (t < t1) load_tile(cur, meta, perm2, qarr, t, lane);

   const int base = b * B;
   const int nloc = min(B, n - base);
   for (int i = tid; i < Bp; i += THREADS) s_alpha[i] = (i < nloc) ? x[base + i] : 0.0;
   for (int i = tid; i < CG * kNos * kMomStride; i += THREADS) s_mom[i] = 0.0;
   __syncthreads();
   stamp<ABL>(1);

   for (; t < t1; t += nwaves) {
      TileRegs nxt;
      const int tn = t + nwaves;
      if (PREFETCH && tn < t1) load_tile(nxt, meta, perm2, qarr, tn, lane);  // prefetch the next run
      double acc[kNC];
#pragma unroll
      for (int d = 0; d < kNC; d++) acc[d] = 0.0;
      if (ABL == 4) {
         // mixed precision: moments d <= 5 in fp64; d = 6..11 (<= 2.4e-4 of the window peak in the taps,
         // so fp32 rounding contributes ~1e-11 relative) as packed fp32 on point pairs; all 16 alpha
         // gathers are issued before the arithmetic
         double a[kR];
#pragma unroll
         for (int r = 0; r < kR; r++) {
            const uint32_t loc = (r & 1) ? (cur.pp[r >> 1] >> 16) : (cur.pp[r >> 1] & 0xFFFFu);
            a[r] = s_alpha[loc];
         }
         typedef float f2 __attribute__((ext_vector_type(2)));
         f2 hi[kNC - 6];
#pragma unroll
         for (int d = 0; d < kNC - 6; d++) hi[d] = f2{0.f, 0.f};
#pragma unroll
         for (int r = 0; r < kR; r += 2) {
            const double u0 = q_to_u(cur.qq[r]);
            const double u1 = q_to_u(cur.qq[r + 1]);
            double p0 = a[r], p1 = a[r + 1];
            acc[0] += p0;
            acc[0] += p1;
#pragma unroll
            for (int d = 1; d < 6; d++) {
               p0 *= u0;
               p1 *= u1;
               acc[d] += p0;
               acc[d] += p1;
            }
            f2 tp = f2{(float)(p0 * u0), (float)(p1 * u1)};
            const f2 uu = f2{(float)u0, (float)u1};
            hi[0] += tp;
#pragma unroll
            for (int d = 1; d < kNC - 6; d++) {
               tp *= uu;
               hi[d] += tp;
            }
         }
#pragma unroll
         for (int d = 0; d < kNC - 6; d++) acc[6 + d] = (double)hi[d].x + (double)hi[d].y;
      } else
#pragma unroll
      for (int r = 0; r < kR; r++) {
         const uint32_t loc = (r & 1) ? (cur.pp[r >> 1] >> 16) : (cur.pp[r >> 1] & 0xFFFFu);
         const double u = q_to_u(cur.qq[r]);
         // ABL (timing experiments only, wrong results): 1 = no alpha gather, 2 = no moment powers
         double tpow = (ABL == 1) ? (double)loc : s_alpha[loc];
         acc[0] += tpow;
         if (ABL == 2) {
            acc[1] += u;
         } else {
#pragma unroll
            for (int d = 1; d < kNC; d++) {
               tpow *= u;
               acc[d] += tpow;
            }
         }
      }
      const int comp_local = (int)(cur.mt >> 6) - c0;
      const int cell = (int)(cur.mt & 63u);
      double* dst = s_mom + (comp_local * kNos + cell) * kMomStride;
      if (ABL == 3) {  // no flush atomics: one plain store
         if (acc[0] == 12345.0) dst[0] = acc[1] + acc[11];
      } else {
#pragma unroll
         for (int d = 0; d < kNC; d++) atomicAdd(dst + d, acc[d]);  // ds_add_f64
      }
      if (PREFETCH) {
         if (tn < t1) cur = nxt;
      } else if (tn < t1) {
         load_tile(cur, meta, perm2, qarr, tn, lane);
      }
   }
   __syncthreads();
   }
   stamp<ABL>(2);

   // fold moments into the 64-cell partial grid of every window of this group:
   //   g[gi] = sum_t sum_d C[t][d] M[(gi + m - t) mod 64][d]
   const int ncomp = min(CG, nw - c0);
   for (int idx = tid; idx < ncomp * kNos; idx += THREADS) {
      const int cl = idx / kNos;
      const int gi = idx % kNos;
      double v = 0.0;
#pragma unroll 1
      for (int tp = 0; tp < kTaps; tp++) {
         const double* mrow = s_mom + (cl * kNos + ((gi + kM - tp) & (kNos - 1))) * kMomStride;
#pragma unroll
         for (int d = 0; d < kNC; d++) v = fma(c_taps[tp * kNC + d], mrow[d], v);
      }
      part[((size_t)(c0 + cl) * nblocks + b) * kNos + gi] = v;  // [comp][block][cell]
   }
   if (ABL == 5) {
      __syncthreads();
      stamp<ABL>(3);
   }
}

// ------------------------------------------------------------------------------------------------
// persistent spread: a resident workgroup walks items (block, group) = it, it + G, it + 2G, ...
// The next item's alpha slice is loaded into registers and its first runs into the tile registers
// while the current item is processed, so the per-item prologue no longer waits on HBM; the fold uses
// every thread with independent per-tap accumulators.
// ------------------------------------------------------------------------------------------------
template <int THREADS, int BMAX>
__global__ __launch_bounds__(THREADS, 2 * THREADS / 256) void k_spread_persist(
    const uint16_t* __restrict__ meta, const uint32_t* __restrict__ perm2, const uint32_t* __restrict__ qarr,
    const int* __restrict__ tile_off, const double* __restrict__ x, int n, int B, int nblocks, int ngroups, int CG,
    int nw, double* __restrict__ part)
{
   extern __shared__ __attribute__((aligned(16))) double smem[];
   constexpr int kPer = (BMAX + 2 + THREADS - 1) / THREADS;  // alpha values per thread (B + pad slot)
   const int Bp = (B + 2) & ~1;
   double* s_alpha = smem;
   double* s_mom = smem + Bp;
   const int tid = threadIdx.x;
   const int lane = tid & 63;
   const int wave = tid >> 6;
   constexpr int nwaves = THREADS / 64;
   const int nitems = ((nblocks + 7) / 8) * 8 * ngroups;
   const int G = gridDim.x;

   auto decode = [&](int it, int& b, int& g) {
      const int xcd = it & 7;
      const int rest = it >> 3;
      g = rest % ngroups;
      b = (rest / ngroups) * 8 + xcd;
   };
   auto next_valid = [&](int it) {
      while (it < nitems) {
         int bb, gg;
         decode(it, bb, gg);
         if (bb < nblocks) return it;
         it += G;
      }
      return nitems;
   };

   int it = next_valid(blockIdx.x);
   if (it >= nitems) return;
   int b, g;
   decode(it, b, g);
   // prologue of the first item: alpha into registers, first run into tile registers
   double areg[kPer];
   auto load_alpha = [&](int bb) {
      const int base = bb * B;
      const int nloc = min(B, n - base);
#pragma unroll
      for (int k = 0; k < kPer; k++) {
         const int i = tid + k * THREADS;
         areg[k] = (i < nloc) ? x[base + i] : 0.0;
      }
   };
   load_alpha(b);
   TileRegs cur;
   int t = tile_off[b * ngroups + g] + wave;
   if (t < tile_off[b * ngroups + g + 1]) load_tile(cur, meta, perm2, qarr, t, lane);

   while (true) {
      const int c0 = g * CG;
      const int t1 = tile_off[b * ngroups + g + 1];
      // stage alpha, clear moments
#pragma unroll
      for (int k = 0; k < kPer; k++) {
         const int i = tid + k * THREADS;
         if (i < Bp) s_alpha[i] = areg[k];
      }
      for (int i = tid; i < CG * kNos * kMomStride; i += THREADS) s_mom[i] = 0.0;
      __syncthreads();
      // next item: alpha loads in flight during this item's runs
      const int it_next = next_valid(it + G);
      int bn = 0, gn = 0;
      if (it_next < nitems) {
         decode(it_next, bn, gn);
         load_alpha(bn);
      }
      const int tfirst_next = (it_next < nitems) ? tile_off[bn * ngroups + gn] + wave : 0;
      const int tend_next = (it_next < nitems) ? tile_off[bn * ngroups + gn + 1] : 0;

      for (; t < t1; t += nwaves) {
         TileRegs nxt;
         const int tn = t + nwaves;
         // prefetch the next run: in this item, or the first run of the next item
         const int tpre = (tn < t1) ? tn : tfirst_next;
         const bool has_pre = (tn < t1) || (tfirst_next < tend_next);
         if (has_pre) load_tile(nxt, meta, perm2, qarr, tpre, lane);
         double acc[kNC];
#pragma unroll
         for (int d = 0; d < kNC; d++) acc[d] = 0.0;
#pragma unroll
         for (int r = 0; r < kR; r++) {
            const uint32_t loc = (r & 1) ? (cur.pp[r >> 1] >> 16) : (cur.pp[r >> 1] & 0xFFFFu);
            const double u = q_to_u(cur.qq[r]);
            double tpow = s_alpha[loc];
            acc[0] += tpow;
#pragma unroll
            for (int d = 1; d < kNC; d++) {
               tpow *= u;
               acc[d] += tpow;
            }
         }
         double* dst = s_mom + (((int)(cur.mt >> 6) - c0) * kNos + (int)(cur.mt & 63u)) * kMomStride;
#pragma unroll
         for (int d = 0; d < kNC; d++) atomicAdd(dst + d, acc[d]);  // ds_add_f64
         if (has_pre) cur = nxt;
      }
      // a wave whose run list of this item was empty still has to pick up the next item's first run
      if (t == tile_off[b * ngroups + g] + wave && t >= t1 && tfirst_next < tend_next)
         load_tile(cur, meta, perm2, qarr, tfirst_next, lane);
      __syncthreads();

      // fold: every thread, two partial sums of 5 taps each (independent chains), combined in LDS-free
      // registers via the pair lane (tid ^ 1 holds the other half of the same output)
      const int ncomp = min(CG, nw - c0);
      for (int idx = tid; idx < 2 * ncomp * kNos; idx += THREADS) {
         const int o = idx >> 1;
         const int half = idx & 1;
         const int cl = o / kNos;
         const int gi = o % kNos;
         // taps half*5 .. half*5+4; two interleaved accumulators (even / odd degree) per tap
         double s = 0.0;
#pragma unroll 1
         for (int j = 0; j < 5; j++) {
            const int tp = half * 5 + j;
            const double* mrow = s_mom + (cl * kNos + ((gi + kM - tp) & (kNos - 1))) * kMomStride;
            const double* crow = c_taps + tp * kNC;
            double a0 = 0.0, a1 = 0.0;
#pragma unroll
            for (int d = 0; d < kNC; d += 2) {
               a0 = fma(crow[d], mrow[d], a0);
               a1 = fma(crow[d + 1], mrow[d + 1], a1);
            }
            s += a0 + a1;
         }
         s += __shfl_xor(s, 1, 64);
         if (half == 0) part[((size_t)(c0 + cl) * nblocks + b) * kNos + gi] = s;
      }
      if (it_next >= nitems) break;
      __syncthreads();  // s_alpha / s_mom are overwritten by the next item
      it = it_next;
      b = bn;
      g = gn;
      t = tfirst_next;
   }
}

// ------------------------------------------------------------------------------------------------
// three-deep register ring: every wave keeps its next TWO runs in flight while it computes one
// (bytes in flight per CU, not VALU or LDS, bound the streaming rate of the one-deep kernels)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void spread_run(const TileRegs& T, const double* __restrict__ s_alpha,
                                           double* __restrict__ s_mom, int c0)
{
   double acc[kNC];
#pragma unroll
   for (int d = 0; d < kNC; d++) acc[d] = 0.0;
#pragma unroll
   for (int r = 0; r < kR; r++) {
      const uint32_t loc = (r & 1) ? (T.pp[r >> 1] >> 16) : (T.pp[r >> 1] & 0xFFFFu);
      const double u = q_to_u(T.qq[r]);
      double tpow = s_alpha[loc];
      acc[0] += tpow;
#pragma unroll
      for (int d = 1; d < kNC; d++) {
         tpow *= u;
         acc[d] += tpow;
      }
   }
   double* dst = s_mom + (((int)(T.mt >> 6) - c0) * kNos + (int)(T.mt & 63u)) * kMomStride;
#pragma unroll
   for (int d = 0; d < kNC; d++) atomicAdd(dst + d, acc[d]);  // ds_add_f64
}

template <int THREADS>
__global__ __launch_bounds__(THREADS) void k_spread3(
    const uint16_t* __restrict__ meta, const uint32_t* __restrict__ perm2, const uint32_t* __restrict__ qarr,
    const int* __restrict__ tile_off, const double* __restrict__ x, int n, int B, int nblocks, int ngroups, int CG,
    int nw, double* __restrict__ part)
{
   extern __shared__ __attribute__((aligned(16))) double smem[];
   const int Bp = (B + 2) & ~1;
   double* s_alpha = smem;
   double* s_mom = smem + Bp;
   const int xcd = blockIdx.x & 7;
   const int rest = blockIdx.x >> 3;
   const int g = rest % ngroups;
   const int b = (rest / ngroups) * 8 + xcd;
   if (b >= nblocks) return;
   const int tid = threadIdx.x;
   const int lane = tid & 63;
   const int wave = tid >> 6;
   constexpr int nwv = THREADS / 64;
   const int c0 = g * CG;
   const int t1 = tile_off[b * ngroups + g + 1];
   int t = tile_off[b * ngroups + g] + wave;
   TileRegs A, Bq, Cq;
   if (t < t1) load_tile(A, meta, perm2, qarr, t, lane);
   if (t + nwv < t1) load_tile(Bq, meta, perm2, qarr, t + nwv, lane);
   const int base = b * B;
   const int nloc = min(B, n - base);
   for (int i = tid; i < Bp; i += THREADS) s_alpha[i] = (i < nloc) ? x[base + i] : 0.0;
   for (int i = tid; i < CG * kNos * kMomStride; i += THREADS) s_mom[i] = 0.0;
   __syncthreads();
   while (true) {
      if (t + 2 * nwv < t1) load_tile(Cq, meta, perm2, qarr, t + 2 * nwv, lane);
      if (t >= t1) break;
      spread_run(A, s_alpha, s_mom, c0);
      t += nwv;
      if (t + 2 * nwv < t1) load_tile(A, meta, perm2, qarr, t + 2 * nwv, lane);
      if (t >= t1) break;
      spread_run(Bq, s_alpha, s_mom, c0);
      t += nwv;
      if (t + 2 * nwv < t1) load_tile(Bq, meta, perm2, qarr, t + 2 * nwv, lane);
      if (t >= t1) break;
      spread_run(Cq, s_alpha, s_mom, c0);
      t += nwv;
   }
   __syncthreads();
   const int ncomp = min(CG, nw - c0);
   for (int idx = tid; idx < ncomp * kNos; idx += THREADS) {
      const int cl = idx / kNos;
      const int gi = idx % kNos;
      double v = 0.0;
#pragma unroll 1
      for (int tp = 0; tp < kTaps; tp++) {
         const double* mrow = s_mom + (cl * kNos + ((gi + kM - tp) & (kNos - 1))) * kMomStride;
#pragma unroll
         for (int d = 0; d < kNC; d++) v = fma(c_taps[tp * kNC + d], mrow[d], v);
      }
      part[((size_t)(c0 + cl) * nblocks + b) * kNos + gi] = v;  // [comp][block][cell]
   }
}

template <bool GRAD>
__device__ __forceinline__ void interp_run(const TileRegs& T, const double* __restrict__ H,
                                           const double* __restrict__ Hd, double* __restrict__ s_y,
                                           double* __restrict__ s_yd)
{
   const size_t hoff = (size_t)T.mt * kNC;  // (comp*64 + cell) * kNC
   double hc[kNC], hdc[GRAD ? kNC : 1];
#pragma unroll
   for (int d = 0; d < kNC; d += 2) {
      const double2 v = *reinterpret_cast<const double2*>(H + hoff + d);
      hc[d] = v.x;
      hc[d + 1] = v.y;
      if (GRAD) {
         const double2 vd = *reinterpret_cast<const double2*>(Hd + hoff + d);
         hdc[d] = vd.x;
         hdc[d + 1] = vd.y;
      }
   }
#pragma unroll
   for (int r = 0; r < kR; r++) {
      const uint32_t loc = (r & 1) ? (T.pp[r >> 1] >> 16) : (T.pp[r >> 1] & 0xFFFFu);
      const double u = q_to_u(T.qq[r]);
      double v = hc[kNC - 1];
#pragma unroll
      for (int d = kNC - 2; d >= 0; d--) v = fma(v, u, hc[d]);
      atomicAdd(s_y + loc, v);
      if (GRAD) {
         double vd = hdc[kNC - 1];
#pragma unroll
         for (int d = kNC - 2; d >= 0; d--) vd = fma(vd, u, hdc[d]);
         atomicAdd(s_yd + loc, vd);
      }
   }
}

template <bool GRAD, int THREADS>
__global__ __launch_bounds__(THREADS) void k_interp3(
    const uint16_t* __restrict__ meta, const uint32_t* __restrict__ perm2, const uint32_t* __restrict__ qarr,
    const int* __restrict__ tile_off, const double* __restrict__ H, const double* __restrict__ Hd,
    const double* __restrict__ x, double* __restrict__ y, int n, int B, int ngroups, double alpha, double beta,
    double f, double mu)
{
   extern __shared__ __attribute__((aligned(16))) double smem[];
   const int Bp = (B + 2) & ~1;
   double* s_y = smem;
   double* s_yd = smem + Bp;
   const int b = blockIdx.x;
   const int tid = threadIdx.x;
   const int base = b * B;
   const int nloc = min(B, n - base);
   const int lane = tid & 63;
   const int wave = tid >> 6;
   constexpr int nwv = THREADS / 64;
   const int t1 = tile_off[(b + 1) * ngroups];
   int t = tile_off[b * ngroups] + wave;
   TileRegs A, Bq, Cq;
   if (t < t1) load_tile(A, meta, perm2, qarr, t, lane);
   if (t + nwv < t1) load_tile(Bq, meta, perm2, qarr, t + nwv, lane);
   for (int i = tid; i < Bp; i += THREADS) {
      s_y[i] = 0.0;
      if (GRAD) s_yd[i] = 0.0;
   }
   __syncthreads();
   while (true) {
      if (t + 2 * nwv < t1) load_tile(Cq, meta, perm2, qarr, t + 2 * nwv, lane);
      if (t >= t1) break;
      interp_run<GRAD>(A, H, Hd, s_y, s_yd);
      t += nwv;
      if (t + 2 * nwv < t1) load_tile(A, meta, perm2, qarr, t + 2 * nwv, lane);
      if (t >= t1) break;
      interp_run<GRAD>(Bq, H, Hd, s_y, s_yd);
      t += nwv;
      if (t + 2 * nwv < t1) load_tile(Bq, meta, perm2, qarr, t + 2 * nwv, lane);
      if (t >= t1) break;
      interp_run<GRAD>(Cq, H, Hd, s_y, s_yd);
      t += nwv;
   }
   __syncthreads();
   const double ff = f * f;
   for (int j = tid; j < nloc; j += THREADS) {
      const size_t gj = (size_t)base + j;
      const double xj = x[gj];
      if (!GRAD) {
         const double v = ff * (s_y[j] + mu * xj);
         y[gj] = (beta == 0.0) ? alpha * v : fma(beta, y[gj], alpha * v);
      } else {
         const double v0 = 2.0 * f * (s_y[j] + mu * xj);
         const double v1 = ff * s_yd[j];
         const double v2 = ff * xj;
         double* y0 = y;
         double* y1 = y + n;
         double* y2 = y + 2 * (size_t)n;
         if (beta == 0.0) {
            y0[gj] = alpha * v0;
            y1[gj] = alpha * v1;
            y2[gj] = alpha * v2;
         } else {
            y0[gj] = fma(beta, y0[gj], alpha * v0);
            y1[gj] = fma(beta, y1[gj], alpha * v1);
            y2[gj] = fma(beta, y2[gj], alpha * v2);
         }
      }
   }
}

// ------------------------------------------------------------------------------------------------
// spread with the grid step fused into its tail (default single-GPU path)
//   every workgroup adds its 64-cell partial grids into gsum[comp][64] with memory-side fp64 atomics,
//   then takes an arrival ticket for its window group; the LAST workgroup of the group reads the
//   sums back with returning atomics (coherent across XCDs), applies the circulant, writes the
//   interpolation polynomials H (and Hd), and clears gsum / the ticket for the next launch.
//   Protocol per MI355X_MICROARCH.md "Workgroup dispatch ... visibility": every adding wave drains
//   its atomics (s_waitcnt vmcnt(0)) before the workgroup barrier, one lane releases at agent scope
//   and takes the ticket; the last arriver acquires before reading.
// ------------------------------------------------------------------------------------------------
__device__ void fused_grid_tail(int comp, const double* __restrict__ s_g, const double* __restrict__ w,
                                double* __restrict__ H, double* s_w, double* s_h, int tid, int nthreads)
{
   // s_g: this component's summed grid (LDS); computes H[comp] with threads [0, nthreads)
   if (tid < kNos) s_w[tid] = w[(size_t)comp * kNos + tid];
   __syncthreads();
   if (tid < kNos) {
      double h = 0.0;
#pragma unroll 8
      for (int l2 = 0; l2 < kNos; l2++) h = fma(s_w[(tid - l2) & (kNos - 1)], s_g[l2], h);
      s_h[tid] = h;
   }
   __syncthreads();
   for (int idx = tid; idx < kNos * kNC; idx += nthreads) {
      const int cell = idx / kNC;
      const int d = idx % kNC;
      double v = 0.0;
#pragma unroll
      for (int tp = 0; tp < kTaps; tp++) v = fma(s_h[(cell - kM + tp) & (kNos - 1)], c_taps[tp * kNC + d], v);
      H[((size_t)comp * kNos + cell) * kNC + d] = v;
   }
   __syncthreads();
}

template <int THREADS>
__global__ __launch_bounds__(THREADS) void k_spread_fused(
    const uint16_t* __restrict__ meta, const uint32_t* __restrict__ perm2, const uint32_t* __restrict__ qarr,
    const int* __restrict__ tile_off, const double* __restrict__ x, int n, int B, int nblocks, int ngroups, int CG,
    int nw, double* __restrict__ gsum, unsigned int* __restrict__ tickets, const double* __restrict__ w,
    const double* __restrict__ wd, double* __restrict__ H, double* __restrict__ Hd, int grad)
{
   extern __shared__ __attribute__((aligned(16))) double smem[];
   __shared__ int s_last;
   __shared__ double s_w[kNos], s_h[kNos];
   const int Bp = (B + 2) & ~1;
   double* s_alpha = smem;
   double* s_mom = smem + Bp;
   const int xcd = blockIdx.x & 7;
   const int rest = blockIdx.x >> 3;
   const int g = rest % ngroups;
   const int b = (rest / ngroups) * 8 + xcd;
   if (b >= nblocks) return;
   const int tid = threadIdx.x;
   const int lane = tid & 63;
   const int wave = tid >> 6;
   constexpr int nwaves = THREADS / 64;
   const int c0 = g * CG;
   const int t0 = tile_off[b * ngroups + g];
   const int t1 = tile_off[b * ngroups + g + 1];
   TileRegs cur;
   int t = t0 + wave;
   if (t < t1) load_tile(cur, meta, perm2, qarr, t, lane);
   const int base = b * B;
   const int nloc = min(B, n - base);
   for (int i = tid; i < Bp; i += THREADS) s_alpha[i] = (i < nloc) ? x[base + i] : 0.0;
   for (int i = tid; i < CG * kNos * kMomStride; i += THREADS) s_mom[i] = 0.0;
   __syncthreads();
   for (; t < t1; t += nwaves) {
      double acc[kNC];
#pragma unroll
      for (int d = 0; d < kNC; d++) acc[d] = 0.0;
#pragma unroll
      for (int r = 0; r < kR; r++) {
         const uint32_t loc = (r & 1) ? (cur.pp[r >> 1] >> 16) : (cur.pp[r >> 1] & 0xFFFFu);
         const double u = q_to_u(cur.qq[r]);
         double tpow = s_alpha[loc];
         acc[0] += tpow;
#pragma unroll
         for (int d = 1; d < kNC; d++) {
            tpow *= u;
            acc[d] += tpow;
         }
      }
      double* dst = s_mom + (((int)(cur.mt >> 6) - c0) * kNos + (int)(cur.mt & 63u)) * kMomStride;
#pragma unroll
      for (int d = 0; d < kNC; d++) atomicAdd(dst + d, acc[d]);  // ds_add_f64
      if (t + nwaves < t1) load_tile(cur, meta, perm2, qarr, t + nwaves, lane);
   }
   __syncthreads();

   // fold into partial grids and add them to gsum (memory-side fp64 atomics, no return)
   const int ncomp = min(CG, nw - c0);
   for (int idx = tid; idx < ncomp * kNos; idx += THREADS) {
      const int cl = idx / kNos;
      const int gi = idx % kNos;
      double v = 0.0;
#pragma unroll 1
      for (int tp = 0; tp < kTaps; tp++) {
         const double* mrow = s_mom + (cl * kNos + ((gi + kM - tp) & (kNos - 1))) * kMomStride;
#pragma unroll
         for (int d = 0; d < kNC; d++) v = fma(c_taps[tp * kNC + d], mrow[d], v);
      }
      atomicAdd(gsum + (size_t)(c0 + cl) * kNos + gi, v);
   }
   asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every adding wave drains its atomics
   __syncthreads();
   if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned old = __hip_atomic_fetch_add(tickets + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = (old == (unsigned)(nblocks - 1)) ? 1 : 0;
   }
   __syncthreads();
   if (!s_last) return;
   __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
   asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
   __syncthreads();
   // last arriver of group g: summed grids -> LDS (returning atomics read the memory-side value and
   // clear it for the next launch), circulant, polynomials
   double* s_g = s_mom;  // reuse: ncomp*64 doubles
   for (int idx = tid; idx < ncomp * kNos; idx += THREADS) {
      double* p = gsum + (size_t)c0 * kNos + idx;
      s_g[idx] = __hip_atomic_exchange(p, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
   }
   __syncthreads();
   for (int cl = 0; cl < ncomp; cl++) {
      fused_grid_tail(c0 + cl, s_g + cl * kNos, w, H, s_w, s_h, tid, THREADS);
      if (grad) fused_grid_tail(c0 + cl, s_g + cl * kNos, wd, Hd, s_w, s_h, tid, THREADS);
   }
   if (tid == 0) __hip_atomic_store(tickets + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// copy the diagnostic timeline out (tools/ only)
extern "C" int Nfft4GPAmdDebugStamps(unsigned long long* out, int nwg)
{
   if (nwg > kMaxStampWG) nwg = kMaxStampWG;
   NFFT4GP_HIP_CHECK(hipDeviceSynchronize());
   NFFT4GP_HIP_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 4 * nwg));
   return nwg;
}

// ------------------------------------------------------------------------------------------------
// grid: sum partial grids, circulant, interpolation polynomials
// ------------------------------------------------------------------------------------------------
__device__ void grid_tail(int comp, const double* __restrict__ s_g, const double* __restrict__ w,
                          double* __restrict__ H, double* s_w, double* s_h)
{
   const int tid = threadIdx.x;
   if (tid < kNos) s_w[tid] = w[(size_t)comp * kNos + tid];
   __syncthreads();
   if (tid < kNos) {
      double h = 0.0;
#pragma unroll 8
      for (int l2 = 0; l2 < kNos; l2++) h = fma(s_w[(tid - l2) & (kNos - 1)], s_g[l2], h);
      s_h[tid] = h;
   }
   __syncthreads();
   for (int idx = tid; idx < kNos * kNC; idx += blockDim.x) {
      const int cell = idx / kNC;
      const int d = idx % kNC;
      double v = 0.0;
#pragma unroll
      for (int tp = 0; tp < kTaps; tp++) v = fma(s_h[(cell - kM + tp) & (kNos - 1)], c_taps[tp * kNC + d], v);
      H[((size_t)comp * kNos + cell) * kNC + d] = v;
   }
   __syncthreads();
}

// part: [nw][nparts][64] (from_sum = 0) or the summed grids [nw][64] (from_sum = 1)
__global__ __launch_bounds__(kGridThreads) void k_grid(const double* __restrict__ part, int nparts,
                                                      const double* __restrict__ w, const double* __restrict__ wd,
                                                      double* __restrict__ H, double* __restrict__ Hd, int grad,
                                                      int from_sum)
{
   __shared__ double s_red[kGridThreads];
   __shared__ double s_g[kNos];
   __shared__ double s_h[kNos];
   __shared__ double s_w[kNos];
   const int comp = blockIdx.x;
   const int tid = threadIdx.x;
   if (from_sum) {
      if (tid < kNos) s_g[tid] = part[(size_t)comp * kNos + tid];
   } else {
      // 16 strands per cell over this window's contiguous partial grids; 4 independent accumulators
      // per strand keep loads in flight; fixed order -> deterministic
      const int cell = tid & 63;
      const int strand = tid >> 6;
      constexpr int nstr = kGridThreads / 64;
      const double* src = part + (size_t)comp * nparts * kNos + cell;
      double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
      int p = strand;
      for (; p + 3 * nstr < nparts; p += 4 * nstr) {
         s0 += src[(size_t)p * kNos];
         s1 += src[(size_t)(p + nstr) * kNos];
         s2 += src[(size_t)(p + 2 * nstr) * kNos];
         s3 += src[(size_t)(p + 3 * nstr) * kNos];
      }
      for (; p < nparts; p += nstr) s0 += src[(size_t)p * kNos];
      s_red[tid] = (s0 + s1) + (s2 + s3);
      __syncthreads();
      if (tid < kNos) {
         double v = 0.0;
         for (int k = 0; k < nstr; k++) v += s_red[k * 64 + tid];
         s_g[tid] = v;
      }
   }
   __syncthreads();
   grid_tail(comp, s_g, w, H, s_w, s_h);
   if (grad) grid_tail(comp, s_g, wd, Hd, s_w, s_h);
}

// gsum[comp][cell] = sum_b part[comp][b][cell]   (row-sharded path: before the all-reduce)
__global__ __launch_bounds__(256) void k_reduce_parts(const double* __restrict__ part, int nparts, int nw,
                                                     double* __restrict__ gsum)
{
   const int idx = blockIdx.x * blockDim.x + threadIdx.x;
   if (idx >= nw * kNos) return;
   const int comp = idx / kNos, cell = idx % kNos;
   const double* src = part + (size_t)comp * nparts * kNos + cell;
   double s = 0.0;
   for (int p = 0; p < nparts; p++) s += src[(size_t)p * kNos];
   gsum[idx] = s;
}

// ------------------------------------------------------------------------------------------------
// interpolation + epilogue
// ------------------------------------------------------------------------------------------------
template <bool GRAD, int THREADS, bool PREFETCH, int ABL = 0>
__global__ __launch_bounds__(THREADS) void k_interp(
    const uint16_t* __restrict__ meta, const uint32_t* __restrict__ perm2, const uint32_t* __restrict__ qarr,
    const int* __restrict__ tile_off, const double* __restrict__ H, const double* __restrict__ Hd,
    const double* __restrict__ x, double* __restrict__ y, int n, int B, int ngroups, double alpha, double beta,
    double f, double mu)
{
   extern __shared__ __attribute__((aligned(16))) double smem[];
   const int Bp = (B + 2) & ~1;
   double* s_y = smem;
   double* s_yd = smem + Bp;  // GRAD only
   const int b = blockIdx.x;
   const int tid = threadIdx.x;
   const int base = b * B;
   const int nloc = min(B, n - base);
   const int lane = tid & 63;
   const int wave = tid >> 6;
   constexpr int nwaves = THREADS / 64;
   const int t0 = tile_off[b * ngroups];
   const int t1 = tile_off[(b + 1) * ngroups];
   TileRegs cur;
   int t = t0 + wave;
   if (t < t1) load_tile(cur, meta, perm2, qarr, t, lane);
   for (int i = tid; i < Bp; i += THREADS) {
      s_y[i] = 0.0;
      if (GRAD) s_yd[i] = 0.0;
   }
   __syncthreads();

   for (; t < t1; t += nwaves) {
      TileRegs nxt;
      const int tn = t + nwaves;
      if (PREFETCH && tn < t1) load_tile(nxt, meta, perm2, qarr, tn, lane);  // prefetch the next run
      const size_t hoff = (size_t)cur.mt * kNC;  // (comp*64 + cell) * kNC: meta is comp<<6|cell
      double hc[kNC], hdc[GRAD ? kNC : 1];
#pragma unroll
      for (int d = 0; d < kNC; d += 2) {
         const double2 v = *reinterpret_cast<const double2*>(H + hoff + d);
         hc[d] = v.x;
         hc[d + 1] = v.y;
         if (GRAD) {
            const double2 vd = *reinterpret_cast<const double2*>(Hd + hoff + d);
            hdc[d] = vd.x;
            hdc[d + 1] = vd.y;
         }
      }
#pragma unroll
      for (int r = 0; r < kR; r++) {
         const uint32_t loc = (r & 1) ? (cur.pp[r >> 1] >> 16) : (cur.pp[r >> 1] & 0xFFFFu);
         const double u = q_to_u(cur.qq[r]);
         double v = hc[kNC - 1];
         if (ABL == 1) {
            v = u;
         } else {
#pragma unroll
            for (int d = kNC - 2; d >= 0; d--) v = fma(v, u, hc[d]);
         }
         if (ABL == 2) {
            if (v == 12345.0) s_y[loc] = v;
         } else {
            atomicAdd(s_y + loc, v);
         }
         if (GRAD) {
            double vd = hdc[kNC - 1];
#pragma unroll
            for (int d = kNC - 2; d >= 0; d--) vd = fma(vd, u, hdc[d]);
            atomicAdd(s_yd + loc, vd);
         }
      }
      if (PREFETCH) {
         if (tn < t1) cur = nxt;
      } else if (tn < t1) {
         load_tile(cur, meta, perm2, qarr, tn, lane);
      }
   }
   __syncthreads();

   const double ff = f * f;
   for (int j = tid; j < nloc; j += THREADS) {
      const size_t gj = (size_t)base + j;
      const double xj = x[gj];
      if (!GRAD) {
         const double v = ff * (s_y[j] + mu * xj);
         y[gj] = (beta == 0.0) ? alpha * v : fma(beta, y[gj], alpha * v);
      } else {
         // nfft_interface.c:547-549 summed over windows: (2f)(Kx + mu x), ff*dscale*K'x, ff*x
         const double v0 = 2.0 * f * (s_y[j] + mu * xj);
         const double v1 = ff * s_yd[j];
         const double v2 = ff * xj;
         double* y0 = y;
         double* y1 = y + n;
         double* y2 = y + 2 * (size_t)n;
         if (beta == 0.0) {
            y0[gj] = alpha * v0;
            y1[gj] = alpha * v1;
            y2[gj] = alpha * v2;
         } else {
            y0[gj] = fma(beta, y0[gj], alpha * v0);
            y1[gj] = fma(beta, y1[gj], alpha * v1);
            y2[gj] = fma(beta, y2[gj], alpha * v2);
         }
      }
   }
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
static size_t spread_lds_bytes(const AdditivePlan& P)
{
   const int Bp = (P.B + 2) & ~1;
   return sizeof(double) * ((size_t)Bp + (size_t)P.CG * kNos * kMomStride);
}

static size_t interp_lds_bytes(const AdditivePlan& P, int grad)
{
   const int Bp = (P.B + 2) & ~1;
   return sizeof(double) * (size_t)Bp * (grad ? 2 : 1);
}

int upload_tap_coeffs()
{
   // constant memory is per device: upload once per device this process uses
   static bool done[64] = {false};
   int dev = 0;
   NFFT4GP_HIP_CHECK(hipGetDevice(&dev));
   if (dev < 0 || dev >= 64) return -1;
   if (!done[dev]) {
      const std::vector<double>& C = tap_poly_coeffs();
      NFFT4GP_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_taps), C.data(), sizeof(double) * kTaps * kNC));
      done[dev] = true;
   }
   return 0;
}

typedef void (*SpreadFn)(const uint16_t*, const uint32_t*, const uint32_t*, const int*, const double*, int, int, int,
                         int, int, int, double*);
struct SpreadVariant {
   SpreadFn fn;
   int threads;
   int persistent_bmax = 0;  // > 0: persistent kernel for blocks up to this size
};
static const SpreadVariant kSpreadVariants[] = {
    {k_spread<512, 1, true>, 512},   // 0: 8 waves, next-run prefetch
    {k_spread<512, 1, false>, 512},  // 1: 8 waves, no prefetch
    {k_spread<256, 1, true>, 256},   // 2: 4 waves, prefetch
    {k_spread<512, 3, false>, 512},  // 3: 8 waves, >= 3 waves/SIMD register budget, no prefetch
    {k_spread<1024, 1, false>, 1024},  // 4: 16 waves, no prefetch
    // ablations for timing experiments only (WRONG results): 5 no alpha gather, 6 no powers, 7 no flush
    {k_spread<512, 1, false, 1>, 512},
    {k_spread<512, 1, false, 2>, 512},
    {k_spread<512, 1, false, 3>, 512},
    // contiguous wave ranges + flush on key change: 8 contig 512 thr, 9 contig 256 thr, 10 contig 1024 thr
    {k_spread<512, 1, true, 0, true>, 512},
    {k_spread<256, 1, true, 0, true>, 256},
    {k_spread<1024, 1, true, 0, true>, 1024},
    // 11/12: mixed-precision high moments + up-front alpha gathers (prefetch / no prefetch)
    {k_spread<512, 1, true, 4>, 512},
    {k_spread<512, 1, false, 4>, 512},
    // 13: diagnostic timeline build of variant 1 (s_memrealtime stamps per workgroup)
    {k_spread<512, 1, false, 5>, 512},
    // 14: persistent workgroups, next-item alpha/run prefetch (B <= 4096)
    {k_spread_persist<512, 4096>, 512, 4096},
    // 15: persistent, 256 threads
    {k_spread_persist<256, 4096>, 256, 4096},
    // 16/17: three-deep run ring
    {k_spread3<512>, 512},
    {k_spread3<256>, 256},
};
constexpr int kNumSpreadVariants = sizeof(kSpreadVariants) / sizeof(kSpreadVariants[0]);

typedef void (*InterpFn)(const uint16_t*, const uint32_t*, const uint32_t*, const int*, const double*,
                         const double*, const double*, double*, int, int, int, double, double, double, double);
struct InterpVariant {
   InterpFn fn, fn_grad;
   int threads;
};
static const InterpVariant kInterpVariants[] = {
    {k_interp<false, 1024, true>, k_interp<true, 1024, true>, 1024},  // 0
    {k_interp<false, 1024, false>, k_interp<true, 1024, false>, 1024},  // 1
    {k_interp<false, 512, true>, k_interp<true, 512, true>, 512},  // 2
    // ablations (WRONG results): 3 no H gather/Horner, 4 no LDS atomics
    {k_interp<false, 1024, false, 1>, k_interp<true, 1024, false, 1>, 1024},
    {k_interp<false, 1024, false, 2>, k_interp<true, 1024, false, 2>, 1024},
    // 5/6: three-deep run ring
    {k_interp3<false, 1024>, k_interp3<true, 1024>, 1024},
    {k_interp3<false, 512>, k_interp3<true, 512>, 512},
};
constexpr int kNumInterpVariants = sizeof(kInterpVariants) / sizeof(kInterpVariants[0]);

static void raise_lds_limit_once()
{
   static bool raised = false;
   if (raised) return;
   for (int i = 0; i < kNumSpreadVariants; i++)
      (void)hipFuncSetAttribute((const void*)kSpreadVariants[i].fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
   for (int i = 0; i < kNumInterpVariants; i++) {
      (void)hipFuncSetAttribute((const void*)kInterpVariants[i].fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
      (void)hipFuncSetAttribute((const void*)kInterpVariants[i].fn_grad,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
   }
   (void)hipGetLastError();
   raised = true;
}

int launch_spread(const AdditivePlan& P, const double* d_x, double* d_part, hipStream_t stream)
{
   if (P.dl.ntiles == 0 || P.n == 0) return 0;
   raise_lds_limit_once();
   const SpreadVariant& V = kSpreadVariants[std::min(std::max(P.spread_variant, 0), kNumSpreadVariants - 1)];
   const size_t lds = spread_lds_bytes(P);
   int gridx = ((P.nblocks + 7) / 8) * 8 * P.ngroups;
   if (V.persistent_bmax > 0) {
      if (P.B > V.persistent_bmax) {
         fprintf(stderr, "nfft4gp_amd: block size %d exceeds the persistent spread kernel's %d\n", P.B,
                 V.persistent_bmax);
         return -1;
      }
      // resident workgroups: occupancy x CUs, a multiple of 8 (item -> XCD affinity), at most the items
      static int cached_dev = -1, cached_cus = 0;
      int dev = 0;
      NFFT4GP_HIP_CHECK(hipGetDevice(&dev));
      if (dev != cached_dev) {
         NFFT4GP_HIP_CHECK(hipDeviceGetAttribute(&cached_cus, hipDeviceAttributeMultiprocessorCount, dev));
         cached_dev = dev;
      }
      int per_cu = 0;
      NFFT4GP_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)V.fn, V.threads, lds));
      int G = std::max(1, per_cu) * cached_cus;
      G = std::max(8, (G / 8) * 8);
      gridx = std::min(gridx, G);
   }
   hipLaunchKernelGGL(V.fn, dim3(gridx), dim3(V.threads), lds, stream, P.dl.meta, P.dl.perm2, P.dl.q,
                      P.dl.tile_off, d_x, P.n, P.B, P.nblocks, P.ngroups, P.CG, P.nw, d_part);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int launch_spread_fused(const AdditivePlan& P, const double* d_x, int grad, hipStream_t stream)
{
   if (P.n == 0) return 0;
   raise_lds_limit_once();
   static bool raised = false;
   if (!raised) {
      (void)hipFuncSetAttribute((const void*)k_spread_fused<512>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
      (void)hipGetLastError();
      raised = true;
   }
   const size_t lds = spread_lds_bytes(P);
   const int gridx = ((P.nblocks + 7) / 8) * 8 * P.ngroups;
   hipLaunchKernelGGL(k_spread_fused<512>, dim3(gridx), dim3(512), lds, stream, P.dl.meta, P.dl.perm2, P.dl.q,
                      P.dl.tile_off, d_x, P.n, P.B, P.nblocks, P.ngroups, P.CG, P.nw, P.d_grid, P.d_tickets, P.d_w,
                      P.d_wd, P.d_H, P.d_Hd, grad);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int launch_grid(const AdditivePlan& P, const double* d_part, int nparts, int grad, hipStream_t stream)
{
   hipLaunchKernelGGL(k_grid, dim3(P.nw), dim3(kGridThreads), 0, stream, d_part, nparts, P.d_w, P.d_wd, P.d_H,
                      P.d_Hd, grad, 0);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int launch_grid_from_sum(const AdditivePlan& P, const double* d_gridsum, int grad, hipStream_t stream)
{
   hipLaunchKernelGGL(k_grid, dim3(P.nw), dim3(kGridThreads), 0, stream, d_gridsum, 1, P.d_w, P.d_wd, P.d_H,
                      P.d_Hd, grad, 1);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int launch_reduce_parts(const AdditivePlan& P, const double* d_part, double* d_gridsum, hipStream_t stream)
{
   const int total = P.nw * kNos;
   hipLaunchKernelGGL(k_reduce_parts, dim3((total + 255) / 256), dim3(256), 0, stream, d_part, P.nblocks, P.nw,
                      d_gridsum);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int launch_interp(const AdditivePlan& P, int grad, double alpha, const double* d_x, double beta, double* d_y,
                  hipStream_t stream)
{
   if (P.n == 0) return 0;
   raise_lds_limit_once();
   const InterpVariant& V = kInterpVariants[std::min(std::max(P.interp_variant, 0), kNumInterpVariants - 1)];
   const size_t lds = interp_lds_bytes(P, grad);
   hipLaunchKernelGGL(grad ? V.fn_grad : V.fn, dim3(P.nblocks), dim3(V.threads), lds, stream, P.dl.meta, P.dl.perm2,
                      P.dl.q, P.dl.tile_off, P.d_H, P.d_Hd, d_x, d_y, P.n, P.B, P.ngroups, alpha, beta, P.f, P.mu);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

}  // namespace nfft4gp_amd
