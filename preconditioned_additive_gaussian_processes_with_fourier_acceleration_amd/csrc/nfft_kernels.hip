// nfft_kernels.hip -- CDNA4 (gfx950) kernels of the additive NFFT matvec.
//
// Per matvec three launches on one stream (see internal.h for the algebra):
//   k_spread  one workgroup per (block of B points, group of CG windows).  The workgroup stages the
//             block's alpha slice (B doubles) in LDS once for its windows (by LDS-DMA,
//             global_load_lds_dwordx4: no VGPR round trip, 46.7 -> 43.1 us at config C); each lane walks one R-point
//             run of a single (window, cell), accumulates the kNC = 10 moments alpha*u^d in registers and
//             flushes them with ds_add_f64 into an LDS moment table; the workgroup finally folds the
//             moments into 64-cell partial grids (taps = C * M) and writes them to part[comp][block].
//             HBM: 5 B per (point, window) -- 12-bit local index + 26-bit offset in the cell -- + alpha.
//   k_grid    one workgroup per window: sum of the partial grids (fixed order, deterministic), the
//             64x64 real circulant (= FFT . diag(bhat/phihut^2) . IFFT restricted to Re), and the
//             per-cell interpolation polynomials H = C^T h.
//   k_interp  one workgroup per block: lanes walk the same runs, load H[comp][cell] once per run,
//             Horner per point, ds_add_f64 into an LDS y-block; the epilogue applies
//             y = beta*y + alpha*ff*(sum + mu*x) (grad: the three outputs of nfft_interface.c:547-549)
//             in one coalesced pass.
// Rejected experiments (persistent workgroups, prefetching runs, three-deep run rings, mixed-precision moments,
// the grid step fused into the spread tail) are in the git history; DESIGN.md 3.5 has their numbers.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "internal.h"
#include "reduce.hpp"

namespace nfft4gp_amd {

constexpr int kGridThreads = 1024;
// The spread's LDS moment table of a window group.  MOMT 1 (the default): [window][degree][cell], kMomWin
// doubles per window (kNC x 64 plus 4: the windows' tables start 4 banks apart), so a run's 10 flushes are
// one address each 64 doubles apart and the fold's lanes (consecutive cells) read consecutive doubles; 20.6 KB
// for 4 windows, which with a 4064-point alpha slice still fits three workgroups per CU.  MOMT 0 (round 4):
// [window][cell][degree] rows of kMomStride = 11 doubles (3 windows: 16.9 KB; 4 would not fit three per CU).
constexpr int kMomStride = kNC + 1;
constexpr int kMomWin = kNC * kNos + 4;
template <int MOMT>
__host__ __device__ constexpr int mom_doubles_per_window()
{
   return MOMT ? kMomWin : kNos * kMomStride;
}
template <int MOMT>
__device__ __forceinline__ int mom_index(int cl, int cell, int d)
{
   return MOMT ? cl * kMomWin + d * kNos + cell : (cl * kNos + cell) * kMomStride + d;
}

// the point's centred offset in its cell scaled by 2^32, s = 2^32 u: the q word read as int32 (slot_word,
// internal.h) -- one conversion, no mask, no scale (the tap coefficients below carry the 2^-32d; scaling by
// powers of two is exact, so the moments, H and Horner are those of u, bit for bit)
__device__ __forceinline__ double q_to_s(uint32_t q) { return (double)(int)q; }

// tap polynomial coefficients C[t][d] 2^-32d (monomials in s = 2^32 u) in constant memory: wave-uniform reads
// become scalar loads; c_taps_u: C[t][d] itself (monomials in u: the 32-bit mode's fp32 moments)
__constant__ double c_taps[kTaps * kNC];
__constant__ double c_taps_u[kTaps * kNC];
typedef float f32x2 __attribute__((ext_vector_type(2)));

// diagnostic timeline (TIMELINE builds only): per workgroup 4 s_memrealtime stamps (100 MHz)
constexpr int kMaxStampWG = 16384;
__device__ unsigned long long g_stamps[kMaxStampWG * 4];

__device__ __forceinline__ void stamp(int slot)
{
   if (threadIdx.x == 0 && blockIdx.x < kMaxStampWG)
      g_stamps[blockIdx.x * 4 + slot] = __builtin_amdgcn_s_memrealtime();
}

struct TileRegs {
   uint32_t mt;
   uint32_t lo[kR / 4];  // local index bits 4-11, one byte per point
   uint32_t qq[kR];      // slot_word (internal.h): offset in the cell, bit 31 flipped; bits 0-3 = local index bits 0-3
};

// REC: the layout's record (AdditivePlan::rec): 5 bytes (q word + lo byte) or 4 (slot_word4: no lo array)
template <int REC = 5>
__device__ __forceinline__ void load_tile(TileRegs& T, const uint16_t* __restrict__ meta,
                                          const uint32_t* __restrict__ lo, const uint32_t* __restrict__ qarr,
                                          int t, int lane)
{
   // 16 B per lane per load: lo quads [t][1][lane], q quads [t][4][lane] (layout.cpp)
   T.mt = meta[(size_t)t * 64 + lane];
   const uint4* l4 = reinterpret_cast<const uint4*>(lo) + (size_t)t * (kR / 16) * 64 + lane;
   const uint4* q4 = reinterpret_cast<const uint4*>(qarr) + (size_t)t * (kR / 4) * 64 + lane;
#pragma unroll
   for (int k = 0; k < (REC == 5 ? kR / 16 : 0); k++) {
      const uint4 v = l4[k * 64];
      T.lo[4 * k + 0] = v.x;
      T.lo[4 * k + 1] = v.y;
      T.lo[4 * k + 2] = v.z;
      T.lo[4 * k + 3] = v.w;
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

// byte offset of point r's entry in a block's LDS slice of doubles: 8 x the local index (0..B-1, or B + lane % 32
// for a dummy slot), whose bits 4-11 are the lo byte and bits 0-3 the low bits of the q word
template <int REC = 5>
__device__ __forceinline__ uint32_t slot_off(const TileRegs& T, int r)
{
   if (REC == 4) return (T.qq[r] << 3) & 0x7FF8u;  // slot_word4: the whole index in bits 0-11
   // v_lshlrev_b32_sdwa (the byte, shifted) + v_lshlrev_b32 + v_and_or_b32: left to itself the compiler adds the
   // two fields and the slice's LDS base 0 with an extra v_and + v_add3
   const uint32_t hi = ((T.lo[r >> 2] >> (8 * (r & 3))) & 255u) << 7;
   uint32_t off;
   asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(off) : "v"(T.qq[r] << 3), "s"(0x78u), "v"(hi));
   return off;
}

template <class V>
__device__ __forceinline__ V* at_off(V* base, uint32_t byte_off)
{
   return reinterpret_cast<V*>(reinterpret_cast<char*>(base) + byte_off);
}

// the double at LDS byte address `byte_off`: the first dynamic slice of a kernel WITHOUT static LDS starts at LDS
// address 0 (the launchers check that the kernel's static LDS is 0 bytes: static_lds_zero).  Through the extern
// __shared__ pointer the compiler adds the slice base (a link-time constant) to every per-point offset, one VALU
// add per point
typedef __attribute__((address_space(3))) double lds_f64;
__device__ __forceinline__ lds_f64* lds_at(uint32_t byte_off) { return (lds_f64*)(size_t)byte_off; }
// ds_add_f64 at LDS byte address byte_off (the same convention)
__device__ __forceinline__ void lds_add(uint32_t byte_off, double v)
{
   (void)__hip_atomic_fetch_add(lds_at(byte_off), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Stage x[base, base + nloc) of a block into LDS (zero beyond nloc, up to B, plus kPad zero entries that the
// layout's dummy slots point at) by LDS-DMA (global_load_lds_dwordx4): each wave moves 1 KB pieces straight into LDS (lane l
// lands at the wave-uniform base + 16 l), no VGPR round trip and no ds_write; the ragged tail and the pad go
// through plain stores.  The caller waits vmcnt(0) before the barrier that publishes the slice.
template <int THREADS>
__device__ __forceinline__ void stage_block_glds(double* __restrict__ s, const double* __restrict__ x, int base,
                                                 int nloc, int B)
{
   const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
   const double* src = x + base;
   const int nfull = ((reinterpret_cast<uintptr_t>(src) & 15) == 0) ? nloc / 128 : 0;  // whole 1 KB pieces
   for (int p = wave; p < nfull; p += THREADS / 64)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 128 * p + 2 * lane),
                                       (__attribute__((address_space(3))) void*)(s + 128 * p), 16, 0, 0);
   for (int e = 128 * nfull + tid; e < B + kPad; e += THREADS) s[e] = e < nloc ? src[e] : 0.0;
}

// ------------------------------------------------------------------------------------------------
// spread
// ------------------------------------------------------------------------------------------------
// DET (deterministic spread): every run's moment is rounded, before its ds_add_f64 into the moment
// table, to a multiple of ulp(C_d), C_d = 1.5 2^E_d, with E_d chosen so that every partial sum of a table entry is
// a multiple of that ulp below 2^(E_d + 1): the additions are then exact, so the table -- and the whole spread --
// does not depend on the order the waves flush in.  The bound: |M_d| <= cm max|alpha| 2^31d (cm = the most
// points of one (window, cell) in the workgroup, from the layout; |s| <= 2^31), a run's |moment| <= 16 max|alpha|
// 2^31d, so E_d = e(max|alpha|) + max(log2 cm, 6) + 1 + 31 d.  Rounding costs ~2^-45 of a cell's moment.
__device__ __forceinline__ double det_grid(uint32_t bexp)  // 1.5 x 2^(bexp - 1023) (bexp: a biased exponent)
{
   return __hiloint2double((int)((bexp << 20) | 0x80000u), 0);
}
__device__ __forceinline__ double det_round(double v, double C) { return (v + C) - C; }

// The biased exponent field of max |alpha| over the block's staged slice (hi words: exact in any order), without a
// second barrier: after the staging barrier each wave takes the max of its eighth of the LDS slice, publishes it in
// s_red[wave] and counts itself in s_red[nwaves] (release); a wave reads the total only before its first flush
// (det_max_wait: acquire-spin, normally satisfied at once -- every wave published before it computed a run).
template <int THREADS>
__device__ __forceinline__ void det_max_publish(const double* s_alpha, int nloc, uint32_t* s_red)
{
   constexpr int nwaves = THREADS / 64;
   const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
   const int per = (nloc + nwaves - 1) / nwaves;
   const uint32_t* hw = reinterpret_cast<const uint32_t*>(s_alpha);
   uint32_t m = 0;
   for (int e = wave * per + lane; e < min(nloc, (wave + 1) * per); e += 64) m = max(m, hw[2 * e + 1] & 0x7FFFFFFFu);
   for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
   if (lane == 0) {
      s_red[wave] = m;
      __hip_atomic_fetch_add(s_red + nwaves, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
   }
}
template <int THREADS>
__device__ __forceinline__ uint32_t det_max_wait(uint32_t* s_red)
{
   constexpr int nwaves = THREADS / 64;
   while (__hip_atomic_load(s_red + nwaves, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < (uint32_t)nwaves)
      __builtin_amdgcn_s_sleep(1);
   uint32_t m = 0;
#pragma unroll
   for (int w = 0; w < nwaves; w++) m = max(m, s_red[w]);
   return (uint32_t)__builtin_amdgcn_readfirstlane((int)m) >> 20;
}

// DET interpolation: y_j sums one value per window, |f_c| <= hb[c] (k_grid), so with Y = sum_c hb[c] every partial
// sum is below Y: each value is rounded to a multiple of ulp(C), C = 1.5 2^(e(Y) + 2), and the ds_add_f64 sums are
// exact (order-independent).  Returns the biased exponent of C.
__device__ __forceinline__ uint32_t det_interp_exp(const double* __restrict__ hb, int nw)
{
   double Y = 0.0;
   for (int c = 0; c < nw; c++) Y += hb[c];
   const uint32_t bY = ((uint32_t)__double2hiint(Y) >> 20) & 0x7FFu;
   return min(bY + 2u, 2046u);
}

// at most 80 VGPRs, so three 512-thread workgroups (24 waves) share a CU
// PIPE (variant 3, layouts past the Infinity Cache): the next tile's loads issued before the current tile's moments
template <int THREADS, bool TIMELINE = false, int MOMT = 1, bool DET = false, int REC = 5, bool PIPE = false>
__global__ __launch_bounds__(THREADS, 6) void k_spread(const uint16_t* __restrict__ meta,
                                                      const uint32_t* __restrict__ lo,
                                                      const uint32_t* __restrict__ qarr,
                                                      const int* __restrict__ tile_off, const int* __restrict__ cmax,
                                                      const double* __restrict__ x, int n, int B, int nblocks,
                                                      int ngroups, int CG, int nw, double* __restrict__ part,
                                                      double* __restrict__ gsum)
{
   extern __shared__ __attribute__((aligned(16))) double smem[];
   const int Bp = B + kPad;
   double* s_alpha = smem;     // Bp
   double* s_mom = smem + Bp;  // CG windows' moment tables (mom_index)
   uint32_t* s_red = reinterpret_cast<uint32_t*>(s_mom + CG * mom_doubles_per_window<MOMT>());  // DET: nwaves

   // One workgroup = one block of points x one group of CG windows.  XCD-aware decode: the groups of one
   // block land on one XCD (blockIdx % 8), so its alpha slice is read into one L2.  Placement is speed only.
   const int xcd = blockIdx.x & 7;
   const int rest = blockIdx.x >> 3;
   const int g = rest % ngroups;
   const int b = (rest / ngroups) * 8 + xcd;
   if (b >= nblocks) return;
   if (TIMELINE) stamp(0);

   const int tid = threadIdx.x;
   const int lane = tid & 63;
   const int wave = tid >> 6;
   constexpr int nwaves = THREADS / 64;

   // the first run's loads and the alpha slice are in flight together
   TileRegs cur, nxt;
   const int t1 = tile_off[b * ngroups + g + 1];
   int t = tile_off[b * ngroups + g] + wave;
   if (t < t1) load_tile<REC>(cur, meta, lo, qarr, t, lane);
   const int base = b * B;
   stage_block_glds<THREADS>(s_alpha, x, base, min(B, n - base), B);
   for (int i = tid; i < CG * mom_doubles_per_window<MOMT>(); i += THREADS) s_mom[i] = 0.0;
   if (DET && tid == 0) s_red[nwaves] = 0u;
   asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA pieces have landed
   __syncthreads();
   if (TIMELINE) stamp(1);
   // DET: the rounding grids C_d (biased exponent of C_0, + 31 d), wave-uniform, formed once before the runs (the
   // wait is for the other waves' maxima of the slice, published right after the barrier)
   double Cd[kNC];
   if (DET) {
      det_max_publish<THREADS>(s_alpha, min(B, n - base), s_red);
      const int cm = cmax[b * ngroups + g];
      const uint32_t lcm = max(cm > 1 ? 32u - (uint32_t)__clz(cm - 1) : 0u, 6u) + 1u;
      const uint32_t bC0 = det_max_wait<THREADS>(s_red) + lcm;
#pragma unroll
      for (int d = 0; d < kNC; d++) Cd[d] = det_grid(REC == 4 ? bC0 : bC0 + 31u * d);
   }

   const int c0 = g * CG;
   for (; t < t1; t += nwaves) {
      if (PIPE && t + nwaves < t1) load_tile<REC>(nxt, meta, lo, qarr, t + nwaves, lane);
      double acc[kNC];
      if constexpr (REC == 4) {
         // the 32-bit mode (BASELINE configs[4]: fp32 matvec, fp64 accumulation): a run's moments in fp32, two
         // degrees per packed instruction (v_pk_mul_f32 / v_pk_add_f32), u = the offset in the cell - 1/2 (not
         // scaled by 2^32: fp32 would overflow; the fold uses the unscaled taps), flushed into the fp64 table
         static_assert(kNC == 8, "the packed moment chain is written for degree 7");
         f32x2 m01 = {0.f, 0.f}, m23 = {0.f, 0.f}, m45 = {0.f, 0.f}, m67 = {0.f, 0.f};
#pragma unroll
         for (int r = 0; r < kR; r++) {
            const float u = (float)(int)cur.qq[r] * 0x1p-32f;
            const float al = (float)*lds_at(slot_off<REC>(cur, r));  // s_alpha is the first dynamic slice
            const float u2 = u * u;
            f32x2 p = {al, al * u};
            m01 += p;
            p *= u2;
            m23 += p;
            p *= u2;
            m45 += p;
            p *= u2;
            m67 += p;
         }
         acc[0] = m01.x, acc[1] = m01.y, acc[2] = m23.x, acc[3] = m23.y;
         acc[4] = m45.x, acc[5] = m45.y, acc[6] = m67.x, acc[7] = m67.y;
      } else {
#pragma unroll
         for (int d = 0; d < kNC; d++) acc[d] = 0.0;
#pragma unroll
         for (int r = 0; r < kR; r++) {
            const double u = q_to_s(cur.qq[r]);
            double tpow = *lds_at(slot_off<REC>(cur, r));  // s_alpha is the first dynamic slice
            acc[0] += tpow;
#pragma unroll
            for (int d = 1; d < kNC; d++) {
               tpow *= u;
               acc[d] += tpow;
            }
         }
      }
      const int comp_local = (int)(cur.mt >> 6) - c0;
      const int cell = (int)(cur.mt & 63u);
      double* dst = s_mom + mom_index<MOMT>(comp_local, cell, 0);
#pragma unroll
      for (int d = 0; d < kNC; d++) {
         // (32-bit mode: moments in u, |u| <= 1/2, so one grid for every degree)
         const double a = DET ? det_round(acc[d], Cd[d]) : acc[d];
         atomicAdd(dst + mom_index<MOMT>(0, 0, d), a);  // ds_add_f64
      }
      if (PIPE)
         cur = nxt;
      else if (t + nwaves < t1)
         load_tile<REC>(cur, meta, lo, qarr, t + nwaves, lane);
   }
   __syncthreads();
   if (TIMELINE) stamp(2);

   // fold moments into the 64-cell partial grid of every window of this group:
   //   g[gi] = sum_t sum_d C[t][d] M[(gi + m - t) mod 64][d]
   const int ncomp = min(CG, nw - c0);
   for (int idx = tid; idx < ncomp * kNos; idx += THREADS) {
      const int cl = idx / kNos;
      const int gi = idx % kNos;
      double v = 0.0;
#pragma unroll 1
      for (int tp = 0; tp < kTaps; tp++) {
         const double* mrow = s_mom + mom_index<MOMT>(cl, (gi + kM - tp) & (kNos - 1), 0);
#pragma unroll
         for (int d = 0; d < kNC; d++)
            v = fma((REC == 4 ? c_taps_u : c_taps)[tp * kNC + d], mrow[mom_index<MOMT>(0, 0, d)], v);
      }
      if (gsum)
         atomicAdd(gsum + (size_t)(c0 + cl) * kNos + gi, v);  // launch_spread_grid's atomic sum
      else
         part[((size_t)(c0 + cl) * nblocks + b) * kNos + gi] = v;  // [comp][block][cell]
   }
   if (TIMELINE) {
      __syncthreads();
      stamp(3);
   }
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
// circulant h = w (*) g, then H[cell][d] = sum_t h[cell - m + t] C[t][d].  The circulant runs as 16
// strands of 4 terms per output summed in a fixed butterfly inside the wave (blockDim >= 1024: 4 outputs
// x 16 strands per wave); one 64-term chain per output was bound by its dependent LDS reads.
// wreg: this thread's circulant entry w[comp][tid] (tid < 64); ct: the tap coefficients C[t][tid % kNC] of this
// thread's output H[tid / kNC][tid % kNC] (tid < 64 kNC; blockDim == kGridThreads >= 64 kNC).  Both are
// loaded by the caller at kernel entry, so their latency overlaps the grid loads instead of following the
// last barrier.
__device__ __forceinline__ void grid_tail_coeffs(double (&ct)[kTaps])
{
   const int tid = threadIdx.x;
   const int d = tid % kNC;
#pragma unroll
   for (int tp = 0; tp < kTaps; tp++) ct[tp] = tid < kNos * kNC ? c_taps[tp * kNC + d] : 0.0;
}

// hb (det, may be NULL): hb[comp] = max over cells of sum_d |H[cell][d]| 2^31d, a bound on |f(s)| for |s| <= 2^31
// (the interpolation's rounding grid); s_scr: kNos * kNC doubles of LDS scratch when hb is given
__device__ void grid_tail(int comp, const double* __restrict__ s_g, double wreg, const double (&ct)[kTaps],
                          double* __restrict__ H, double* s_w, double* s_h, double* __restrict__ hb = nullptr,
                          double* s_scr = nullptr)
{
   static_assert(kGridThreads >= kNos * kNC, "one H entry per thread");
   const int tid = threadIdx.x;
   if (tid < kNos) s_w[tid] = wreg;
   __syncthreads();
   {
      const int o = tid >> 4, st = tid & 15;
      double h = 0.0;
      if (o < kNos) {
#pragma unroll
         for (int k = 0; k < 4; k++) {
            const int l2 = st * 4 + k;
            h = fma(s_w[(o - l2) & (kNos - 1)], s_g[l2], h);
         }
      }
      for (int off = 8; off > 0; off >>= 1) h += __shfl_xor(h, off, 64);
      if (o < kNos && st == 0) s_h[o] = h;
   }
   __syncthreads();
   if (tid < kNos * kNC) {
      const int cell = tid / kNC;
      const int d = tid % kNC;
      double v = 0.0;
#pragma unroll
      for (int tp = 0; tp < kTaps; tp++) v = fma(s_h[(cell - kM + tp) & (kNos - 1)], ct[tp], v);
      H[((size_t)comp * kNos + cell) * kNC + d] = v;
      if (hb) s_scr[tid] = ldexp(fabs(v), 31 * d);
   }
   if (hb) {
      __syncthreads();
      if (tid < kNos) {  // one wave: a cell per lane, summed in degree order, then the max over the cells
         double m = 0.0;
#pragma unroll
         for (int d = 0; d < kNC; d++) m += s_scr[tid * kNC + d];
         for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off, 64));
         if (tid == 0) hb[comp] = m;
      }
   }
   __syncthreads();
}

// part: [nw][nparts][64] (from_sum = 0) or the summed grids [nw][64] (from_sum = 1)
// blockIdx.y: right-hand side (two-vector matvec): part and H advance by part_rs / h_rs elements per vector
// hb (det, may be NULL): the bounds of H at hb[comp] and of Hd at hb[nw + comp], per vector at hb + 2 nw y
__global__ __launch_bounds__(kGridThreads) void k_grid(const double* __restrict__ part, int nparts,
                                                      const double* __restrict__ w, const double* __restrict__ wd,
                                                      double* __restrict__ H, double* __restrict__ Hd, int grad,
                                                      int from_sum, long long part_rs = 0, long long h_rs = 0,
                                                      double* __restrict__ hb = nullptr, int clear_sum = 0)
{
   __shared__ double s_red[kGridThreads];
   __shared__ double s_g[kNos];
   __shared__ double s_h[kNos];
   __shared__ double s_w[kNos];
   const int comp = blockIdx.x;
   part += blockIdx.y * part_rs;
   H += blockIdx.y * h_rs;
   const int tid = threadIdx.x;
   const double wv = tid < kNos ? w[(size_t)comp * kNos + tid] : 0.0;
   const double wdv = (grad && tid < kNos) ? wd[(size_t)comp * kNos + tid] : 0.0;
   double ct[kTaps];
   grid_tail_coeffs(ct);
   if (from_sum) {
      if (tid < kNos) {
         s_g[tid] = part[(size_t)comp * kNos + tid];
         // launch_spread_grid's atomic sums start from zero at the next matvec
         if (clear_sum) const_cast<double*>(part)[(size_t)comp * kNos + tid] = 0.0;
      }
   } else {
      // 16 strands per cell over this window's contiguous partial grids; each strand issues up to
      // kPer loads before its first add (one memory latency for nparts <= 256); fixed order ->
      // deterministic
      constexpr int kPer = 16;
      const int cell = tid & 63;
      const int strand = tid >> 6;
      constexpr int nstr = kGridThreads / 64;
      const double* src = part + (size_t)comp * nparts * kNos + cell;
      double acc = 0.0;
      for (int p0 = strand; p0 < nparts; p0 += kPer * nstr) {
         double v[kPer];
#pragma unroll
         for (int k = 0; k < kPer; k++) {
            const int p = p0 + k * nstr;
            v[k] = p < nparts ? src[(size_t)p * kNos] : 0.0;
         }
#pragma unroll
         for (int k = 0; k < kPer; k++) acc += v[k];
      }
      s_red[tid] = acc;
      __syncthreads();
      if (tid < kNos) {
         double v = 0.0;
         for (int k = 0; k < nstr; k++) v += s_red[k * 64 + tid];
         s_g[tid] = v;
      }
   }
   __syncthreads();
   if (hb) hb += 2 * (size_t)gridDim.x * blockIdx.y;
   grid_tail(comp, s_g, wv, ct, H, s_w, s_h, hb, s_red);
   if (grad) grid_tail(comp, s_g, wdv, ct, Hd, s_w, s_h, hb ? hb + gridDim.x : nullptr, s_red);
}

// Row shards with few blocks, split interpolation (launch_shard_finish_split): the grid kernel from the summed
// grids also initialises y = beta y + alpha f^2 mu diag x (a grid-stride loop over all its threads), and the
// interpolation runs S workgroups per block, each over a contiguous range of window groups, adding alpha f^2
// times its LDS y-slice into y with global atomics.  A shard of config C on 8 GPUs has 62 blocks: the
// one-workgroup-per-block interpolation runs on 62 of the 256 CUs.
// ---- the peer exchange (PeerArgs, dist.hip) ----
// A rank's buffer holds two slots (the epoch's parity) of nw x 64 entries; an entry is two 64-bit words, the
// low and the high half of the double's bits, each with the epoch in its upper 32 bits.  A 64-bit store is
// single-copy atomic, so a reader that sees the epoch in both words has the value -- one round trip, no
// separate flag and no fence (a release here would write back the whole L2, an acquire invalidate it: 9 us
// per matvec at N = 8 in the first version).  Every word is stored and loaded at system scope (written
// through to memory, never served stale from a cache).  A rank two epochs ahead would need this rank's
// entries of the epoch in between, so a slot is never rewritten while a reader still needs it.
constexpr int kPeerLanes = kGridThreads / 64;  // ranks gathered per pass (a wave per rank, a lane per cell)

__device__ __forceinline__ unsigned long long* peer_slot(char* buf, const PeerArgs& A)
{
   return (unsigned long long*)(buf + (A.epoch & 1u) * A.slot_doubles * 16);
}

// rank r's buffer: the first kPeerInline from the kernel arguments (no dependent global load), then the table
__device__ __forceinline__ char* peer_buf(const PeerArgs& A, int r)
{
   char* b = A.inl[0];
#pragma unroll
   for (int k = 1; k < kPeerInline; k++)
      if (r == k) b = A.inl[k];
   return r < kPeerInline ? b : A.bufs[r];
}

// this rank's value of (window comp, cell) into its slot of the epoch
__device__ __forceinline__ void peer_put(const PeerArgs& A, int comp, int cell, double v)
{
   unsigned long long* p = peer_slot(A.own, A) + 2 * ((size_t)comp * kNos + cell);
   const unsigned long long bits = (unsigned long long)__double_as_longlong(v);
   const unsigned long long e = (unsigned long long)A.epoch << 32;
   __hip_atomic_store(p, (bits & 0xffffffffull) | e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
   __hip_atomic_store(p + 1, (bits >> 32) | e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// s_g[cell] = sum over ranks r = 0, 1, ... (in that order) of rank r's value of (comp, cell).  Wave w of the
// workgroup polls rank r0 + w's entries (lane = cell) until both words carry the epoch -- at most A.spin
// polls, then it sets *A.err and gives up (the host fails the next call) -- so up to kPeerLanes ranks' loads
// are in flight at once; the sum runs over LDS in rank order, the first term as is (no 0 + t: -0 stays -0,
// as in a two-rank all-reduce).  Every thread of the workgroup calls it.
__device__ __forceinline__ void peer_gather(const PeerArgs& A, int comp, double* s_g)
{
   __shared__ double s_v[kPeerLanes][kNos];
   const int tid = threadIdx.x, cell = tid & (kNos - 1), lr = tid / kNos;
   double v = 0.0;
   for (int r0 = 0; r0 < A.world; r0 += kPeerLanes) {
      const int r = r0 + lr;
      if (r < A.world) {
         const unsigned long long* p = peer_slot(peer_buf(A, r), A) + 2 * ((size_t)comp * kNos + cell);
         unsigned long long w0, w1;
         for (long long it = 0;; it++) {
            w0 = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            w1 = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((unsigned int)(w0 >> 32) == A.epoch && (unsigned int)(w1 >> 32) == A.epoch) break;
            if (it >= A.spin) {
               __hip_atomic_store(A.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
               break;
            }
            __builtin_amdgcn_s_sleep(2);
         }
         s_v[lr][cell] = __longlong_as_double((long long)((w0 & 0xffffffffull) | (w1 << 32)));
      }
      __syncthreads();
      if (tid < kNos)
         for (int k = 0; k < kPeerLanes && r0 + k < A.world; k++) v = (r0 + k == 0) ? s_v[k][tid] : v + s_v[k][tid];
      __syncthreads();
   }
   if (tid < kNos) s_g[tid] = v;
}

// window comp's sum over the shard's nparts partial grids, for threads tid < 64 (cell tid; every thread of the
// workgroup calls it): k_grid's 16 strands per cell with 16 loads in flight each, then the strands in order
__device__ __forceinline__ double parts_sum(const double* __restrict__ part, int nparts, int comp, double* s_red)
{
   const int tid = threadIdx.x;
   constexpr int kPer = 16;
   const int cell = tid & 63;
   const int strand = tid >> 6;
   constexpr int nstr = kGridThreads / 64;
   const double* src = part + (size_t)comp * nparts * kNos + cell;
   double acc = 0.0;
   for (int p0 = strand; p0 < nparts; p0 += kPer * nstr) {
      double v[kPer];
#pragma unroll
      for (int k = 0; k < kPer; k++) {
         const int p = p0 + k * nstr;
         v[k] = p < nparts ? src[(size_t)p * kNos] : 0.0;
      }
#pragma unroll
      for (int k = 0; k < kPer; k++) acc += v[k];
   }
   s_red[tid] = acc;
   __syncthreads();
   double v = 0.0;
   if (tid < kNos)
      for (int k = 0; k < nstr; k++) v += s_red[k * 64 + tid];
   return v;
}

__global__ __launch_bounds__(kGridThreads) void k_peer_sum(PeerArgs A, double* __restrict__ grid)
{
   __shared__ double s_g[kNos];
   peer_gather(A, blockIdx.x, s_g);
   if (threadIdx.x < kNos) grid[(size_t)blockIdx.x * kNos + threadIdx.x] = s_g[threadIdx.x];
}

// With A (the peer exchange) and part: this rank's window comp summed from its nparts partial grids and put
// into its slot first (k_reduce_parts folded in: the shard's matvec is three launches), then the y
// initialisation, then the gather of every rank's window comp.
__global__ __launch_bounds__(kGridThreads) void k_grid_sum_yinit(const double* __restrict__ gsum,
                                                                const double* __restrict__ w, double* __restrict__ H,
                                                                double* __restrict__ y, const double* __restrict__ x,
                                                                int n, double beta, double amu, PeerArgs A,
                                                                const double* __restrict__ part, int nparts)
{
   __shared__ double s_g[kNos];
   __shared__ double s_h[kNos];
   __shared__ double s_w[kNos];
   const int comp = blockIdx.x;
   const int tid = threadIdx.x;
   const double wv = tid < kNos ? w[(size_t)comp * kNos + tid] : 0.0;
   double ct[kTaps];
   grid_tail_coeffs(ct);
   if (!A.bufs && tid < kNos) s_g[tid] = gsum[(size_t)comp * kNos + tid];
   if (A.bufs && part) {
      __shared__ double s_red[kGridThreads];
      const double v = parts_sum(part, nparts, comp, s_red);
      if (tid < kNos) peer_put(A, comp, tid, v);
   }
   // y init: 4 elements per thread per pass, all loads issued before the first store (one latency per
   // pass instead of one per element)
   constexpr int kU = 4;
   const size_t stride = (size_t)gridDim.x * kGridThreads;
   for (size_t j0 = (size_t)blockIdx.x * kGridThreads + tid; j0 < (size_t)n; j0 += kU * stride) {
      double xv[kU], yv[kU];
#pragma unroll
      for (int u = 0; u < kU; u++) {
         const size_t j = j0 + u * stride;
         xv[u] = j < (size_t)n ? x[j] : 0.0;
         yv[u] = (beta != 0.0 && j < (size_t)n) ? y[j] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < kU; u++) {
         const size_t j = j0 + u * stride;
         if (j < (size_t)n) y[j] = (beta == 0.0 ? 0.0 : beta * yv[u]) + amu * xv[u];
      }
   }
   if (A.bufs) peer_gather(A, comp, s_g);  // after the y initialisation: the peers' spreads overlap it
   __syncthreads();
   grid_tail(comp, s_g, wv, ct, H, s_w, s_h);
}

template <int THREADS, int REC = 5>
__global__ __launch_bounds__(THREADS) void k_interp_part(const uint16_t* __restrict__ meta,
                                                        const uint32_t* __restrict__ lo,
                                                        const uint32_t* __restrict__ qarr,
                                                        const int* __restrict__ tile_off, const double* __restrict__ H,
                                                        double* __restrict__ y, int n, int B, int ngroups, int S,
                                                        double scale)
{
   extern __shared__ __attribute__((aligned(16))) double smem[];
   double* s_y = smem;
   const int b = blockIdx.x / S, part = blockIdx.x % S;
   const int g0 = part * ngroups / S, g1 = (part + 1) * ngroups / S;
   const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
   constexpr int nwaves = THREADS / 64;
   const int base = b * B;
   const int nloc = min(B, n - base);
   const int t1 = tile_off[b * ngroups + g1];
   int t = tile_off[b * ngroups + g0] + wave;
   TileRegs cur;
   if (t < t1) load_tile<REC>(cur, meta, lo, qarr, t, lane);
   for (int i = tid; i < B + kPad; i += THREADS) s_y[i] = 0.0;
   __syncthreads();
   for (; t < t1; t += nwaves) {
      const size_t hoff = (size_t)cur.mt * kNC;
      double hc[kNC];
#pragma unroll
      for (int d = 0; d < kNC; d += 2) {
         const double2 v = *reinterpret_cast<const double2*>(H + hoff + d);
         hc[d] = v.x;
         hc[d + 1] = v.y;
      }
#pragma unroll
      for (int r = 0; r < kR; r++) {
         const uint32_t off = slot_off<REC>(cur, r);
         const double u = q_to_s(cur.qq[r]);
         double v = hc[kNC - 1];
#pragma unroll
         for (int d = kNC - 2; d >= 0; d--) v = fma(v, u, hc[d]);
         lds_add(off, v);  // s_y is the first dynamic slice
      }
      const int tn = t + nwaves;
      if (tn < t1) load_tile<REC>(cur, meta, lo, qarr, tn, lane);
   }
   __syncthreads();
   for (int j = tid; j < nloc; j += THREADS) atomicAdd(y + (size_t)base + j, scale * s_y[j]);
}

// gsum[comp][cell] = sum_b part[comp][b][cell]   (row-sharded path: before the all-reduce).  One
// workgroup per window, k_grid's 16 strands per cell with 16 loads in flight each (a thread per cell
// summing the partials one after another took 16 us at an 8-GPU shard of config C)
// A.bufs: the sums go to this rank's slot of A.epoch (peer_put) instead of gsum
__global__ __launch_bounds__(kGridThreads) void k_reduce_parts(const double* __restrict__ part, int nparts, int nw,
                                                              double* __restrict__ gsum, PeerArgs A)
{
   __shared__ double s_red[kGridThreads];
   const int comp = blockIdx.x;
   const int tid = threadIdx.x;
   const double v = parts_sum(part, nparts, comp, s_red);
   if (tid < kNos) {
      if (A.bufs)
         peer_put(A, comp, tid, v);
      else
         gsum[(size_t)comp * kNos + tid] = v;
   }
}

// ------------------------------------------------------------------------------------------------
// interpolation + epilogue
// ------------------------------------------------------------------------------------------------
constexpr int kEpMax = 8;  // epilogue values per thread held in registers (B <= kEpMax * THREADS)

// DOT (non-GRAD only): also forms (y_out, x) -- the (q, p) of a CG step when y = A p -- with a
// deterministic grid-wide sum written to *dot_out by the last block (reduce.hpp)
// DET: the y adds rounded on the grid of det_interp_exp (hb: the bounds of H, and of Hd at hb + nw)
template <bool GRAD, int THREADS, bool DOT = false, bool DET = false, int REC = 5>
__global__ __launch_bounds__(THREADS) void k_interp(
    const uint16_t* __restrict__ meta, const uint32_t* __restrict__ lo, const uint32_t* __restrict__ qarr,
    const int* __restrict__ tile_off, const double* __restrict__ H, const double* __restrict__ Hd,
    const double* __restrict__ x, double* __restrict__ y, int n, int B, int ngroups, double alpha, double beta,
    double f, double mu, double dg, double* __restrict__ dot_part, unsigned int* __restrict__ dot_ticket,
    double* __restrict__ dot_out, const double* __restrict__ hb, int nw)
{
   extern __shared__ __attribute__((aligned(16))) double smem[];
   const int Bp = B + kPad;
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
   if (t < t1) load_tile<REC>(cur, meta, lo, qarr, t, lane);
   // the epilogue's x (mu term) and, when beta != 0, y are fetched now, behind the first run
   const bool ep_regs = B <= kEpMax * THREADS;
   double xe[kEpMax], ye[kEpMax];
   if (ep_regs) {
#pragma unroll
      for (int k = 0; k < kEpMax; k++) {
         const int j = tid + k * THREADS;
         xe[k] = (j < nloc) ? x[(size_t)base + j] : 0.0;
         ye[k] = (!GRAD && beta != 0.0 && j < nloc) ? y[(size_t)base + j] : 0.0;
      }
   }
   for (int i = tid; i < Bp; i += THREADS) {
      s_y[i] = 0.0;
      if (GRAD) s_yd[i] = 0.0;
   }
   double Cy = 0.0, Cyd = 0.0;
   if (DET) {
      Cy = det_grid(det_interp_exp(hb, nw));
      if (GRAD) Cyd = det_grid(det_interp_exp(hb + nw, nw));
   }
   __syncthreads();

   for (; t < t1; t += nwaves) {
      const int tn = t + nwaves;
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
         const uint32_t off = slot_off<REC>(cur, r);
         const double u = q_to_s(cur.qq[r]);
         double v = hc[kNC - 1];
#pragma unroll
         for (int d = kNC - 2; d >= 0; d--) v = fma(v, u, hc[d]);
         lds_add(off, DET ? det_round(v, Cy) : v);  // s_y is the first dynamic slice
         if (GRAD) {
            double vd = hdc[kNC - 1];
#pragma unroll
            for (int d = kNC - 2; d >= 0; d--) vd = fma(vd, u, hdc[d]);
            lds_add(off + 8u * (uint32_t)Bp, DET ? det_round(vd, Cyd) : vd);  // s_yd follows it
         }
      }
      if (tn < t1) load_tile<REC>(cur, meta, lo, qarr, tn, lane);
   }
   __syncthreads();

   const double ff = f * f;
   double dacc = 0.0;
   double* y0 = y;
   double* y1 = y + n;
   double* y2 = y + 2 * (size_t)n;
#pragma unroll
   for (int k = 0; k < kEpMax; k++) {
      // registers path: k-th value of this thread; fallback (B > kEpMax*THREADS): strided loop below
      if (!ep_regs) break;
      const int j = tid + k * THREADS;
      if (j >= nloc) break;
      const size_t gj = (size_t)base + j;
      const double xj = xe[k];
      if (!GRAD) {
         const double v = ff * (s_y[j] + mu * xj);
         const double yo = (beta == 0.0) ? alpha * v : fma(beta, ye[k], alpha * v);
         y[gj] = yo;
         if (DOT) dacc = fma(yo, xj, dacc);
      } else {
         // nfft_interface.c:547-549 summed over windows: (2f)(Kx + mu x), ff*dscale*K'x, ff*x
         const double v0 = 2.0 * f * (s_y[j] + mu * xj);
         const double v1 = ff * s_yd[j];
         const double v2 = dg * ff * xj;  // dg: 0 on component shards without the diagonal
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
   if (!ep_regs) {
      for (int j = tid; j < nloc; j += THREADS) {
         const size_t gj = (size_t)base + j;
         const double xj = x[gj];
         if (!GRAD) {
            const double v = ff * (s_y[j] + mu * xj);
            const double yo = (beta == 0.0) ? alpha * v : fma(beta, y[gj], alpha * v);
            y[gj] = yo;
            if (DOT) dacc = fma(yo, xj, dacc);
         } else {
            const double v0 = 2.0 * f * (s_y[j] + mu * xj);
            const double v1 = ff * s_yd[j];
            const double v2 = dg * ff * xj;  // dg: 0 on component shards without the diagonal
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
   if (DOT && !GRAD) {
      // LDS scratch after the y slices (kRedScratch bytes): the kernel keeps no static LDS (lds_add addresses its
      // first dynamic slice absolutely)
      double* s_scr = smem + (GRAD ? 2 : 1) * Bp;
      dacc = block_sum0_s<THREADS>(dacc, s_scr);
      double tot;
      if (grid_total_s<THREADS>(dacc, dot_part, dot_ticket, &tot, reinterpret_cast<int*>(s_scr + 2 * (THREADS / 64)),
                                s_scr + THREADS / 64) &&
          threadIdx.x == 0)
         *dot_out = tot;
   }
}

// ------------------------------------------------------------------------------------------------
// the plain interpolation with the window group's H rows staged in LDS
// ------------------------------------------------------------------------------------------------
// k_interp gathers each run's 8 coefficients H[comp][cell][0..7] from global memory: 64 B per run from a table of
// nw x 4 KB that L1 cannot hold beside the layout stream, so at config E the gather costs ~20 % of the kernel (a
// probe that read one window's 4 KB for every run ran 671 -> 535 us).  Here a workgroup walks its block's tiles
// group by group (tile_off orders them so) and reads the coefficients from LDS: two slots of CG windows x 64 cells x
// 8 degrees ([window][degree][cell], windows kHlWin = 513 doubles apart so two windows' even cells fall on
// different banks).  Groups 0 and 1 are staged by the whole workgroup before the loop; afterwards the LAST wave to
// leave group g (an LDS counter per group) stages group g + 2 into g's slot and publishes it (ready[slot] = g + 2,
// release), and a wave entering group g >= 2 waits for that (acquire, s_sleep, bounded).  A wave waits only for a
// group every wave has left two groups before, and the stager stages before it waits for anything, so the waves
// never wait on one another in a cycle.  Same arithmetic as k_interp's plain path (bitwise equal results).
constexpr int kHlWin = kNC * kNos + 1;

__host__ __device__ constexpr size_t hl_lds_bytes(int B, int CG, int ngroups, int ns)
{
   return sizeof(double) * ((size_t)B + kPad) + sizeof(double) * (size_t)ns * CG * kHlWin +
          sizeof(int) * (1 + (size_t)ns + 2 * (size_t)ngroups);
}

// one wave stages group g's H rows (windows [g CG, min((g + 1) CG, nw))) into slot `slot` of s_H
__device__ __forceinline__ void hl_stage_wave(double* s_H, const double* __restrict__ H, int g, int slot, int CG, int nw,
                                              int lane)
{
   const int c0 = g * CG;
   const int ncomp = min(CG, nw - c0);
   const double2* src = reinterpret_cast<const double2*>(H + (size_t)c0 * kNos * kNC);
   double* dst = s_H + (size_t)slot * CG * kHlWin;
   const int pairs = ncomp * kNos * kNC / 2;
#pragma unroll 4
   for (int i = lane; i < pairs; i += 64) {
      const double2 v = src[i];
      const int e = 2 * i;                       // element of [cl][cell][d]
      const int cl = e / (kNos * kNC);
      const int cell = (e / kNC) & (kNos - 1);
      const int d = e & (kNC - 1);
      double* row = dst + cl * kHlWin + cell;
      row[d * kNos] = v.x;
      row[(d + 1) * kNos] = v.y;
   }
}

template <int THREADS, bool DET = false, int REC = 5>
__global__ __launch_bounds__(THREADS) void k_interp_hl(const uint16_t* __restrict__ meta, const uint32_t* __restrict__ lo,
                                                       const uint32_t* __restrict__ qarr, const int* __restrict__ tile_off,
                                                       const double* __restrict__ H, const double* __restrict__ x,
                                                       double* __restrict__ y, int n, int B, int ngroups, int CG, int nw,
                                                       double alpha, double beta, double f, double mu,
                                                       const double* __restrict__ hb, int ns)
{
   extern __shared__ __attribute__((aligned(16))) double smem[];
   const int Bp = B + kPad;
   double* s_y = smem;  // the first dynamic slice (lds_add addresses it absolutely)
   double* s_H = smem + Bp;  // ns slots (2 <= ns <= nwaves): group g in slot g % ns
   int* s_ready = reinterpret_cast<int*>(s_H + (size_t)ns * CG * kHlWin);
   int* s_done = s_ready + ns;
   int* s_toff = s_done + ngroups;  // the block's group boundaries tile_off[b ngroups .. (b + 1) ngroups]
   const int b = blockIdx.x;
   const int tid = threadIdx.x;
   const int base = b * B;
   const int nloc = min(B, n - base);
   const int lane = tid & 63;
   const int wave = tid >> 6;
   constexpr int nwaves = THREADS / 64;
   const int gbase = b * ngroups;
   const int t0 = tile_off[gbase];
   const int t1 = tile_off[gbase + ngroups];
   TileRegs cur;
   int t = t0 + wave;
   if (t < t1) load_tile<REC>(cur, meta, lo, qarr, t, lane);
   const bool ep_regs = B <= kEpMax * THREADS;
   double xe[kEpMax], ye[kEpMax];
   if (ep_regs) {
#pragma unroll
      for (int k = 0; k < kEpMax; k++) {
         const int j = tid + k * THREADS;
         xe[k] = (j < nloc) ? x[(size_t)base + j] : 0.0;
         ye[k] = (beta != 0.0 && j < nloc) ? y[(size_t)base + j] : 0.0;
      }
   }
   for (int i = tid; i < Bp; i += THREADS) s_y[i] = 0.0;
   for (int i = tid; i < ngroups; i += THREADS) s_done[i] = 0;
   for (int i = tid; i <= ngroups; i += THREADS) s_toff[i] = tile_off[gbase + i];
   if (tid < ns) s_ready[tid] = tid;
   // groups 0 .. ns - 1, one wave each
   if (wave < ns && wave < ngroups) hl_stage_wave(s_H, H, wave, wave, CG, nw, lane);
   const double Cy = DET ? det_grid(det_interp_exp(hb, nw)) : 0.0;
   __syncthreads();

   int g = 0, gslot = 0;
   int gend = s_toff[1];
   // wave leaves group gl: count it; the last one stages group gl + ns into gl's slot and publishes it
   auto leave = [&](int gl) {
      int old = 0;
      if (lane == 0) old = __hip_atomic_fetch_add(s_done + gl, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
      old = __builtin_amdgcn_readfirstlane(old);
      if (old == nwaves - 1 && gl + ns < ngroups) {
         const int sl = gl % ns;
         hl_stage_wave(s_H, H, gl + ns, sl, CG, nw, lane);
         __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
         if (lane == 0) __hip_atomic_store(s_ready + sl, gl + ns, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
   };
   for (; t < t1; t += nwaves) {
      while (t >= gend) {
         leave(g);
         g++;
         gend = s_toff[g + 1];
         gslot = g % ns;
         if (g >= ns) {
            for (long spin = 0; spin < (1l << 24); spin++) {
               if (__hip_atomic_load(s_ready + gslot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == g) break;
               __builtin_amdgcn_s_sleep(1);
            }
         }
      }
      const int cl = (int)(cur.mt >> 6) - g * CG;
      const int cell = (int)(cur.mt & 63u);
      const double* hrow = s_H + ((size_t)gslot * CG + cl) * kHlWin + cell;
      double hc[kNC];
#pragma unroll
      for (int d = 0; d < kNC; d++) hc[d] = hrow[d * kNos];
#pragma unroll
      for (int r = 0; r < kR; r++) {
         const uint32_t off = slot_off<REC>(cur, r);
         const double u = q_to_s(cur.qq[r]);
         double v = hc[kNC - 1];
#pragma unroll
         for (int d = kNC - 2; d >= 0; d--) v = fma(v, u, hc[d]);
         lds_add(off, DET ? det_round(v, Cy) : v);
      }
      if (t + nwaves < t1) load_tile<REC>(cur, meta, lo, qarr, t + nwaves, lane);
   }
   for (; g < ngroups; g++) leave(g);  // the groups this wave has no (more) tiles in
   __syncthreads();

   const double ff = f * f;
#pragma unroll
   for (int k = 0; k < kEpMax; k++) {
      if (!ep_regs) break;
      const int j = tid + k * THREADS;
      if (j >= nloc) break;
      const double v = ff * (s_y[j] + mu * xe[k]);
      y[(size_t)base + j] = (beta == 0.0) ? alpha * v : fma(beta, ye[k], alpha * v);
   }
   if (!ep_regs) {
      for (int j = tid; j < nloc; j += THREADS) {
         const size_t gj = (size_t)base + j;
         const double v = ff * (s_y[j] + mu * x[gj]);
         y[gj] = (beta == 0.0) ? alpha * v : fma(beta, y[gj], alpha * v);
      }
   }
}

// ------------------------------------------------------------------------------------------------
// two right-hand sides per pass over the layout (SLQ probes in lockstep, krylov.hip)
// ------------------------------------------------------------------------------------------------
// The interpolation reads the layout (5 B per (point, window)) once for both vectors and shares the
// per-point decode; each vector keeps its own H and LDS y-slice (planar, so the layout's bank balancing
// for ds_add_f64 holds).  The spread stays one launch per vector: a two-vector spread needs 98 KB of LDS
// per workgroup at B = 4064 (two alpha slices and 21-double moment rows), one workgroup per CU, and
// measured slower than two single-vector spreads; the two-vector interpolation measured
// 51 us against 2 x 34 us.

// y_v = beta y_v + alpha f^2 (sum_windows interp_v + mu x_v), v = 0, 1; H of vector v at H + v * h_rs
// DET: as k_interp's, each vector on the grid of its own bounds (hb, hb + 2 nw: k_grid's per-vector layout), so
// each column equals the single-vector matvec bit for bit
template <int THREADS, bool DET = false, int REC = 5>
__global__ __launch_bounds__(THREADS) void k_interp2(const uint16_t* __restrict__ meta,
                                                     const uint32_t* __restrict__ lo,
                                                     const uint32_t* __restrict__ qarr,
                                                     const int* __restrict__ tile_off, const double* __restrict__ H,
                                                     size_t h_rs, const double* __restrict__ x0,
                                                     const double* __restrict__ x1, double* __restrict__ y0,
                                                     double* __restrict__ y1, int n, int B, int ngroups, double alpha,
                                                     double beta, double f, double mu, const double* __restrict__ hb,
                                                     int nw)
{
   extern __shared__ __attribute__((aligned(16))) double smem[];
   const int Bp = B + kPad;
   double* s_y0 = smem;
   double* s_y1 = smem + Bp;
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
   if (t < t1) load_tile<REC>(cur, meta, lo, qarr, t, lane);
   for (int i = tid; i < Bp; i += THREADS) s_y0[i] = s_y1[i] = 0.0;
   double C0 = 0.0, C1 = 0.0;
   if (DET) {
      C0 = det_grid(det_interp_exp(hb, nw));
      C1 = det_grid(det_interp_exp(hb + 2 * nw, nw));
   }
   __syncthreads();
   const double* H1 = H + h_rs;
   for (; t < t1; t += nwaves) {
      const size_t hoff = (size_t)cur.mt * kNC;
      double h0[kNC], h1[kNC];
#pragma unroll
      for (int d = 0; d < kNC; d += 2) {
         const double2 v0 = *reinterpret_cast<const double2*>(H + hoff + d);
         const double2 v1 = *reinterpret_cast<const double2*>(H1 + hoff + d);
         h0[d] = v0.x;
         h0[d + 1] = v0.y;
         h1[d] = v1.x;
         h1[d + 1] = v1.y;
      }
#pragma unroll
      for (int r = 0; r < kR; r++) {
         const uint32_t off = slot_off<REC>(cur, r);
         const double u = q_to_s(cur.qq[r]);
         double v0 = h0[kNC - 1], v1 = h1[kNC - 1];
#pragma unroll
         for (int d = kNC - 2; d >= 0; d--) {
            v0 = fma(v0, u, h0[d]);
            v1 = fma(v1, u, h1[d]);
         }
         lds_add(off, DET ? det_round(v0, C0) : v0);                      // s_y0: the first dynamic slice
         lds_add(off + 8u * (uint32_t)Bp, DET ? det_round(v1, C1) : v1);  // s_y1 follows it
      }
      if (t + nwaves < t1) load_tile<REC>(cur, meta, lo, qarr, t + nwaves, lane);
   }
   __syncthreads();
   const double ff = f * f;
   for (int j = tid; j < nloc; j += THREADS) {
      const size_t gj = (size_t)base + j;
      const double v0 = ff * (s_y0[j] + mu * x0[gj]);
      const double v1 = ff * (s_y1[j] + mu * x1[gj]);
      y0[gj] = (beta == 0.0) ? alpha * v0 : fma(beta, y0[gj], alpha * v0);
      y1[gj] = (beta == 0.0) ? alpha * v1 : fma(beta, y1[gj], alpha * v1);
   }
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
// plain launch, or (timing mode) a launch whose start / stop events are the dispatch's own timestamps
template <typename F, typename... A>
static void launch_ev(F fn, dim3 grid, dim3 block, size_t lds, hipStream_t s, const hipEvent_t* ev, A... args)
{
   if (ev)
      hipExtLaunchKernelGGL(fn, grid, block, (std::uint32_t)lds, s, ev[0], ev[1], 0u, args...);
   else
      hipLaunchKernelGGL(fn, grid, block, lds, s, args...);
}

static int spread_momt(const AdditivePlan& P) { return P.spread_variant == 2 ? 0 : 1; }

static size_t spread_lds_bytes(const AdditivePlan& P)
{
   const size_t per = spread_momt(P) ? mom_doubles_per_window<1>() : mom_doubles_per_window<0>();
   return sizeof(double) * ((size_t)P.B + kPad + (size_t)P.CG * per) + (P.det ? 64 : 0);  // DET: a word per wave (kSpreadThreads / 64) and a counter
}

// the fused dot's reduction scratch after the y slices: 2 x (1024 / 64) doubles and an int
constexpr size_t kRedScratch = sizeof(double) * (2 * (1024 / 64) + 1);

static size_t interp_lds_bytes(const AdditivePlan& P, int grad)
{
   return sizeof(double) * ((size_t)P.B + kPad) * (grad ? 2 : 1) + kRedScratch;
}

int upload_tap_coeffs()
{
   // constant memory is per device: upload once per device this process uses
   static bool done[64] = {false};
   int dev = 0;
   NFFT4GP_HIP_CHECK(hipGetDevice(&dev));
   if (dev < 0 || dev >= 64) return -1;
   if (!done[dev]) {
      NFFT4GP_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_taps_u), tap_poly_coeffs().data(), sizeof(double) * kTaps * kNC));
      // C[t][d] 2^-32d: the kernels evaluate the polynomials in s = 2^32 u (q_to_s)
      std::vector<double> C = tap_poly_coeffs();
      for (int t = 0; t < kTaps; t++)
         for (int d = 0; d < kNC; d++) C[t * kNC + d] = std::ldexp(C[t * kNC + d], -32 * d);
      NFFT4GP_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_taps), C.data(), sizeof(double) * kTaps * kNC));
      done[dev] = true;
   }
   return 0;
}

typedef void (*SpreadFn)(const uint16_t*, const uint32_t*, const uint32_t*, const int*, const int*, const double*, int,
                         int, int, int, int, int, double*, double*);
// 0: the spread; 1: the same with per-workgroup s_memrealtime stamps (tools/timeline_spread.py); 2: the round-4
// moment table (MOMT 0, A/B).  Variants that measured slower or neutral (prefetching runs, persistent workgroups,
// several groups per workgroup, the fold in two chains, register-staged alpha, the row shards' block sum in the
// spread's tail) were removed in round 4; DESIGN.md 3.5 keeps their numbers.
constexpr int kSpreadThreads = 512;
// [record 5 / 4][plain / deterministic][variant]
static const SpreadFn kSpreadFns[2][2][4] = {
    {{k_spread<kSpreadThreads>, k_spread<kSpreadThreads, true>, k_spread<kSpreadThreads, false, 0>,
      k_spread<kSpreadThreads, false, 1, false, 5, true>},
     {k_spread<kSpreadThreads, false, 1, true>, k_spread<kSpreadThreads, true, 1, true>,
      k_spread<kSpreadThreads, false, 0, true>, k_spread<kSpreadThreads, false, 1, true, 5, true>}},
    {{k_spread<kSpreadThreads, false, 1, false, 4>, k_spread<kSpreadThreads, true, 1, false, 4>,
      k_spread<kSpreadThreads, false, 0, false, 4>, k_spread<kSpreadThreads, false, 1, false, 4, true>},
     {k_spread<kSpreadThreads, false, 1, true, 4>, k_spread<kSpreadThreads, true, 1, true, 4>,
      k_spread<kSpreadThreads, false, 0, true, 4>, k_spread<kSpreadThreads, false, 1, true, 4, true>}}};
constexpr int kNumSpreadVariants = 4;
// a layout past the 256 MB Infinity Cache streams from HBM: the spread then loads each wave's next tile before the
// current tile's moments (variant 3; E32 606 -> 584 us, E64 739 -> 719), which costs 1.8 % on a cache-resident
// layout (config C, 175 MB), so the choice follows the layout's size (profiles/r06_matvec_variants_ab.txt)
constexpr size_t kInfinityCacheBytes = 256ull << 20;
static SpreadFn spread_fn(const AdditivePlan& P)
{
   int v = P.spread_variant;
   if (v < 0) v = P.dl.bytes > kInfinityCacheBytes ? 3 : 0;
   v = std::min(v, kNumSpreadVariants - 1);
   return kSpreadFns[P.rec == 4 ? 1 : 0][P.det ? 1 : 0][v];
}

constexpr int kInterpThreads = 1024;
typedef void (*InterpFn)(const uint16_t*, const uint32_t*, const uint32_t*, const int*, const double*,
                         const double*, const double*, double*, int, int, int, double, double, double, double,
                         double, double*, unsigned int*, double*, const double*, int);

// the interpolation kernel of a launch: gradient or not, fused (q, p) or not, 512 or 1024 threads, deterministic
template <int T, int REC>
static InterpFn interp_fn_t(bool grad, bool dot, bool det)
{
   if (grad) return det ? k_interp<true, T, false, true, REC> : k_interp<true, T, false, false, REC>;
   if (dot) return det ? k_interp<false, T, true, true, REC> : k_interp<false, T, true, false, REC>;
   return det ? k_interp<false, T, false, true, REC> : k_interp<false, T, false, false, REC>;
}
static InterpFn interp_fn(bool grad, bool dot, bool small, bool det, int rec)
{
   if (rec == 4) return small ? interp_fn_t<512, 4>(grad, dot, det) : interp_fn_t<kInterpThreads, 4>(grad, dot, det);
   return small ? interp_fn_t<512, 5>(grad, dot, det) : interp_fn_t<kInterpThreads, 5>(grad, dot, det);
}
constexpr int kInterp2Threads = 1024;
typedef void (*Interp2Fn)(const uint16_t*, const uint32_t*, const uint32_t*, const int*, const double*, size_t,
                          const double*, const double*, double*, double*, int, int, int, double, double, double, double,
                          const double*, int);
// 512-thread workgroups at >= 512 blocks, as the single-vector interpolation (launch_interp)
template <int REC>
static Interp2Fn interp2_fn_t(bool det, bool small)
{
   if (small) return det ? k_interp2<512, true, REC> : k_interp2<512, false, REC>;
   return det ? k_interp2<kInterp2Threads, true, REC> : k_interp2<kInterp2Threads, false, REC>;
}
static Interp2Fn interp2_fn(bool det, bool small, int rec)
{
   return rec == 4 ? interp2_fn_t<4>(det, small) : interp2_fn_t<5>(det, small);
}
typedef void (*InterpPartFn)(const uint16_t*, const uint32_t*, const uint32_t*, const int*, const double*, double*, int,
                             int, int, int, double);
static InterpPartFn interp_part_fn(int rec) { return rec == 4 ? k_interp_part<512, 4> : k_interp_part<512, 5>; }

// a kernel whose dynamic slice is addressed absolutely (lds_at) must have no static LDS
static bool static_lds_zero(const void* fn)
{
   hipFuncAttributes a;
   if (hipFuncGetAttributes(&a, fn) != hipSuccess) return false;
   return a.sharedSizeBytes == 0;
}

// every interpolation kernel the launchers pick
typedef void (*InterpHlFn)(const uint16_t*, const uint32_t*, const uint32_t*, const int*, const double*, const double*,
                           double*, int, int, int, int, int, double, double, double, double, const double*, int);
static InterpHlFn interp_hl_fn(bool small, bool det, int rec)
{
   if (rec == 4)
      return small ? (det ? k_interp_hl<512, true, 4> : k_interp_hl<512, false, 4>)
                   : (det ? k_interp_hl<1024, true, 4> : k_interp_hl<1024, false, 4>);
   return small ? (det ? k_interp_hl<512, true, 5> : k_interp_hl<512, false, 5>)
                : (det ? k_interp_hl<1024, true, 5> : k_interp_hl<1024, false, 5>);
}
// k_interp_hl for layouts past the Infinity Cache (config E: 785 -> 717 us fp64, 671 -> 652 us in the 32-bit mode);
// on a cache-resident layout (config C) its one-wave stagings stall the waves, which there run about one tile per
// group (31 -> 42 us), so k_interp stays.  NFFT4GP_AMD_INTERP_HL=0 / 1 forces either
// (profiles/r06_matvec_variants_ab.txt)
static bool interp_hl_on(const AdditivePlan& P)
{
   static const int v = getenv("NFFT4GP_AMD_INTERP_HL") ? atoi(getenv("NFFT4GP_AMD_INTERP_HL")) : -1;
   return v < 0 ? P.dl.bytes > kInfinityCacheBytes : v != 0;
}

static std::vector<const void*> interp_kernels()
{
   std::vector<const void*> v;
   for (int sm = 0; sm < 2; sm++)
      for (int det = 0; det < 2; det++)
         for (int rec = 4; rec <= 5; rec++) v.push_back((const void*)interp_hl_fn(sm, det, rec));
   for (int g = 0; g < 2; g++)
      for (int d = 0; d < 2; d++)
         for (int sm = 0; sm < 2; sm++)
            for (int det = 0; det < 2; det++)
               for (int rec = 4; rec <= 5; rec++) v.push_back((const void*)interp_fn(g, d && !g, sm, det, rec));
   for (int det = 0; det < 2; det++)
      for (int sm = 0; sm < 2; sm++)
         for (int rec = 4; rec <= 5; rec++) v.push_back((const void*)interp2_fn(det, sm, rec));
   for (int rec = 4; rec <= 5; rec++) v.push_back((const void*)interp_part_fn(rec));
   return v;
}

static void raise_lds_limit_once()
{
   // a function-local static initialiser runs once (thread-safe)
   static const bool raised = []() {
      for (const auto& byrec : kSpreadFns)
         for (const auto& bydet : byrec)
            for (const SpreadFn f : bydet)
               (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      for (const void* f : interp_kernels())
         (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipGetLastError();
      return true;
   }();
   (void)raised;
}

// every kernel that addresses its dynamic LDS absolutely (lds_at / lds_add) has no static LDS
static bool abs_lds_ok()
{
   static const bool ok = [] {
      std::vector<const void*> v = interp_kernels();
      for (const auto& byrec : kSpreadFns)
         for (const auto& bydet : byrec)
            for (const SpreadFn f : bydet) v.push_back((const void*)f);
      for (const void* f : v)
         if (!static_lds_zero(f)) return false;
      return true;
   }();
   if (!ok) fprintf(stderr, "nfft4gp_amd: a matvec kernel has static LDS; its absolute LDS addressing would be wrong\n");
   return ok;
}

static int launch_spread_to(const AdditivePlan& P, const double* d_x, double* d_part, double* d_gsum,
                            hipStream_t stream)
{
   if (P.dl.ntiles == 0 || P.n == 0) return 0;
   raise_lds_limit_once();
   if (!abs_lds_ok()) return -1;
   const SpreadFn fn = spread_fn(P);
   const int gridx = ((P.nblocks + 7) / 8) * 8 * P.ngroups;
   launch_ev(fn, dim3(gridx), dim3(kSpreadThreads), spread_lds_bytes(P), stream, P.kev ? P.kev + 0 : nullptr,
             P.dl.meta, P.dl.lo, P.dl.q, P.dl.tile_off, (const int*)P.dl.cmax, d_x, P.n, P.B, P.nblocks, P.ngroups,
             P.CG, P.nw, d_part, d_gsum);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int launch_spread(const AdditivePlan& P, const double* d_x, double* d_part, hipStream_t stream)
{
   return launch_spread_to(P, d_x, d_part, nullptr, stream);
}

// The atomic grid sum: each spread workgroup adds its CG x 64 grid values into d_gsum (device-scope fp64 atomics,
// executed at the memory side) instead of writing a partial grid, and k_grid reads the nw x 64 sums (and clears
// them for the next matvec) instead of summing nblocks partial grids per window -- at config C 246 x 64 loads per
// window, most of k_grid's 5 us.  The sums' order then follows the workgroups' arrival, so deterministic mode keeps
// the partials; with many blocks (config E: 2461 adds per address) the adds would contend, so they keep them too.
constexpr int kAtomicGridMaxBlocks = 512;
static bool grid_atomic(const AdditivePlan& P)
{
   static const int v = getenv("NFFT4GP_AMD_GRID_ATOMIC") ? atoi(getenv("NFFT4GP_AMD_GRID_ATOMIC")) : -1;
   if (P.det || v == 0) return false;
   return v > 0 || P.nblocks <= kAtomicGridMaxBlocks;
}

int launch_spread_grid(AdditivePlan& P, const double* d_x, int grad, hipStream_t stream)
{
   if (!grid_atomic(P) || P.nblocks == 0) {
      if (launch_spread(P, d_x, P.d_part, stream)) return -1;
      return launch_grid(P, P.d_part, P.nparts, grad, stream);
   }
   if (!P.d_gsum) {
      NFFT4GP_HIP_CHECK(hipMalloc((void**)&P.d_gsum, sizeof(double) * (size_t)P.nw * kNos));
      NFFT4GP_HIP_CHECK(hipMemsetAsync(P.d_gsum, 0, sizeof(double) * (size_t)P.nw * kNos, stream));
   }
   if (launch_spread_to(P, d_x, nullptr, P.d_gsum, stream)) return -1;
   launch_ev(k_grid, dim3(P.nw), dim3(kGridThreads), 0, stream, P.kev ? P.kev + 2 : nullptr, (const double*)P.d_gsum, 1,
             (const double*)P.d_w, (const double*)P.d_wd, P.d_H, P.d_Hd, grad, 1, 0ll, 0ll, (double*)nullptr, 1);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int launch_grid(const AdditivePlan& P, const double* d_part, int nparts, int grad, hipStream_t stream)
{
   launch_ev(k_grid, dim3(P.nw), dim3(kGridThreads), 0, stream, P.kev ? P.kev + 2 : nullptr, d_part, nparts,
             (const double*)P.d_w, (const double*)P.d_wd, P.d_H, P.d_Hd, grad, 0, 0ll, 0ll,
             P.det ? P.d_hb : (double*)nullptr, 0);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int launch_grid_from_sum(const AdditivePlan& P, const double* d_gridsum, int grad, hipStream_t stream)
{
   launch_ev(k_grid, dim3(P.nw), dim3(kGridThreads), 0, stream, P.kev ? P.kev + 2 : nullptr, d_gridsum, 1,
             (const double*)P.d_w, (const double*)P.d_wd, P.d_H, P.d_Hd, grad, 1, 0ll, 0ll,
             P.det ? P.d_hb : (double*)nullptr, 0);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int launch_shard_finish_split(const AdditivePlan& P, const double* d_gridsum, double alpha, const double* d_x,
                              double beta, double* d_y, int S, hipStream_t stream, const PeerArgs* A,
                              const double* d_part)
{
   constexpr int T = 512;
   raise_lds_limit_once();
   if (!abs_lds_ok()) return -1;
   if (A && A->slot_doubles != (long long)P.nw * kNos) return -1;
   const double ff = P.f * P.f;
   hipLaunchKernelGGL(k_grid_sum_yinit, dim3(P.nw), dim3(kGridThreads), 0, stream, d_gridsum, (const double*)P.d_w,
                      P.d_H, d_y, d_x, P.n, beta, alpha * ff * P.mu * P.diag, A ? *A : PeerArgs{},
                      // a shard without blocks puts zeros (nparts 0: the pointer is not read, but must be non-null)
                      A ? (P.nblocks ? d_part : (const double*)P.d_w) : (const double*)nullptr,
                      P.nblocks ? P.nparts : 0);
   if (P.n > 0)
      hipLaunchKernelGGL(interp_part_fn(P.rec), dim3(P.nblocks * S), dim3(T), sizeof(double) * (size_t)(P.B + kPad), stream,
                         P.dl.meta, P.dl.lo, P.dl.q, P.dl.tile_off, (const double*)P.d_H, d_y, P.n, P.B, P.ngroups, S,
                         alpha * ff);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

// the peer exchange's grid step on its own (one launch: partial-grid sum + put + gather + H), for a
// shard whose interpolation runs unsplit (k_interp's epilogue, no y initialisation here)
int launch_peer_grid(const AdditivePlan& P, const PeerArgs& A, const double* d_part, hipStream_t stream)
{
   if (A.slot_doubles != (long long)P.nw * kNos) return -1;
   hipLaunchKernelGGL(k_grid_sum_yinit, dim3(P.nw), dim3(kGridThreads), 0, stream, (const double*)nullptr,
                      (const double*)P.d_w, P.d_H, (double*)nullptr, (const double*)nullptr, 0, 0.0, 0.0, A,
                      P.nblocks ? d_part : (const double*)P.d_w, P.nblocks ? P.nparts : 0);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int launch_reduce_parts(const AdditivePlan& P, const double* d_part, double* d_gridsum, hipStream_t stream,
                        const PeerArgs* A)
{
   PeerArgs a = A ? *A : PeerArgs{};
   if (A && A->slot_doubles != (long long)P.nw * kNos) return -1;  // with A: this rank's slot (peer_put)
   // no blocks (a shard without rows): nparts = 0 writes zeros (and publishes them)
   hipLaunchKernelGGL(k_reduce_parts, dim3(P.nw), dim3(kGridThreads), 0, stream, d_part, P.nblocks ? P.nparts : 0,
                      P.nw, d_gridsum, a);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int launch_peer_sum(const AdditivePlan& P, const PeerArgs& A, double* d_grid, hipStream_t stream)
{
   if (A.slot_doubles != (long long)P.nw * kNos) return -1;
   hipLaunchKernelGGL(k_peer_sum, dim3(P.nw), dim3(kGridThreads), 0, stream, A, d_grid);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int launch_interp(const AdditivePlan& P, int grad, double alpha, const double* d_x, double beta, double* d_y,
                  hipStream_t stream, double* d_dot)
{
   if (P.n == 0) return 0;
   raise_lds_limit_once();
   if (!abs_lds_ok()) return -1;
   if (d_dot && (grad || P.nblocks > kRedMaxBlocks)) {
      fprintf(stderr, "nfft4gp_amd: fused matvec-dot needs a plain matvec and <= %d blocks\n", kRedMaxBlocks);
      return -1;
   }
   // 512-thread workgroups once there are >= 512 blocks (two workgroups per CU overlap one another's prologue
   // and epilogue: 787 -> 734 us at config E; with fewer blocks half the CU would idle, 30.8 -> 34.3 us at
   // config C; profiles/r04_interp_threads_ab.txt).  NFFT4GP_AMD_INTERP_THREADS=512 / 1024 forces either.
   static const int forced = getenv("NFFT4GP_AMD_INTERP_THREADS") ? atoi(getenv("NFFT4GP_AMD_INTERP_THREADS")) : 0;
   const bool small = forced == 512 || (forced != 1024 && P.nblocks >= 512);
   if (!grad && !d_dot && interp_hl_on(P) && P.ngroups >= 1) {
      // staging slots: 2 on 512-thread workgroups (two per CU fit 2 x 81 KB of LDS), up to 6 on 1024
      static const int slots_env = getenv("NFFT4GP_AMD_HL_SLOTS") ? atoi(getenv("NFFT4GP_AMD_HL_SLOTS")) : 0;
      const int ns = std::max(2, std::min(slots_env > 0 ? slots_env : 2, small ? 2 : 6));
      launch_ev(interp_hl_fn(small, P.det, P.rec), dim3(P.nblocks), dim3(small ? 512 : kInterpThreads),
                hl_lds_bytes(P.B, P.CG, P.ngroups, ns), stream, P.kev ? P.kev + 4 : nullptr, P.dl.meta, P.dl.lo,
                P.dl.q, P.dl.tile_off, (const double*)P.d_H, d_x, d_y, P.n, P.B, P.ngroups, P.CG, P.nw, alpha, beta,
                P.f, P.mu * P.diag, (const double*)P.d_hb, ns);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return 0;
   }
   const InterpFn fn = interp_fn(grad, d_dot != nullptr, small, P.det, P.rec);
   launch_ev(fn, dim3(P.nblocks), dim3(small ? 512 : kInterpThreads), interp_lds_bytes(P, grad), stream,
             P.kev ? P.kev + 4 : nullptr, P.dl.meta, P.dl.lo, P.dl.q, P.dl.tile_off, (const double*)P.d_H,
             (const double*)P.d_Hd, d_x, d_y, P.n, P.B, P.ngroups, alpha, beta, P.f, P.mu * P.diag, P.diag,
             P.d_dot_part, P.d_dot_ticket, d_dot, (const double*)P.d_hb, P.nw);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

// the plain interpolation (no gradient, no fused dot) of blocks [b0, b1) only: the kernel sees a layout
// whose first block is b0 (tile_off, x and y offset by b0 blocks), so each launch writes rows
// [b0 B, min(b1 B, n)) exactly as the whole launch would
int launch_interp_blocks(const AdditivePlan& P, double alpha, const double* d_x, double beta, double* d_y, int b0,
                         int b1, hipStream_t stream)
{
   if (P.n == 0 || b1 <= b0) return 0;
   raise_lds_limit_once();
   if (!abs_lds_ok()) return -1;
   const size_t off = (size_t)b0 * P.B;
   hipLaunchKernelGGL(interp_fn(false, false, false, P.det, P.rec), dim3(b1 - b0), dim3(kInterpThreads),
                      interp_lds_bytes(P, 0), stream, P.dl.meta, P.dl.lo, P.dl.q, P.dl.tile_off + (size_t)b0 * P.ngroups,
                      (const double*)P.d_H, (const double*)P.d_Hd, d_x + off, d_y + off, P.n - (int)off, P.B, P.ngroups,
                      alpha, beta, P.f, P.mu * P.diag, P.diag, (double*)nullptr, (unsigned int*)nullptr,
                      (double*)nullptr, (const double*)P.d_hb, P.nw);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

// y_v = beta y_v + alpha A x_v for two vectors: one spread per vector, both grids in one launch, one two-vector
// interpolation (1-D layouts, whole-row handles).  A two-vector spread (both alpha slices and 21-double moment
// rows in LDS, the layout and u^d shared) measured slower at every shape tried in round 4
int launch_matvec2(AdditivePlan& P, double alpha, const double* x0, const double* x1, double beta, double* y0,
                   double* y1, hipStream_t stream)
{
   if (P.n == 0) return 0;
   if (P.md.on) return -1;
   raise_lds_limit_once();
   if (!abs_lds_ok()) return -1;
   const size_t part_rs = (size_t)std::max(1, P.nparts) * P.nw * kNos;
   const size_t h_rs = (size_t)P.nw * kNos * kNC;
   // both vectors' partial grids in one allocation, so k_grid's per-vector stride stays inside it
   if (!P.d_part2) NFFT4GP_HIP_CHECK(hipMalloc((void**)&P.d_part2, sizeof(double) * 2 * part_rs));
   if (!P.d_H2) NFFT4GP_HIP_CHECK(hipMalloc((void**)&P.d_H2, sizeof(double) * 2 * h_rs));
   if (launch_spread(P, x0, P.d_part2, stream) || launch_spread(P, x1, P.d_part2 + part_rs, stream)) return -1;
   // P.d_hb holds [vector][H, Hd][nw]: the grid writes each vector's H bound at hb + 2 nw y
   hipLaunchKernelGGL(k_grid, dim3(P.nw, 2), dim3(kGridThreads), 0, stream, (const double*)P.d_part2, P.nparts,
                      (const double*)P.d_w, (const double*)P.d_wd, P.d_H2, P.d_Hd, 0, 0, (long long)part_rs,
                      (long long)h_rs, P.det ? P.d_hb : (double*)nullptr, 0);
   const size_t lds_i = sizeof(double) * 2 * ((size_t)P.B + kPad);
   // 1024 threads: 512-thread workgroups at config E's 2461 blocks measured the same loss (1.700 s either way,
   // profiles/r05_interp2_ab.txt); NFFT4GP_AMD_INTERP2_THREADS=512 selects them
   static const int forced = getenv("NFFT4GP_AMD_INTERP2_THREADS") ? atoi(getenv("NFFT4GP_AMD_INTERP2_THREADS")) : 0;
   const bool small = forced == 512;
   hipLaunchKernelGGL(interp2_fn(P.det, small, P.rec), dim3(P.nblocks), dim3(small ? 512 : kInterp2Threads), lds_i, stream,
                      P.dl.meta, P.dl.lo,
                      P.dl.q, P.dl.tile_off, (const double*)P.d_H2, h_rs, x0, x1, y0, y1, P.n, P.B, P.ngroups, alpha,
                      beta, P.f, P.mu * P.diag, (const double*)P.d_hb, P.nw);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

}  // namespace nfft4gp_amd
