// nfft_md.hip -- the additive operator for windows of 2 to 5 features (TEST1's bike / poletele windows of 2 and
// 3, BASELINE config A), and any handle mixing them with 1-D windows.
//
// Same algorithm as the 1-D path (NFFT3 fastsum with N = 32, n_os = 64, m = 4, nfft_interface.c:216-256,
// :426, :533-534; see window.cpp), on 64^d grids:
//   spread    g = B^T x         each point adds x_j * prod_t PHI taps to 10^d cells (PRE_PSI taps from the
//                               first setup, fp64 atomics into the component's grid, which stays in L2)
//   forward   a = (E x ... x E) g   E = [e^{+2 pi i (k-16) l / 64} / PHI_HUT(k-16)]  (32 x 64), one axis
//                                   per launch, then a *= weight * bhat_k * prod_t 1/PHI_HUT(k_t - 16)
//   backward  h = Re (E^* x ... x E^*) a   (the reference keeps Re f, nfft_interface.c:436)
//   interp    (K x)_j = sum over the point's 10^d cells of h * taps, one wave per point, all components
//             of the point in the same wave (the per-point sum over windows is in a fixed order)
// and the 1-D path's epilogue (y = beta y + alpha f^2 (sum + mu x), or the three gradient outputs of
// nfft_interface.c:547-549).  The grid work per component is 3 x 32 x 64^2 x 64 complex MACs in 3-D
// (tiny); the spread/interp are 1000 taps per point and component.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "internal.h"
#include "reduce.hpp"

namespace nfft4gp_amd {

namespace {

__constant__ double2 c_tw[kNos];       // e^{+2 pi i m / 64}
__constant__ double c_phinv[kBand];    // 1 / PHI_HUT(k - 16)

constexpr int kMdThreads = 256;
constexpr int kMdInterpBlocks = 2048;  // grid-stride interp (grid_total handles <= kRedMaxBlocks)

__device__ __forceinline__ int ipow_i(int b, int e)
{
   int r = 1;
   for (int i = 0; i < e; i++) r *= b;
   return r;
}

// tap row `hi` (digits over axes 1..d-1) of point j: grid row offset and the product of its taps
__device__ __forceinline__ double tap_row(const int* uj, const double* pj, int d, int hi, long long* base)
{
   double w = 1.0;
   long long b = 0, stride = kNos;
   int rem = hi;
   for (int t = 1; t < d; t++) {
      const int lt = rem % kTaps;
      rem /= kTaps;
      b += (long long)((uj[t] + lt) & (kNos - 1)) * stride;
      stride *= kNos;
      w *= pj[t * kTaps + lt];
   }
   *base = b;
   return w;
}

// ---- fixed-point accumulation of the spread -----------------------------------------------------------
// Every tap contribution a = x_j * prod psi is scaled to the integer A = a 2^s_c (rounded at 2^0) and split as
// A = H 2^32 + L with H = floor(A / 2^32) (signed) and L in [0, 2^32); the H's and the L's of a cell are summed
// in two separate 64-bit integer accumulators (LDS ds_add_u64, then global atomic adds, no return values).
// Integer adds are exact, so each cell's pair (sum H, sum L) -- and its value (sum H) 2^32 + sum L -- is the
// same whatever order the atomics run in: the spread, hence the matvec, is bitwise reproducible.
// s_c = 93 - ilogb(B_c) with the bound B_c = n max|x| psi_max^d_c >= every |partial sum| of component c (d_c
// features): B_c < 2^(ilogb(B_c) + 1), so |sum A| < 2^94, |sum H| < 2^62 and sum L < n 2^32 <= 2^63 never
// overflow, and one contribution is rounded at 2^-93 B_c (B_c can exceed a cell's value by ~2^22: still ~2^-71
// of it).  k_md_fix2f forms the doubles.  x with a NaN or an infinity (or B_c >= 1e300, beyond the fixed
// point's range) makes every grid value NaN, so the matvec returns NaN as the fp64 sums would.
__global__ void k_md_absmax(const double* __restrict__ x, int n, unsigned long long* __restrict__ out)
{
   unsigned long long m = 0ull;
   for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x)
      m = max(m, (unsigned long long)__double_as_longlong(fabs(x[j])));  // |x| >= 0 orders like its bits
   for (int off = 32; off > 0; off >>= 1) m = max(m, (unsigned long long)__shfl_xor((long long)m, off, 64));
   if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

// exponent s_c of component c (d_c features): B = n max|x| psi_max^d_c
__device__ __forceinline__ int fix_exp(const unsigned long long* xmax, double n, double psi_max, int dc)
{
   double B = __longlong_as_double((long long)*xmax) * n;
   for (int t = 0; t < dc; t++) B *= psi_max;
   return (B > 0.0 && B < 1e300) ? 93 - ilogb(B) : 0;
}

// B_c out of the fixed point's range: x holds a NaN or an infinity (their bits order above every finite
// |x|), or n max|x| psi_max^d_c >= 1e300
__device__ __forceinline__ bool fix_out_of_range(const unsigned long long* xmax, double n, double psi_max, int dc)
{
   double B = __longlong_as_double((long long)*xmax) * n;
   for (int t = 0; t < dc; t++) B *= psi_max;
   return !(B < 1e300);
}

// a 2^s = H 2^32 + L (truncated below 2^0): t = a 2^(s-32), H = floor(t), L = (t - H) 2^32
__device__ __forceinline__ void to_fix(double a, int s, unsigned long long& L, long long& H)
{
   const double t = ldexp(a, s - 32);
   const double h = floor(t);
   const double f = t - h;  // exact; 1.0 only when t is a tiny negative number (then the value rounds to 0)
   H = (long long)h + (f >= 1.0 ? 1 : 0);
   L = f >= 1.0 ? 0ull : (unsigned long long)(unsigned int)ldexp(f, 32);
}

// acc[0] += L, acc[1] += H (LDS or global; exact integer adds, no carries needed)
__device__ __forceinline__ void fix_add(unsigned long long* acc, unsigned long long L, long long H)
{
   if (L) atomicAdd(acc, L);
   if (H) atomicAdd(acc + 1, (unsigned long long)H);
}

// grid[c][i] = ((sum H) 2^32 + sum L) 2^-s_c; component c = c0 + blockIdx.y; fx: [blockIdx.y][i][sum L, sum H]
// (the launch's components only: all of them, or one at a time for large grids, MdPlan::gfix_per_window)
__global__ void k_md_fix2f(const MdComp* __restrict__ comps, const unsigned long long* __restrict__ fx, long long G,
                           const unsigned long long* __restrict__ xmax, double n, double psi_max,
                           double* __restrict__ grid, int c0)
{
   const int c = c0 + blockIdx.y;
   const int e = fix_exp(xmax, n, psi_max, comps[c].d);
   const bool nan = fix_out_of_range(xmax, n, psi_max, comps[c].d);
   fx += 2 * (long long)blockIdx.y * G;
   grid += (long long)c * G;
   for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < G; i += (long long)gridDim.x * blockDim.x) {
      const double lo = (double)fx[2 * i];
      const double hi = (double)(long long)fx[2 * i + 1];
      grid[i] = nan ? __longlong_as_double(0x7ff8000000000000ll) : ldexp(fma(hi, 4294967296.0, lo), -e);
   }
}

// thread = (point, tap row); the row's 10 cells along axis 0 get fixed-point atomic adds
__global__ __launch_bounds__(kMdThreads) void k_md_spread(const MdComp* __restrict__ comps,
                                                          const int* __restrict__ u, const double* __restrict__ psi,
                                                          const double* __restrict__ x, int n, int hi_max,
                                                          unsigned long long* __restrict__ grid, long long G,
                                                          const unsigned long long* __restrict__ xmax, double psi_max,
                                                          int c0)
{
   const MdComp cp = comps[c0 + blockIdx.y];  // grid: the launch's components (blockIdx.y) only
   const long long idx = (long long)blockIdx.x * kMdThreads + threadIdx.x;
   if (idx >= (long long)n * hi_max) return;
   const int j = (int)(idx / hi_max), hi = (int)(idx % hi_max);
   if (hi >= cp.hicount) return;
   const int* uj = u + cp.u_off + (long long)j * cp.d;
   const double* pj = psi + (cp.u_off + (long long)j * cp.d) * kTaps;
   long long base;
   const double w = x[j] * tap_row(uj, pj, cp.d, hi, &base);
   unsigned long long* g = grid + 2 * ((long long)blockIdx.y * G + base);
   const int ex = fix_exp(xmax, (double)n, psi_max, cp.d);
   const int u0 = uj[0];
#pragma unroll
   for (int lt = 0; lt < kTaps; lt++) {
      unsigned long long lo;
      long long hi;
      to_fix(w * pj[lt], ex, lo, hi);
      fix_add(g + 2 * ((u0 + lt) & (kNos - 1)), lo, hi);
   }
}

// Tiled spread: work item (component, tile, first, end) = the points of one 8^d tile of first-tap cells (a
// chunk of them); their 10^d taps are summed into the tile's (8 + 9)^d footprint in LDS (ds_add_f64), and
// the footprint's non-zero cells are then added to the grid (one global add per cell and item instead of
// one per tap: 1000 per point in 3-D).
// Deterministic: the footprint's lines along axis 0 (one per coordinate of axes 1..d-1: 17^(d-1) of them)
// are dealt to the workgroup's waves (line % 8), and each wave walks every point of the item, 64 at a time
// (lane = point), adding only the tap rows that fall on its own lines -- so every LDS cell is updated by one
// wave, in program order (point chunks, then the point's rows), and the item's sums do not depend on the
// wave schedule.  The items overlap at their halos, so the grid takes their sums in exact fixed point
// (to_fix / fix_add above).
constexpr int kMdTile = 8;
constexpr int kMdFoot = kMdTile + kTaps - 1;  // 17
constexpr int kMdSpreadThreads = 512;
__global__ __launch_bounds__(kMdSpreadThreads) void k_md_spread_tiled(const MdComp* __restrict__ comps,
                                                                      const int4* __restrict__ items,
                                                                      const int* __restrict__ perm,
                                                                      const int* __restrict__ u,
                                                                      const double* __restrict__ psi,
                                                                      const double* __restrict__ x, int n,
                                                                      unsigned long long* __restrict__ grid, long long G,
                                                                      const unsigned long long* __restrict__ xmax,
                                                                      double psi_max)
{
   extern __shared__ double s_acc[];  // kMdFoot^d
   constexpr int NW = kMdSpreadThreads / 64;
   const int4 it = items[blockIdx.x];
   const MdComp cp = comps[it.x];
   const int d = cp.d;
   int foot = 1;
   for (int t = 0; t < d; t++) foot *= kMdFoot;
   int lo[kMdTiledMaxDim];
   {
      int rem = it.y;
      for (int t = 0; t < d; t++) {
         lo[t] = (rem % (kNos / kMdTile)) * kMdTile;
         rem /= kNos / kMdTile;
      }
   }
   for (int e = threadIdx.x; e < foot; e += kMdSpreadThreads) s_acc[e] = 0.0;
   __syncthreads();
   const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
   const int* pp = perm + (long long)it.x * n;
   const int npts = it.w - it.z;
   for (int k = lane; k < npts; k += 64) {
      const int j = pp[it.z + k];
      const int* uj = u + cp.u_off + (long long)j * d;
      const double* pj = psi + (cp.u_off + (long long)j * d) * kTaps;
      const double xj = x[j];
      const int x0 = (uj[0] & (kNos - 1)) - lo[0];
      if (d == 1) {
         if (wv == 0) {
#pragma unroll
            for (int lt = 0; lt < kTaps; lt++) atomicAdd(s_acc + x0 + lt, xj * pj[lt]);
         }
         continue;
      }
      const int y0 = (uj[1] & (kNos - 1)) - lo[1];
      const int nz = d == 3 ? kTaps : 1;
      const int z0 = d == 3 ? (uj[2] & (kNos - 1)) - lo[2] : 0;
      for (int lz = 0; lz < nz; lz++) {
         const int z = z0 + lz;
         const double wz = d == 3 ? xj * pj[2 * kTaps + lz] : xj;
         // this wave's lines y + 17 z (line % NW == wv): y = y0 + ly with ly in [0, kTaps)
         int ly = ((wv - kMdFoot * z - y0) % NW + NW) % NW;
         for (; ly < kTaps; ly += NW) {
            const double wt = wz * pj[kTaps + ly];
            double* row = s_acc + ((size_t)(y0 + ly) + (size_t)kMdFoot * z) * kMdFoot + x0;
#pragma unroll
            for (int lt = 0; lt < kTaps; lt++) atomicAdd(row + lt, wt * pj[lt]);
         }
      }
   }
   __syncthreads();
   const int ex = fix_exp(xmax, (double)n, psi_max, d);
   unsigned long long* g = grid + 2 * (long long)it.x * G;
   for (int e = threadIdx.x; e < foot; e += kMdSpreadThreads) {
      const double v = s_acc[e];
      if (v == 0.0) continue;
      long long idx = 0, stride = 1;
      int rem = e;
      for (int t = 0; t < d; t++) {
         idx += (long long)((lo[t] + rem % kMdFoot) & (kNos - 1)) * stride;
         rem /= kMdFoot;
         stride *= kNos;
      }
      unsigned long long L;
      long long H;
      to_fix(v, ex, L, H);
      fix_add(g + 2 * idx, L, H);
   }
}

// Line-owned spread (NFFT4GP_AMD_MD_SPREAD=2, A/B): the tiled spread's work items, but a thread owns one line
// of the tile's footprint along axis 0 (17^(d-1) lines: 289 in 3-D) and keeps its 17 cells in registers; the
// item's points are staged 64 at a time in LDS (x_j folded into the axis-0 taps, padded by 8 zeros on each
// side so a point's taps land on the line's cells by an offset read), and every line walks them in order,
// adding the point's row when it covers the line.  No LDS atomics: each cell is summed by one thread in
// point order.  With fewer than 3 features, `groups` copies of the lines walk interleaved points and are
// added in group order in LDS.  The item's cells go to the grid in exact fixed point (to_fix / fix_add).
constexpr int kMdLinesThreads = 320;  // the 289 lines of a 3-D footprint
constexpr int kMdStage = 64;          // points per staging round
constexpr int kMdPadX = 26;           // 8 zeros, 10 taps, 8 zeros
constexpr size_t kMdLinesStageLds = sizeof(double) * kMdStage * (kMdPadX + 2 * kTaps);
constexpr size_t kMdLinesRedLds = sizeof(double) * kMdLinesThreads * kMdFoot;
__global__ __launch_bounds__(kMdLinesThreads) void k_md_spread_lines(const MdComp* __restrict__ comps,
                                                                     const int4* __restrict__ items,
                                                                     const int* __restrict__ perm,
                                                                     const int* __restrict__ u,
                                                                     const double* __restrict__ psi,
                                                                     const double* __restrict__ x, int n,
                                                                     unsigned long long* __restrict__ grid, long long G,
                                                                     const unsigned long long* __restrict__ xmax,
                                                                     double psi_max)
{
   extern __shared__ double sm[];
   double* s_px = sm;                         // [kMdStage][kMdPadX]
   double* s_py = s_px + kMdStage * kMdPadX;  // [kMdStage][kTaps]
   double* s_pz = s_py + kMdStage * kTaps;    // [kMdStage][kTaps]
   double* s_red = s_pz + kMdStage * kTaps;   // [groups][lines][17] (d < 3 only)
   __shared__ int4 s_o[kMdStage];             // the point's first tap cell relative to the tile, per axis
   const int4 it = items[blockIdx.x];
   const MdComp cp = comps[it.x];
   const int d = cp.d;
   int lines = 1;
   for (int t = 1; t < d; t++) lines *= kMdFoot;
   const int groups = kMdLinesThreads / lines;
   const int tid = threadIdx.x;
   const int grp = tid / lines, line = tid - grp * lines;
   const bool active = grp < groups;
   const int yl = line % kMdFoot, zl = line / kMdFoot;
   int lo[kMdTiledMaxDim];
   {
      int rem = it.y;
      for (int t = 0; t < d; t++) {
         lo[t] = (rem % (kNos / kMdTile)) * kMdTile;
         rem /= kNos / kMdTile;
      }
   }
   double acc[kMdFoot];
#pragma unroll
   for (int c = 0; c < kMdFoot; c++) acc[c] = 0.0;
   const int* pp = perm + (long long)it.x * n;
   for (int c0 = it.z; c0 < it.w; c0 += kMdStage) {
      const int cnt = min(kMdStage, it.w - c0);
      for (int e = tid; e < cnt * 32; e += kMdLinesThreads) {
         const int p = e >> 5, q = e & 31;
         const int j = pp[c0 + p];
         const int* uj = u + cp.u_off + (long long)j * d;
         const double* pj = psi + (cp.u_off + (long long)j * d) * kTaps;
         if (q < kTaps) {
            s_px[p * kMdPadX + 8 + q] = x[j] * pj[q];
         } else if (q < 2 * kTaps) {
            s_py[p * kTaps + q - kTaps] = d > 1 ? pj[q] : (q == kTaps ? 1.0 : 0.0);
         } else if (q < 3 * kTaps) {
            s_pz[p * kTaps + q - 2 * kTaps] = d > 2 ? pj[q] : (q == 2 * kTaps ? 1.0 : 0.0);
         } else if (q == 30) {
            s_o[p] = make_int4((uj[0] & (kNos - 1)) - lo[0], d > 1 ? (uj[1] & (kNos - 1)) - lo[1] : 0,
                               d > 2 ? (uj[2] & (kNos - 1)) - lo[2] : 0, 0);
         } else {
#pragma unroll
            for (int z = 0; z < 8; z++) {
               s_px[p * kMdPadX + z] = 0.0;
               s_px[p * kMdPadX + 18 + z] = 0.0;
            }
         }
      }
      __syncthreads();
      if (active) {
         for (int p = grp; p < cnt; p += groups) {
            const int4 o = s_o[p];
            const int ly = yl - o.y, lz = zl - o.z;
            if ((unsigned)ly < (unsigned)kTaps && (unsigned)lz < (unsigned)kTaps) {
               const double wyz = s_py[p * kTaps + ly] * s_pz[p * kTaps + lz];
               const double* px = s_px + p * kMdPadX + 8 - o.x;  // px[c] = x_j psi_x[c - o.x], zero outside
#pragma unroll
               for (int c = 0; c < kMdFoot; c++) acc[c] = fma(wyz, px[c], acc[c]);
            }
         }
      }
      __syncthreads();  // the stage is rewritten next round
   }
   const int ex = fix_exp(xmax, (double)n, psi_max, d);
   unsigned long long* g = grid + 2 * (long long)it.x * G;
   auto flush = [&](int c, int yy, int zz, double v) {
      if (v == 0.0) return;
      long long idx = (lo[0] + c) & (kNos - 1);
      if (d > 1) idx += (long long)((lo[1] + yy) & (kNos - 1)) * kNos;
      if (d > 2) idx += (long long)((lo[2] + zz) & (kNos - 1)) * kNos * kNos;
      unsigned long long L;
      long long H;
      to_fix(v, ex, L, H);
      fix_add(g + 2 * idx, L, H);
   };
   if (groups == 1) {
      if (active) {
#pragma unroll
         for (int c = 0; c < kMdFoot; c++) flush(c, yl, zl, acc[c]);
      }
   } else {
      if (active) {
#pragma unroll
         for (int c = 0; c < kMdFoot; c++) s_red[(grp * lines + line) * kMdFoot + c] = acc[c];
      }
      __syncthreads();
      for (int e = tid; e < lines * kMdFoot; e += kMdLinesThreads) {
         double v = 0.0;
         for (int gr = 0; gr < groups; gr++) v += s_red[gr * lines * kMdFoot + e];
         const int ln = e / kMdFoot;
         flush(e - ln * kMdFoot, ln % kMdFoot, ln / kMdFoot, v);
      }
   }
}

// Tiled interpolation, the spread's work items: the tile's footprint of h (and h' for the gradient) is
// staged in LDS, each point's 10^d taps are read from there by a group of L lanes (L = 64 / 16 / 1 for
// 3 / 2 / 1 features: the point's tap rows strided over the group, a fixed-order butterfly sum), and the
// component's value of the point goes to part[comp][j]; k_md_combine sums the components in order and
// applies the epilogue.
template <int GRAD>
__global__ __launch_bounds__(kMdSpreadThreads) void k_md_interp_tiled(const MdComp* __restrict__ comps,
                                                                      const int4* __restrict__ items,
                                                                      const int* __restrict__ perm,
                                                                      const int* __restrict__ u,
                                                                      const double* __restrict__ psi,
                                                                      const double* __restrict__ h0,
                                                                      const double* __restrict__ h1, long long G,
                                                                      int n, int nw, double* __restrict__ part)
{
   extern __shared__ double s_h[];  // [GRAD + 1][kMdFoot^d]
   const int4 it = items[blockIdx.x];
   const MdComp cp = comps[it.x];
   const int d = cp.d;
   int foot = 1;
   for (int t = 0; t < d; t++) foot *= kMdFoot;
   int lo[kMdTiledMaxDim];
   {
      int rem = it.y;
      for (int t = 0; t < d; t++) {
         lo[t] = (rem % (kNos / kMdTile)) * kMdTile;
         rem /= kNos / kMdTile;
      }
   }
   const double* g0 = h0 + (long long)it.x * G;
   const double* g1 = h1 + (long long)it.x * G;
   for (int e = threadIdx.x; e < foot; e += kMdSpreadThreads) {
      long long idx = 0, stride = 1;
      int rem = e;
      for (int t = 0; t < d; t++) {
         idx += (long long)((lo[t] + rem % kMdFoot) & (kNos - 1)) * stride;
         rem /= kMdFoot;
         stride *= kNos;
      }
      s_h[e] = g0[idx];
      if (GRAD) s_h[foot + e] = g1[idx];
   }
   __syncthreads();
   const int L = d >= 3 ? 64 : d == 2 ? 16 : 1;  // lanes per point
   const int lane = threadIdx.x & (L - 1);
   const int groups = kMdSpreadThreads / L;
   const int* pp = perm + (long long)it.x * n;
   const int npts = it.w - it.z;
   // every group runs the same number of passes (the butterfly needs whole waves)
   for (int k0 = 0; k0 < npts; k0 += groups) {
      const int k = k0 + (int)threadIdx.x / L;
      const bool ok = k < npts;
      double a0 = 0.0, a1 = 0.0;
      int j = 0;
      if (ok) {
         j = pp[it.z + k];
         const int* uj = u + cp.u_off + (long long)j * d;
         const double* pj = psi + (cp.u_off + (long long)j * d) * kTaps;
         const int o0 = (uj[0] & (kNos - 1)) - lo[0];
         for (int hi = lane; hi < cp.hicount; hi += L) {
            double wt = 1.0;
            int e = o0, stride = kMdFoot, rem = hi;
            for (int t = 1; t < d; t++) {
               const int lt = rem % kTaps;
               rem /= kTaps;
               e += (((uj[t] & (kNos - 1)) - lo[t]) + lt) * stride;
               stride *= kMdFoot;
               wt *= pj[t * kTaps + lt];
            }
            double v0 = 0.0, v1 = 0.0;
#pragma unroll
            for (int lt = 0; lt < kTaps; lt++) {
               v0 = fma(s_h[e + lt], pj[lt], v0);
               if (GRAD) v1 = fma(s_h[foot + e + lt], pj[lt], v1);
            }
            a0 = fma(wt, v0, a0);
            if (GRAD) a1 = fma(wt, v1, a1);
         }
      }
      for (int off = L / 2; off > 0; off >>= 1) {
         a0 += __shfl_xor(a0, off, 64);
         if (GRAD) a1 += __shfl_xor(a1, off, 64);
      }
      if (ok && lane == 0) {
         part[(long long)it.x * n + j] = a0;
         if (GRAD) part[((long long)nw + it.x) * n + j] = a1;
      }
   }
}

// y from the components' values in component order, with the 1-D path's epilogue (k_md_interp's)
template <int GRAD, int DOT>
__global__ __launch_bounds__(kMdThreads) void k_md_combine(int nw, const double* __restrict__ part,
                                                           const double* __restrict__ x, double* __restrict__ y,
                                                           int n, double alpha, double beta, double f, double mu,
                                                           double dg, double* __restrict__ dot_part,
                                                           unsigned int* __restrict__ dot_ticket,
                                                           double* __restrict__ dot_out)
{
   const double ff = f * f;
   double dacc = 0.0;
   for (int j = blockIdx.x * kMdThreads + threadIdx.x; j < n; j += gridDim.x * kMdThreads) {
      double s0 = 0.0, s1 = 0.0;
      for (int c = 0; c < nw; c++) {
         s0 += part[(long long)c * n + j];
         if (GRAD) s1 += part[((long long)nw + c) * n + j];
      }
      const double xj = x[j];
      if (!GRAD) {
         const double v = ff * (s0 + mu * xj);
         const double yo = (beta == 0.0) ? alpha * v : fma(beta, y[j], alpha * v);
         y[j] = yo;
         if (DOT) dacc = fma(yo, xj, dacc);
      } else {
         const double v0 = 2.0 * f * (s0 + mu * xj), v1 = ff * s1, v2 = dg * ff * xj;
         double* y1 = y + n;
         double* y2 = y + 2 * (size_t)n;
         if (beta == 0.0) {
            y[j] = alpha * v0;
            y1[j] = alpha * v1;
            y2[j] = alpha * v2;
         } else {
            y[j] = fma(beta, y[j], alpha * v0);
            y1[j] = fma(beta, y1[j], alpha * v1);
            y2[j] = fma(beta, y2[j], alpha * v2);
         }
      }
   }
   if (DOT) {
      dacc = block_sum0<kMdThreads>(dacc);
      double tot;
      if (grid_total<kMdThreads>(dacc, dot_part, dot_ticket, &tot) && threadIdx.x == 0) *dot_out = tot;
   }
}

// forward pass along axis t: in [32^t][64][64^(d-t-1)] (real grid when t == 0) -> out [32^t][32][...]
// The twiddle index ((k - 16) l) & 63 differs across a wave's lanes (k, or l in the backward pass): the 64
// twiddles are staged in LDS once per workgroup (bike 0.335 -> 0.310 ms, 5 features 236 -> 229 ms per matvec
// against per-lane loads from the constant table, profiles/r06_md_twiddles_ab.txt; same bits).
__global__ __launch_bounds__(kMdThreads) void k_md_fwd(const MdComp* __restrict__ comps, int t,
                                                       const double* __restrict__ grid, long long G,
                                                       double2* __restrict__ F0, double2* __restrict__ F1,
                                                       long long Cmax)
{
   __shared__ double2 s_tw[kNos];
   const int c = blockIdx.y;
   const int d = comps[c].d;
   if (t >= d) return;  // uniform over the workgroup
   if (threadIdx.x < kNos) s_tw[threadIdx.x] = c_tw[threadIdx.x];
   __syncthreads();
   const double2* tw = s_tw;
   const int lo = ipow_i(kBand, t), hi = ipow_i(kNos, d - t - 1);
   const int e = blockIdx.x * kMdThreads + threadIdx.x;
   if (e >= lo * kBand * hi) return;
   const int lo_i = e % lo, r = e / lo, k = r % kBand, h = r / kBand;
   double2 acc = {0.0, 0.0};
   if (t == 0) {
      const double* in = grid + (long long)c * G;
      for (int l = 0; l < kNos; l++) {
         const double v = in[lo_i + (long long)lo * (l + kNos * h)];
         const double2 w = tw[((k - kBand / 2) * l) & (kNos - 1)];
         acc.x = fma(v, w.x, acc.x);
         acc.y = fma(v, w.y, acc.y);
      }
   } else {
      const double2* in = ((t - 1) & 1 ? F1 : F0) + (long long)c * Cmax;
      for (int l = 0; l < kNos; l++) {
         const double2 v = in[lo_i + (long long)lo * (l + kNos * h)];
         const double2 w = tw[((k - kBand / 2) * l) & (kNos - 1)];
         acc.x = fma(v.x, w.x, fma(-v.y, w.y, acc.x));
         acc.y = fma(v.x, w.y, fma(v.y, w.x, acc.y));
      }
   }
   double2* out = (t & 1 ? F1 : F0) + (long long)c * Cmax;
   const double s = c_phinv[k];
   out[lo_i + (long long)lo * (k + kBand * h)] = make_double2(acc.x * s, acc.y * s);
}

// Passes t >= 1 with one thread per line: the per-output kernels above give each of a line's 32 (forward) or
// 64 (backward) outputs its own thread, lo = 32^t / 64^t threads apart, so every input is fetched 32 / 64 times
// from L2 or HBM (5 features: 34 ms per backward pass, 550 GB of requests; 230 -> 68 ms per matvec).  Here thread (lo_i, h) reads its
// line once -- lanes run along lo_i, so loads and stores are coalesced -- and forms all the line's outputs:
// the forward keeps 32 accumulators, the backward keeps the 32 inputs, in registers.  Every output is the
// same fma chain in the same order as in the per-output kernels, so the bits are the same.
__global__ __launch_bounds__(kMdThreads) void k_md_fwd_lines(const MdComp* __restrict__ comps, int t,
                                                             double2* __restrict__ F0, double2* __restrict__ F1,
                                                             long long Cmax)
{
   __shared__ double2 s_tw[kNos];
   const int c = blockIdx.y;
   const int d = comps[c].d;
   if (t >= d) return;  // uniform over the workgroup
   if (threadIdx.x < kNos) s_tw[threadIdx.x] = c_tw[threadIdx.x];
   __syncthreads();
   const int lo = ipow_i(kBand, t), hi = ipow_i(kNos, d - t - 1);
   const int e = blockIdx.x * kMdThreads + threadIdx.x;
   if (e >= lo * hi) return;
   const int lo_i = e % lo, h = e / lo;
   const double2* in = ((t - 1) & 1 ? F1 : F0) + (long long)c * Cmax + lo_i + (long long)lo * kNos * h;
   double2 acc[kBand];
#pragma unroll
   for (int k = 0; k < kBand; k++) acc[k] = make_double2(0.0, 0.0);
   for (int l = 0; l < kNos; l++) {
      const double2 v = in[(long long)lo * l];
#pragma unroll
      for (int k = 0; k < kBand; k++) {
         const double2 w = s_tw[((k - kBand / 2) * l) & (kNos - 1)];
         acc[k].x = fma(v.x, w.x, fma(-v.y, w.y, acc[k].x));
         acc[k].y = fma(v.x, w.y, fma(v.y, w.x, acc[k].y));
      }
   }
   double2* out = (t & 1 ? F1 : F0) + (long long)c * Cmax + lo_i + (long long)lo * kBand * h;
#pragma unroll
   for (int k = 0; k < kBand; k++) {
      const double sc = c_phinv[k];
      out[(long long)lo * k] = make_double2(acc[k].x * sc, acc[k].y * sc);
   }
}

__global__ __launch_bounds__(kMdThreads) void k_md_bwd_lines(const MdComp* __restrict__ comps, int t,
                                                             double2* __restrict__ B0, double2* __restrict__ B1,
                                                             double2* __restrict__ B2, double2* __restrict__ B3,
                                                             long long Cmax, double* __restrict__ h0,
                                                             double* __restrict__ h1, long long G)
{
   __shared__ double2 s_tw[kNos];
   const int c = blockIdx.y, chain = blockIdx.z;
   const int d = comps[c].d;
   if (t >= d) return;  // uniform over the workgroup
   if (threadIdx.x < kNos) s_tw[threadIdx.x] = c_tw[threadIdx.x];
   __syncthreads();
   const int lo = ipow_i(kNos, t), hi = ipow_i(kBand, d - t - 1);
   const int e = blockIdx.x * kMdThreads + threadIdx.x;
   if (e >= lo * hi) return;
   const int lo_i = e % lo, h = e / lo;
   double2* Ba = chain ? B2 : B0;
   double2* Bb = chain ? B3 : B1;
   const double2* in = ((t - 1) & 1 ? Bb : Ba) + (long long)c * Cmax + lo_i + (long long)lo * kBand * h;
   double2 v[kBand];
#pragma unroll
   for (int k = 0; k < kBand; k++) v[k] = in[(long long)lo * k];
   const long long o = lo_i + (long long)lo * kNos * h;
#pragma unroll 1
   for (int l = 0; l < kNos; l++) {
      double2 acc = {0.0, 0.0};
#pragma unroll
      for (int k = 0; k < kBand; k++) {
         const double2 w = s_tw[((k - kBand / 2) * l) & (kNos - 1)];  // conjugated below
         acc.x = fma(v[k].x, w.x, fma(v[k].y, w.y, acc.x));
         acc.y = fma(v[k].y, w.x, fma(-v[k].x, w.y, acc.y));
      }
      if (t == d - 1)
         (chain ? h1 : h0)[(long long)c * G + o + (long long)lo * l] = acc.x;
      else
         ((t & 1) ? Bb : Ba)[(long long)c * Cmax + o + (long long)lo * l] = acc;
   }
}

// modes: chain 0 = a * bh, chain 1 = a * bhd
__global__ __launch_bounds__(kMdThreads) void k_md_modes(const MdComp* __restrict__ comps,
                                                         const double2* __restrict__ F0,
                                                         const double2* __restrict__ F1, long long Cmax,
                                                         const double* __restrict__ bh,
                                                         const double* __restrict__ bhd, long long M, int grad,
                                                         double2* __restrict__ M0, double2* __restrict__ M1)
{
   const int c = blockIdx.y;
   const int d = comps[c].d;
   const int e = blockIdx.x * kMdThreads + threadIdx.x;
   if (e >= ipow_i(kBand, d)) return;
   const double2 a = (((d - 1) & 1) ? F1 : F0)[(long long)c * Cmax + e];
   const long long o = (long long)c * M + e;
   const double b0 = bh[o];
   M0[o] = make_double2(a.x * b0, a.y * b0);
   if (grad) {
      const double b1 = bhd[o];
      M1[o] = make_double2(a.x * b1, a.y * b1);
   }
}

// backward pass along axis t for chain blockIdx.z: in [64^t][32][32^(d-t-1)] -> out [64^t][64][...];
// the last axis writes the real part only, to the interpolation grid
__global__ __launch_bounds__(kMdThreads) void k_md_bwd(const MdComp* __restrict__ comps, int t,
                                                       const double2* __restrict__ M0,
                                                       const double2* __restrict__ M1, long long M,
                                                       double2* __restrict__ B0, double2* __restrict__ B1,
                                                       double2* __restrict__ B2, double2* __restrict__ B3,
                                                       long long Cmax, double* __restrict__ h0,
                                                       double* __restrict__ h1, long long G)
{
   __shared__ double2 s_tw[kNos];
   const int c = blockIdx.y, chain = blockIdx.z;
   const int d = comps[c].d;
   if (t >= d) return;  // uniform over the workgroup
   if (threadIdx.x < kNos) s_tw[threadIdx.x] = c_tw[threadIdx.x];
   __syncthreads();
   const double2* tw = s_tw;
   const int lo = ipow_i(kNos, t), hi = ipow_i(kBand, d - t - 1);
   const int e = blockIdx.x * kMdThreads + threadIdx.x;
   if (e >= lo * kNos * hi) return;
   const int lo_i = e % lo, r = e / lo, l = r % kNos, h = r / kNos;
   double2* Ba = chain ? B2 : B0;
   double2* Bb = chain ? B3 : B1;
   const double2* in = (t == 0) ? (chain ? M1 : M0) + (long long)c * M : ((t - 1) & 1 ? Bb : Ba) + (long long)c * Cmax;
   double2 acc = {0.0, 0.0};
   for (int k = 0; k < kBand; k++) {
      const double2 v = in[lo_i + (long long)lo * (k + kBand * h)];
      const double2 w = tw[((k - kBand / 2) * l) & (kNos - 1)];  // conjugated below
      acc.x = fma(v.x, w.x, fma(v.y, w.y, acc.x));
      acc.y = fma(v.y, w.x, fma(-v.x, w.y, acc.y));
   }
   const long long o = lo_i + (long long)lo * (l + kNos * h);
   if (t == d - 1)
      (chain ? h1 : h0)[(long long)c * G + o] = acc.x;
   else
      ((t & 1) ? Bb : Ba)[(long long)c * Cmax + o] = acc;
}

// one wave per point (grid-stride), every component of the point in the wave; 1-D path epilogue
template <int GRAD, int DOT>
__global__ __launch_bounds__(kMdThreads) void k_md_interp(const MdComp* __restrict__ comps, int nw,
                                                          const int* __restrict__ u,
                                                          const double* __restrict__ psi,
                                                          const double* __restrict__ h0,
                                                          const double* __restrict__ h1, long long G,
                                                          const double* __restrict__ x, double* __restrict__ y,
                                                          int n, double alpha, double beta, double f, double mu,
                                                          double dg, double* __restrict__ dot_part,
                                                          unsigned int* __restrict__ dot_ticket,
                                                          double* __restrict__ dot_out)
{
   const int lane = threadIdx.x & 63;
   const int waves = gridDim.x * (kMdThreads / 64);
   const double ff = f * f;
   double dacc = 0.0;
   for (int j = blockIdx.x * (kMdThreads / 64) + (threadIdx.x >> 6); j < n; j += waves) {
      double s0 = 0.0, s1 = 0.0;
      for (int c = 0; c < nw; c++) {
         const MdComp cp = comps[c];
         const int* uj = u + cp.u_off + (long long)j * cp.d;
         const double* pj = psi + (cp.u_off + (long long)j * cp.d) * kTaps;
         const int u0 = uj[0];
         double a0 = 0.0, a1 = 0.0;
         for (int hi = lane; hi < cp.hicount; hi += 64) {
            long long base;
            const double w = tap_row(uj, pj, cp.d, hi, &base);
            const double* r0 = h0 + (long long)c * G + base;
            double v0 = 0.0;
#pragma unroll
            for (int lt = 0; lt < kTaps; lt++) v0 = fma(r0[(u0 + lt) & (kNos - 1)], pj[lt], v0);
            a0 = fma(w, v0, a0);
            if (GRAD) {
               const double* r1 = h1 + (long long)c * G + base;
               double v1 = 0.0;
#pragma unroll
               for (int lt = 0; lt < kTaps; lt++) v1 = fma(r1[(u0 + lt) & (kNos - 1)], pj[lt], v1);
               a1 = fma(w, v1, a1);
            }
         }
         for (int off = 32; off > 0; off >>= 1) {
            a0 += __shfl_xor(a0, off, 64);
            if (GRAD) a1 += __shfl_xor(a1, off, 64);
         }
         s0 += a0;
         s1 += a1;
      }
      if (lane == 0) {
         const double xj = x[j];
         if (!GRAD) {
            const double v = ff * (s0 + mu * xj);
            const double yo = (beta == 0.0) ? alpha * v : fma(beta, y[j], alpha * v);
            y[j] = yo;
            if (DOT) dacc = fma(yo, xj, dacc);
         } else {
            // nfft_interface.c:547-549 summed over windows: (2f)(Kx + mu x), ff*dscale*K'x, ff*x
            const double v0 = 2.0 * f * (s0 + mu * xj), v1 = ff * s1, v2 = dg * ff * xj;
            double* y1 = y + n;
            double* y2 = y + 2 * (size_t)n;
            if (beta == 0.0) {
               y[j] = alpha * v0;
               y1[j] = alpha * v1;
               y2[j] = alpha * v2;
            } else {
               y[j] = fma(beta, y[j], alpha * v0);
               y1[j] = fma(beta, y1[j], alpha * v1);
               y2[j] = fma(beta, y2[j], alpha * v2);
            }
         }
      }
   }
   if (DOT) {
      dacc = block_sum0<kMdThreads>(dacc);
      double tot;
      if (grid_total<kMdThreads>(dacc, dot_part, dot_ticket, &tot) && threadIdx.x == 0) *dot_out = tot;
   }
}

template <class T>
int dalloc(T** p, size_t count)
{
   if (*p) {
      (void)hipFree(*p);
      *p = nullptr;
   }
   NFFT4GP_HIP_CHECK(hipMalloc((void**)p, sizeof(T) * std::max<size_t>(1, count)));
   return 0;
}

template <class T>
void dfree_md(T*& p)
{
   if (p) (void)hipFree(p);
   p = nullptr;
}

int upload_md_constants()
{
   double2 tw[kNos];
   for (int m = 0; m < kNos; m++) {
      const double a = 2.0 * 3.141592653589793238462643383279502884 * (double)m / (double)kNos;
      tw[m] = make_double2(std::cos(a), std::sin(a));
   }
   // exact values where the angle is a multiple of pi/4 (cos/sin of those are not exact in libm)
   for (int m = 0; m < kNos; m += kNos / 4) {
      const int q = m / (kNos / 4);
      tw[m] = make_double2(q == 0 ? 1.0 : q == 2 ? -1.0 : 0.0, q == 1 ? 1.0 : q == 3 ? -1.0 : 0.0);
   }
   double ph[kBand];
   for (int k = 0; k < kBand; k++) ph[k] = 1.0 / kb_phi_hut(k - kBand / 2);
   NFFT4GP_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_tw), tw, sizeof(tw)));
   NFFT4GP_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_phinv), ph, sizeof(ph)));
   return 0;
}

}  // namespace

void md_free(AdditivePlan& P)
{
   MdPlan& D = P.md;
   dfree_md(D.d_comps);
   dfree_md(D.d_u);
   dfree_md(D.d_psi);
   dfree_md(D.d_grid);
   D.d_B[0] = D.d_B[1] = nullptr;  // aliases of d_F
   for (auto& p : D.d_F) dfree_md(p);
   for (auto& p : D.d_Mo) dfree_md(p);
   for (auto& p : D.d_B) dfree_md(p);
   for (auto& p : D.d_h) dfree_md(p);
   dfree_md(D.d_bh);
   dfree_md(D.d_bhd);
   dfree_md(D.d_dot_part);
   dfree_md(D.d_dot_ticket);
   dfree_md(D.d_gfix);
   dfree_md(D.d_xmax);
   dfree_md(D.d_perm);
   dfree_md(D.d_items);
   dfree_md(D.d_part);
   D.nitems = 0;
}

// first setup: PRE_PSI taps of the kept rows (nfft_interface.c:150-213 then fastsum's PRE_PSI), buffers
int md_build_points(AdditivePlan& P, const std::vector<std::vector<double>>& xs)
{
   MdPlan& D = P.md;
   md_free(P);
   D.on = true;
   D.maxd = 1;
   for (int c = 0; c < P.nw; c++) {
      if (P.comp_dims[c] < 1 || P.comp_dims[c] > kMdMaxDim) {
         fprintf(stderr, "nfft4gp_amd: window %d has %d features; windows of 1 to %d features are supported.\n", c,
                 P.comp_dims[c], kMdMaxDim);
         return -1;
      }
      D.maxd = std::max(D.maxd, P.comp_dims[c]);
   }
   D.G = 1;
   D.M = 1;
   for (int t = 0; t < D.maxd; t++) {
      D.G *= kNos;
      D.M *= kBand;
   }
   D.Cmax = D.G / 2;  // 32 * 64^(maxd-1)
   D.comps.assign(P.nw, MdComp());
   long long off = 0;
   for (int c = 0; c < P.nw; c++) {
      MdComp& cp = D.comps[c];
      cp.d = P.comp_dims[c];
      cp.hicount = 1;
      for (int t = 1; t < cp.d; t++) cp.hicount *= kTaps;
      cp.u_off = off;
      off += (long long)P.n * cp.d;
   }
   const int n = P.n, ng = P.n_global;
   // PRE_PSI taps of every (component, point, axis), filled by up to 16 host threads over point ranges
   std::vector<int> u((size_t)off);
   std::vector<double> psi((size_t)off * kTaps);
   auto fill = [&](int c, int j0, int j1) {
      const int d = P.comp_dims[c];
      for (int j = j0; j < j1; j++)
         for (int t = 0; t < d; t++) {
            const double xj = xs[c][(size_t)t * ng + P.row_begin + j];
            const int uj = (int)std::floor(xj * (double)kNos) - kM;
            const size_t e = (size_t)D.comps[c].u_off + (size_t)j * d + t;
            u[e] = uj;
            for (int lt = 0; lt < kTaps; lt++) {
               const double tx = xj - (double)(uj + lt) / (double)kNos;
               psi[e * kTaps + lt] = kb_phi(tx * (double)kNos);
            }
         }
   };
   const int nth = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
   const int per = std::max(4096, (n + nth - 1) / nth);
   {
      std::vector<std::thread> th;
      std::vector<std::pair<int, int>> work;
      for (int c = 0; c < P.nw; c++)
         for (int j0 = 0; j0 < n; j0 += per) work.push_back({c, j0});
      std::atomic<size_t> next{0};
      for (int t = 0; t < nth; t++)
         th.emplace_back([&]() {
            for (size_t w; (w = next.fetch_add(1)) < work.size();)
               fill(work[w].first, work[w].second, std::min(n, work[w].second + per));
         });
      for (auto& t : th) t.join();
   }
   const size_t nw = (size_t)P.nw;
   if (dalloc(&D.d_comps, nw) || dalloc(&D.d_u, u.size()) || dalloc(&D.d_psi, psi.size()) ||
       dalloc(&D.d_grid, nw * D.G) || dalloc(&D.d_F[0], nw * D.Cmax) || dalloc(&D.d_F[1], nw * D.Cmax) ||
       dalloc(&D.d_Mo[0], nw * D.M) || dalloc(&D.d_Mo[1], nw * D.M) || dalloc(&D.d_B[2], nw * D.Cmax) ||
       dalloc(&D.d_B[3], nw * D.Cmax) ||
       dalloc(&D.d_h[0], nw * D.G) || dalloc(&D.d_h[1], nw * D.G) || dalloc(&D.d_bh, nw * D.M) ||
       dalloc(&D.d_bhd, nw * D.M) || dalloc(&D.d_dot_part, (size_t)kMdInterpBlocks) ||
       dalloc(&D.d_dot_ticket, (size_t)kTicketWords) || dalloc(&D.d_xmax, 1))
      return -1;
   // the backward passes of chain 0 run in the forward passes' buffers: k_md_modes has read them by then
   D.d_B[0] = D.d_F[0];
   D.d_B[1] = D.d_F[1];
   // the spread's fixed-point grids (16 B per cell): every window's at once, or -- windows beyond the tiled
   // kernels (4 features: 64^4 cells) whose set would pass 256 MB -- one window's, reused window by window
   D.gfix_per_window = D.maxd > kMdTiledMaxDim && nw > 1 && 16.0 * (double)nw * (double)D.G > 256.0 * (1 << 20);
   if (dalloc(&D.d_gfix, 2 * (D.gfix_per_window ? 1 : nw) * D.G)) return -1;
   D.psi_max = 0.0;
   for (double v : psi) D.psi_max = std::max(D.psi_max, std::fabs(v));
   NFFT4GP_HIP_CHECK(hipMemcpy(D.d_comps, D.comps.data(), sizeof(MdComp) * nw, hipMemcpyHostToDevice));
   if (!u.empty()) {
      NFFT4GP_HIP_CHECK(hipMemcpy(D.d_u, u.data(), sizeof(int) * u.size(), hipMemcpyHostToDevice));
      NFFT4GP_HIP_CHECK(hipMemcpy(D.d_psi, psi.data(), sizeof(double) * psi.size(), hipMemcpyHostToDevice));
   }
   NFFT4GP_HIP_CHECK(hipMemset(D.d_dot_ticket, 0, sizeof(unsigned int) * kTicketWords));
   // tiled spread: per component, a counting sort of the points by the tile of their first tap cell, then
   // items of at most ~2e6 / 10^d points (up to 3 features; 4-feature handles use the untiled kernels)
   if (D.maxd <= kMdTiledMaxDim) {
      // taps per work item (A/B knob NFFT4GP_AMD_MD_CHUNK; the results do not depend on it beyond the spread's
      // fixed-point rounding, which is exact)
      // The spread kernel: line-owned (k_md_spread_lines) when every window has 3 features and the tiles hold
      // ~1000 points or more (n >= 4e5 over 512 tiles), on 1000-point items; otherwise the wave-owned tiled
      // kernel on items of 256 (3-D) / 500 (2-D) points (profiles/r04_md_chunk_sweep.txt, r04_md_lines_ab.txt,
      // r04_md_lines_chunks.txt).  NFFT4GP_AMD_MD_SPREAD (0 untiled, 1 tiled, 2 lines) and
      // NFFT4GP_AMD_MD_CHUNK (taps per item) override.
      int mind = kMdMaxDim;
      for (const MdComp& c : D.comps) mind = std::min(mind, c.d);
      D.lines = mind == 3 && D.maxd == 3 && n >= 400000;
      if (const char* e = getenv("NFFT4GP_AMD_MD_SPREAD")) D.lines = atoi(e) == 2;
      long long chunk_taps = D.lines ? 1000000 : 50000;
      if (const char* e = getenv("NFFT4GP_AMD_MD_CHUNK")) chunk_taps = std::max(1000LL, atoll(e));
      std::vector<int> perm((size_t)P.nw * n);
      std::vector<std::vector<int4>> citems(P.nw);
      auto sort_comp = [&](int c) {
         std::vector<int4>& items = citems[c];
         const MdComp& cp = D.comps[c];
         const int d = cp.d;
         const int tiles_per_axis = kNos / kMdTile;
         int ntiles = 1, taps = 1;
         for (int t = 0; t < d; t++) {
            ntiles *= tiles_per_axis;
            taps *= kTaps;
         }
         std::vector<int> tile(n), cnt(ntiles + 1, 0);
         for (int j = 0; j < n; j++) {
            int tl = 0, mul = 1;
            for (int t = 0; t < d; t++) {
               tl += ((u[cp.u_off + (size_t)j * d + t] & (kNos - 1)) / kMdTile) * mul;
               mul *= tiles_per_axis;
            }
            tile[j] = tl;
            cnt[tl + 1]++;
         }
         for (int t = 0; t < ntiles; t++) cnt[t + 1] += cnt[t];
         std::vector<int> pos(cnt.begin(), cnt.end() - 1);
         int* pc = perm.data() + (size_t)c * n;
         for (int j = 0; j < n; j++) pc[pos[tile[j]]++] = j;
         const int chunk = (int)std::max<long long>(256, chunk_taps / taps);
         for (int t = 0; t < ntiles; t++)
            for (int b = cnt[t]; b < cnt[t + 1]; b += chunk) items.push_back(make_int4(c, t, b, std::min(cnt[t + 1], b + chunk)));
      };
      {
         std::vector<std::thread> th;
         std::atomic<int> next{0};
         for (int t = 0; t < std::min(nth, P.nw); t++)
            th.emplace_back([&]() {
               for (int c; (c = next.fetch_add(1)) < P.nw;) sort_comp(c);
            });
         for (auto& t : th) t.join();
      }
      std::vector<int4> items;
      for (auto& ci : citems) items.insert(items.end(), ci.begin(), ci.end());
      D.nitems = (int)items.size();
      if (dalloc(&D.d_perm, perm.size()) || dalloc(&D.d_items, items.size()) ||
          dalloc(&D.d_part, 2 * (size_t)P.nw * n))
         return -1;
      if (!perm.empty())
         NFFT4GP_HIP_CHECK(hipMemcpy(D.d_perm, perm.data(), sizeof(int) * perm.size(), hipMemcpyHostToDevice));
      if (!items.empty())
         NFFT4GP_HIP_CHECK(hipMemcpy(D.d_items, items.data(), sizeof(int4) * items.size(), hipMemcpyHostToDevice));
   }
   return upload_md_constants();
}

// every setup: weight * bhat * prod 1/PHI_HUT per component (nfft_interface.c:216-256, :536)
int md_setup(AdditivePlan& P)
{
   MdPlan& D = P.md;
   std::vector<double> bh((size_t)P.nw * D.M, 0.0), bhd((size_t)P.nw * D.M, 0.0), b0, b1;
   double phinv[kBand];
   for (int k = 0; k < kBand; k++) phinv[k] = 1.0 / kb_phi_hut(k - kBand / 2);
   for (int c = 0; c < P.nw; c++) {
      const int d = D.comps[c].d;
      const double sc = P.comp_scale[c], sig = P.comp_sigma[c];
      bhat_nd(P.kernel == 0 ? 0 : 2, d, sig, b0);
      bhat_nd(P.kernel == 0 ? 1 : 3, d, sig, b1);
      const double dscale = (P.kernel == 0) ? 2.0 * sc * std::sqrt(2.0) / sig : sc / sig;  // :536
      for (size_t j = 0; j < b0.size(); j++) {
         double di = 1.0;
         size_t jj = j;
         for (int t = 0; t < d; t++) {
            di *= phinv[jj % kBand];
            jj /= kBand;
         }
         bh[(size_t)c * D.M + j] = P.weight * b0[j] * di;
         bhd[(size_t)c * D.M + j] = P.weight * dscale * b1[j] * di;
      }
   }
   NFFT4GP_HIP_CHECK(hipMemcpy(D.d_bh, bh.data(), sizeof(double) * bh.size(), hipMemcpyHostToDevice));
   NFFT4GP_HIP_CHECK(hipMemcpy(D.d_bhd, bhd.data(), sizeof(double) * bhd.size(), hipMemcpyHostToDevice));
   return 0;
}

static int md_spread_fix(const AdditivePlan& P, const double* d_x, double psi_max, hipStream_t s);
static int md_spread_untiled(const AdditivePlan& P, const double* d_x, double psi_max, int c0, int nc, hipStream_t s);

int md_spread(const AdditivePlan& P, const double* d_x, double* d_grid, hipStream_t s)
{
   const MdPlan& D = P.md;
   const size_t count = (size_t)P.nw * D.G;
   if (P.n == 0) {
      NFFT4GP_HIP_CHECK(hipMemsetAsync(d_grid, 0, sizeof(double) * count, s));
      return 0;
   }
   // fixed-point bounds n max|x| psi_max^d_c (max|x| on the device)
   NFFT4GP_HIP_CHECK(hipMemsetAsync(D.d_xmax, 0, sizeof(unsigned long long), s));
   hipLaunchKernelGGL(k_md_absmax, dim3(std::min(1024, (P.n + 255) / 256)), dim3(256), 0, s, d_x, P.n, D.d_xmax);
   const unsigned gx = (unsigned)std::min<long long>(4096, (D.G + 255) / 256);
   if (D.gfix_per_window) {
      // one window's fixed-point grid at a time (4-feature windows: 64^4 cells, 268 MB each), untiled spread
      for (int c = 0; c < P.nw; c++) {
         NFFT4GP_HIP_CHECK(hipMemsetAsync(D.d_gfix, 0, 2 * sizeof(unsigned long long) * D.G, s));
         if (md_spread_untiled(P, d_x, D.psi_max, c, 1, s)) return -1;
         hipLaunchKernelGGL(k_md_fix2f, dim3(gx, 1), dim3(256), 0, s, (const MdComp*)D.d_comps,
                            (const unsigned long long*)D.d_gfix, D.G, (const unsigned long long*)D.d_xmax, (double)P.n,
                            D.psi_max, d_grid, c);
      }
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return 0;
   }
   NFFT4GP_HIP_CHECK(hipMemsetAsync(D.d_gfix, 0, 2 * sizeof(unsigned long long) * count, s));
   if (md_spread_fix(P, d_x, D.psi_max, s)) return -1;
   hipLaunchKernelGGL(k_md_fix2f, dim3(gx, P.nw), dim3(256), 0, s, (const MdComp*)D.d_comps,
                      (const unsigned long long*)D.d_gfix, D.G, (const unsigned long long*)D.d_xmax, (double)P.n,
                      D.psi_max, d_grid, 0);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

static int md_spread_fix(const AdditivePlan& P, const double* d_x, double psi_max, hipStream_t s)
{
   const MdPlan& D = P.md;
   static const int tiled = getenv("NFFT4GP_AMD_MD_SPREAD") ? atoi(getenv("NFFT4GP_AMD_MD_SPREAD")) : 1;
   if (D.lines && D.nitems > 0 && D.maxd <= kMdTiledMaxDim) {
      int mind = kMdMaxDim;
      for (const MdComp& c : D.comps) mind = std::min(mind, c.d);
      const size_t lds = kMdLinesStageLds + (mind < 3 ? kMdLinesRedLds : 0);
      static const bool attr = [] {
         (void)hipFuncSetAttribute((const void*)k_md_spread_lines, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024);
         (void)hipGetLastError();
         return true;
      }();
      (void)attr;
      hipLaunchKernelGGL(k_md_spread_lines, dim3(D.nitems), dim3(kMdLinesThreads), lds, s, D.d_comps, D.d_items,
                         D.d_perm, D.d_u, D.d_psi, d_x, P.n, D.d_gfix, D.G, (const unsigned long long*)D.d_xmax,
                         psi_max);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return 0;
   }
   if (tiled && D.nitems > 0 && D.maxd <= kMdTiledMaxDim) {
      size_t foot = 1;
      for (int t = 0; t < D.maxd; t++) foot *= kMdFoot;
      static bool attr = false;
      if (!attr) {
         (void)hipFuncSetAttribute((const void*)k_md_spread_tiled, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024);
         (void)hipGetLastError();
         attr = true;
      }
      hipLaunchKernelGGL(k_md_spread_tiled, dim3(D.nitems), dim3(kMdSpreadThreads), sizeof(double) * foot,
                         s, D.d_comps, D.d_items, D.d_perm, D.d_u, D.d_psi, d_x, P.n, D.d_gfix, D.G,
                         (const unsigned long long*)D.d_xmax, psi_max);
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return 0;
   }
   return md_spread_untiled(P, d_x, psi_max, 0, P.nw, s);
}

// the untiled spread of components [c0, c0 + nc) into D.d_gfix's first nc windows
static int md_spread_untiled(const AdditivePlan& P, const double* d_x, double psi_max, int c0, int nc, hipStream_t s)
{
   const MdPlan& D = P.md;
   int hi_max = 1;
   for (int t = 1; t < D.maxd; t++) hi_max *= kTaps;
   const long long work = (long long)P.n * hi_max;
   hipLaunchKernelGGL(k_md_spread, dim3((unsigned)((work + kMdThreads - 1) / kMdThreads), nc), dim3(kMdThreads), 0,
                      s, D.d_comps, D.d_u, D.d_psi, d_x, P.n, hi_max, D.d_gfix, D.G,
                      (const unsigned long long*)D.d_xmax, psi_max, c0);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int md_grid(const AdditivePlan& P, const double* d_grid, int grad, hipStream_t s)
{
   const MdPlan& D = P.md;
   // passes t >= 1 one thread per line once the grids pass the Infinity Cache (4 and 5 features: 64^4 complex
   // cells are 268 MB); 2- and 3-feature grids (4 MB) serve the per-output kernels' re-reads from L2 and keep
   // their parallelism (bike 0.31 vs 0.52 ms per matvec).  NFFT4GP_AMD_MD_LINES_DFT=0 / 2 forces one per output /
   // per line; the bits are the same (profiles/r06_md_lines_dft_ab.txt).
   static const int lines_env = getenv("NFFT4GP_AMD_MD_LINES_DFT") ? atoi(getenv("NFFT4GP_AMD_MD_LINES_DFT")) : 1;
   const bool lines_dft = lines_env == 2 || (lines_env == 1 && D.maxd >= 4);
   for (int t = 0; t < D.maxd; t++) {
      // largest pass over the components: 32^(t+1) 64^(maxd-t-1) outputs
      long long outs = 1;
      for (int a = 0; a <= t; a++) outs *= kBand;
      for (int a = t + 1; a < D.maxd; a++) outs *= kNos;
      if (t > 0 && lines_dft)  // one thread per line of 64 inputs
         hipLaunchKernelGGL(k_md_fwd_lines, dim3((unsigned)((outs / kBand + kMdThreads - 1) / kMdThreads), P.nw),
                            dim3(kMdThreads), 0, s, D.d_comps, t, D.d_F[0], D.d_F[1], D.Cmax);
      else
         hipLaunchKernelGGL(k_md_fwd, dim3((unsigned)((outs + kMdThreads - 1) / kMdThreads), P.nw), dim3(kMdThreads), 0,
                            s, D.d_comps, t, d_grid, D.G, D.d_F[0], D.d_F[1], D.Cmax);
   }
   hipLaunchKernelGGL(k_md_modes, dim3((unsigned)((D.M + kMdThreads - 1) / kMdThreads), P.nw), dim3(kMdThreads), 0, s,
                      D.d_comps, D.d_F[0], D.d_F[1], D.Cmax, D.d_bh, D.d_bhd, D.M, grad, D.d_Mo[0], D.d_Mo[1]);
   for (int t = 0; t < D.maxd; t++) {
      long long outs = 1;
      for (int a = 0; a <= t; a++) outs *= kNos;
      for (int a = t + 1; a < D.maxd; a++) outs *= kBand;
      if (t > 0 && lines_dft)  // one thread per line of 32 modes
         hipLaunchKernelGGL(k_md_bwd_lines, dim3((unsigned)((outs / kNos + kMdThreads - 1) / kMdThreads), P.nw,
                                                 grad ? 2 : 1),
                            dim3(kMdThreads), 0, s, D.d_comps, t, D.d_B[0], D.d_B[1], D.d_B[2], D.d_B[3], D.Cmax,
                            D.d_h[0], D.d_h[1], D.G);
      else
         hipLaunchKernelGGL(k_md_bwd, dim3((unsigned)((outs + kMdThreads - 1) / kMdThreads), P.nw, grad ? 2 : 1),
                            dim3(kMdThreads), 0, s, D.d_comps, t, D.d_Mo[0], D.d_Mo[1], D.M, D.d_B[0], D.d_B[1],
                            D.d_B[2], D.d_B[3], D.Cmax, D.d_h[0], D.d_h[1], D.G);
   }
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

int md_interp(const AdditivePlan& P, int grad, double alpha, const double* d_x, double beta, double* d_y,
              hipStream_t s, double* d_dot)
{
   const MdPlan& D = P.md;
   if (P.n == 0) {
      if (d_dot) NFFT4GP_HIP_CHECK(hipMemsetAsync(d_dot, 0, sizeof(double), s));
      return 0;
   }
   static const int tiled = getenv("NFFT4GP_AMD_MD_INTERP") ? atoi(getenv("NFFT4GP_AMD_MD_INTERP")) : 1;
   // small handles (TEST1's bike: ~34 points per 3-D tile) stage more footprint than they read: one wave per
   // point over the L2-resident grid instead
   long long tiles = 1;
   for (int t = 0; t < D.maxd; t++) tiles *= kNos / kMdTile;
   if (tiled && D.nitems > 0 && D.d_part && D.maxd <= kMdTiledMaxDim && (long long)P.n >= 100 * tiles) {
      size_t foot = 1;
      for (int t = 0; t < D.maxd; t++) foot *= kMdFoot;
      static bool attr = false;
      if (!attr) {
         (void)hipFuncSetAttribute((const void*)k_md_interp_tiled<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024);
         (void)hipFuncSetAttribute((const void*)k_md_interp_tiled<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024);
         (void)hipGetLastError();
         attr = true;
      }
      if (grad)
         hipLaunchKernelGGL(k_md_interp_tiled<1>, dim3(D.nitems), dim3(kMdSpreadThreads), 2 * sizeof(double) * foot, s,
                            D.d_comps, D.d_items, D.d_perm, D.d_u, D.d_psi, D.d_h[0], D.d_h[1], D.G, P.n, P.nw,
                            D.d_part);
      else
         hipLaunchKernelGGL(k_md_interp_tiled<0>, dim3(D.nitems), dim3(kMdSpreadThreads), sizeof(double) * foot, s,
                            D.d_comps, D.d_items, D.d_perm, D.d_u, D.d_psi, D.d_h[0], D.d_h[1], D.G, P.n, P.nw,
                            D.d_part);
      const int cb = std::min(kMdInterpBlocks, (P.n + kMdThreads - 1) / kMdThreads);
#define NFFT4GP_MD_COMBINE(G_, D_)                                                                               \
   hipLaunchKernelGGL((k_md_combine<G_, D_>), dim3(cb), dim3(kMdThreads), 0, s, P.nw, (const double*)D.d_part, d_x, \
                      d_y, P.n, alpha, beta, P.f, P.mu * P.diag, P.diag, D.d_dot_part, D.d_dot_ticket, d_dot)
      if (grad)
         NFFT4GP_MD_COMBINE(1, 0);
      else if (d_dot)
         NFFT4GP_MD_COMBINE(0, 1);
      else
         NFFT4GP_MD_COMBINE(0, 0);
#undef NFFT4GP_MD_COMBINE
      NFFT4GP_HIP_CHECK(hipGetLastError());
      return 0;
   }
   const int blocks = std::min(kMdInterpBlocks, (P.n + kMdThreads / 64 - 1) / (kMdThreads / 64));
#define NFFT4GP_MD_INTERP(G_, D_)                                                                              \
   hipLaunchKernelGGL((k_md_interp<G_, D_>), dim3(blocks), dim3(kMdThreads), 0, s, D.d_comps, P.nw, D.d_u, D.d_psi, \
                      D.d_h[0], D.d_h[1], D.G, d_x, d_y, P.n, alpha, beta, P.f, P.mu * P.diag, P.diag, D.d_dot_part,          \
                      D.d_dot_ticket, \
                      d_dot)
   if (grad)
      NFFT4GP_MD_INTERP(1, 0);
   else if (d_dot)
      NFFT4GP_MD_INTERP(0, 1);
   else
      NFFT4GP_MD_INTERP(0, 0);
#undef NFFT4GP_MD_INTERP
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

}  // namespace nfft4gp_amd
