// layout_gpu.hip -- the cell-bucketed chunk layout (layout.cpp) built on the device, bit-identical to the
// host builder: the same stable counting sort per (block, window), the same chunk enumeration and
// column-wise dealing, the same greedy bank balancing per tile, the same 16-byte-quad packing.
//
//   k_lay_count   one workgroup per (block, window group): tiles of the group (chunks / 64)
//   (host)        prefix sum -> tile_off, allocation of meta / lo / q
//   k_lay_emit    one workgroup per (block, window group): a wave per window sorts the block's points by
//                 cell (64-lane ballot ranks keep the order stable), the workgroup deals the chunks into
//                 LDS-staged tiles, one thread per tile balances it, and the tiles are written out.
//
// Called from plan_build_points (nfft_api.cpp) on the quantised coordinates; layout.cpp stays the
// reference the tests compare against (Nfft4GPAmdHostLayout / Nfft4GPAmdDeviceLayout).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "callbacks.hpp"
#include "internal.h"

namespace nfft4gp_amd {

namespace {

constexpr int kLT = 256;
constexpr int kLWaves = kLT / 64;

__global__ __launch_bounds__(kLT) void k_lay_count(const uint32_t* __restrict__ qc, int n, int nw, int B, int CG,
                                                   int ngroups, int* __restrict__ tiles, int* __restrict__ cmax)
{
   __shared__ int hist[kNos];
   __shared__ int nch, mx;
   const int bg = blockIdx.x, b = bg / ngroups, g = bg % ngroups;
   const int base = b * B, nloc = min(B, n - base);
   const int c0 = g * CG, c1 = min(nw, c0 + CG);
   const int tid = threadIdx.x;
   if (tid == 0) nch = mx = 0;
   for (int c = c0; c < c1; c++) {
      const uint32_t* qq = qc + (size_t)c * n + base;
      if (tid < kNos) hist[tid] = 0;
      __syncthreads();
      for (int j = tid; j < nloc; j += kLT) atomicAdd(&hist[qq[j] >> 26], 1);
      __syncthreads();
      if (tid < 64) {
         int v = (hist[tid] + kR - 1) / kR, m = hist[tid];
         for (int off = 32; off > 0; off >>= 1) {
            v += __shfl_xor(v, off, 64);
            m = max(m, __shfl_xor(m, off, 64));
         }
         if (tid == 0) {
            nch += v;
            mx = max(mx, m);
         }
      }
      __syncthreads();
   }
   if (tid == 0) {
      tiles[bg] = (nch + kWave - 1) / kWave;
      cmax[bg] = mx;
   }
}

struct EmitLds {
   // byte offsets into the dynamic LDS block
   size_t off, run, cbase, sorted, sloc, sfr, smeta, cnt, total;
   __host__ __device__ EmitLds(int CG, int B, int Tmax)
   {
      size_t p = 0;
      auto take = [&](size_t bytes) {
         const size_t at = p;
         p += (bytes + 15) & ~(size_t)15;
         return at;
      };
      off = take(sizeof(int) * CG * (kNos + 1));
      run = take(sizeof(int) * CG * kNos);
      cbase = take(sizeof(int) * (CG * kNos + 1));
      // the sorted indices are dead once the chunks are dealt (step 3), before the balance counters are used
      // (step 4): one region serves both, so four windows per group fit at B = 4064
      const size_t sorted_bytes = sizeof(uint16_t) * CG * B, cnt_bytes = sizeof(int) * Tmax * (2 * 32 + 4 * 16);
      sorted = take(sorted_bytes > cnt_bytes ? sorted_bytes : cnt_bytes);
      cnt = sorted;
      sloc = take(sizeof(uint16_t) * Tmax * kWave * kR);
      sfr = take(sizeof(uint32_t) * Tmax * kWave * kR);
      smeta = take(sizeof(uint16_t) * Tmax * kWave);
      total = p;
   }
};

template <int REC>
__global__ __launch_bounds__(kLT) void k_lay_emit(const uint32_t* __restrict__ qc, int n, int nw, int B, int CG,
                                                  int ngroups, int Tmax, const int* __restrict__ tile_off,
                                                  uint16_t* __restrict__ meta, uint32_t* __restrict__ lo,
                                                  uint32_t* __restrict__ q)
{
   extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
   const EmitLds E(CG, B, Tmax);
   int* s_off = reinterpret_cast<int*>(lds + E.off);          // [CG][65]
   int* s_run = reinterpret_cast<int*>(lds + E.run);          // [CG][64]
   int* s_cbase = reinterpret_cast<int*>(lds + E.cbase);      // [CG*64 + 1]
   uint16_t* s_sorted = reinterpret_cast<uint16_t*>(lds + E.sorted);  // [CG][B]
   uint16_t* s_loc = reinterpret_cast<uint16_t*>(lds + E.sloc);       // [T][64][16]
   uint32_t* s_fr = reinterpret_cast<uint32_t*>(lds + E.sfr);         // [T][64][16]
   uint16_t* s_meta = reinterpret_cast<uint16_t*>(lds + E.smeta);     // [T][64]
   int* s_cnt = reinterpret_cast<int*>(lds + E.cnt);                  // [T][128] balance counters (step 4; aliases s_sorted)

   const int bg = blockIdx.x, b = bg / ngroups, g = bg % ngroups;
   const int base = b * B, nloc = min(B, n - base);
   const int c0 = g * CG, c1 = min(nw, c0 + CG), ncomp = c1 - c0;
   const int t0 = tile_off[bg], T = tile_off[bg + 1] - t0;
   const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

   // 1. per window: cell histogram, offsets, stable scatter of the local indices (one wave per window;
   //    uniform loops so every barrier is reached by the whole workgroup)
   for (int ci0 = 0; ci0 < ncomp; ci0 += kLWaves) {
      const int ci = ci0 + wave;
      const bool act = ci < ncomp;
      const uint32_t* qq = qc + (size_t)(c0 + (act ? ci : 0)) * n + base;
      int* off = s_off + (act ? ci : 0) * (kNos + 1);
      int* run = s_run + (act ? ci : 0) * kNos;
      uint16_t* sorted = s_sorted + (size_t)(act ? ci : 0) * B;
      if (act) run[lane] = 0;
      __syncthreads();
      if (act)
         for (int j = lane; j < nloc; j += 64) atomicAdd(&run[qq[j] >> 26], 1);
      __syncthreads();
      if (act) {
         const int v = run[lane];
         int incl = v;
         for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(incl, d, 64);
            if (lane >= d) incl += t;
         }
         off[lane] = incl - v;
         if (lane == 63) off[kNos] = incl;
         run[lane] = incl - v;
      }
      __syncthreads();
      for (int jb = 0; jb < nloc; jb += 64) {
         const int j = jb + lane;
         const bool valid = act && j < nloc;
         const int cell = valid ? (int)(qq[j] >> 26) : 0;
         unsigned long long peers = __ballot(valid);
#pragma unroll
         for (int bit = 0; bit < 6; bit++) {
            const unsigned long long set = __ballot(valid && ((cell >> bit) & 1));
            peers &= ((cell >> bit) & 1) ? set : ~set;
         }
         const int rank = __popcll(peers & ((1ull << lane) - 1ull));
         const int start = valid ? run[cell] : 0;
         __syncthreads();
         if (valid) {
            sorted[start + rank] = (uint16_t)j;
            if (lane == 63 - __clzll(peers)) run[cell] = start + __popcll(peers);  // the group's last lane
         }
         __syncthreads();
      }
   }
   // 2. chunk bases in (window, cell) order
   if (tid == 0) {
      int acc = 0;
      for (int i = 0; i < ncomp * kNos; i++) {
         s_cbase[i] = acc;
         const int* off = s_off + (i / kNos) * (kNos + 1);
         const int cnt = off[i % kNos + 1] - off[i % kNos];
         acc += (cnt + kR - 1) / kR;
      }
      s_cbase[ncomp * kNos] = acc;
   }
   // every slot starts as a dummy chunk of the group's first window
   for (int i = tid; i < T * kWave * kR; i += kLT) {
      s_loc[i] = (uint16_t)(B + ((i / kR) % kWave & 31));
      s_fr[i] = 0u;
   }
   for (int i = tid; i < T * kWave; i += kLT) s_meta[i] = (uint16_t)(c0 << 6);
   __syncthreads();
   // 3. deal the chunks: chunk k -> tile k % T, lane k / T
   const int nchunks = s_cbase[ncomp * kNos];
   for (int k = tid; k < nchunks; k += kLT) {
      int lo_i = 0, hi_i = ncomp * kNos;  // last i with cbase[i] <= k
      while (hi_i - lo_i > 1) {
         const int mid = (lo_i + hi_i) >> 1;
         if (s_cbase[mid] <= k) lo_i = mid;
         else hi_i = mid;
      }
      const int ci = lo_i / kNos, cell = lo_i % kNos;
      const int* off = s_off + ci * (kNos + 1);
      const int s = off[cell] + (k - s_cbase[lo_i]) * kR;
      const int tile = k % T, ln = k / T;
      s_meta[tile * kWave + ln] = (uint16_t)(((c0 + ci) << 6) | cell);
      const uint32_t* qq = qc + (size_t)(c0 + ci) * n + base;
      const uint16_t* sorted = s_sorted + (size_t)ci * B;
      for (int r = 0; r < kR; r++) {
         const int sidx = s + r;
         if (sidx < off[cell + 1]) {
            const int loc = sorted[sidx];
            s_loc[(tile * kWave + ln) * kR + r] = (uint16_t)loc;
            s_fr[(tile * kWave + ln) * kR + r] = qq[loc] & 0x3FFFFFFu;
         }
      }
   }
   __syncthreads();
   // 4. bank balancing, one thread per tile (layout.cpp balance_tile, the same greedy order)
   if (tid < T) {
      uint16_t* L = s_loc + (size_t)tid * kWave * kR;
      uint32_t* F = s_fr + (size_t)tid * kWave * kR;
      int* c32 = s_cnt + tid * 128;  // [2][32]
      int* c16 = c32 + 64;           // [4][16]
      for (int r = 0; r < kR; r++) {
         for (int i = 0; i < 128; i++) c32[i] = 0;
         for (int ln = 0; ln < kWave; ln++) {
            int best = r, best_cost = 1 << 30;
            for (int k = r; k < kR; k++) {
               const int v = L[ln * kR + k];
               const int cost = 2 * c32[(ln >> 5) * 32 + (v & 31)] + c16[(ln >> 4) * 16 + (v & 15)];
               if (cost < best_cost) {
                  best_cost = cost;
                  best = k;
                  if (cost == 0) break;
               }
            }
            const uint16_t tl = L[ln * kR + r];
            L[ln * kR + r] = L[ln * kR + best];
            L[ln * kR + best] = tl;
            const uint32_t tf = F[ln * kR + r];
            F[ln * kR + r] = F[ln * kR + best];
            F[ln * kR + best] = tf;
            const int v = L[ln * kR + r];
            c32[(ln >> 5) * 32 + (v & 31)]++;
            c16[(ln >> 4) * 16 + (v & 15)]++;
         }
      }
   }
   __syncthreads();
   // 5. write the tiles out in the 16-byte-quad layout
   for (int i = tid; i < T * kWave; i += kLT) meta[(size_t)(t0 + i / kWave) * kWave + i % kWave] = s_meta[i];
   for (int i = tid; i < T * kWave * kR; i += kLT) {
      const int tile = i / (kWave * kR), ln = (i / kR) % kWave, r = i % kR;
      const uint32_t loc = s_loc[i];
      q[quad_index(t0 + tile, r, ln, kR)] = REC == 5 ? slot_word(loc, s_fr[i]) : slot_word4(loc, s_fr[i]);
   }
   if (REC != 5) return;
   for (int i = tid; i < T * kWave * (kR / 4); i += kLT) {
      const int tile = i / (kWave * (kR / 4)), ln = (i / (kR / 4)) % kWave, r4 = i % (kR / 4);
      const uint16_t* l4 = s_loc + ((size_t)tile * kWave + ln) * kR + 4 * r4;
      lo[quad_index(t0 + tile, r4, ln, kR / 4)] =
          lo_byte(l4[0]) | (lo_byte(l4[1]) << 8) | (lo_byte(l4[2]) << 16) | (lo_byte(l4[3]) << 24);
   }
}

}  // namespace

// the layout of the device-resident quantised coordinates d_qc ([window][point] u32) into P.dl and
// P.ngroups / P.nblocks; -1 when a (block, group) would not fit the emit kernel's LDS (the caller then
// builds on the host)
int build_layout_dev(const uint32_t* d_qc, int n, int nw, int B, int CG, AdditivePlan& P, hipStream_t s, int rec)
{
   const int ngroups = (nw + CG - 1) / CG, nblocks = (n + B - 1) / B, nbg = ngroups * nblocks;
   const int Tmax_bound = (CG * (B / kR + kNos) + kWave - 1) / kWave + 1;
   // the emit kernel's LDS is sized by the largest (block, group) actually counted (checked below); a group too
   // large even at its smallest possible tile count goes to the host builder at once
   if (EmitLds(CG, B, (CG * ((B + kR - 1) / kR) + kWave - 1) / kWave).total > 160 * 1024) return -1;
   int* d_tiles = nullptr;
   int* d_cmax = nullptr;
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&d_tiles, sizeof(int) * (nbg + 1)));
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&d_cmax, sizeof(int) * std::max(1, nbg)));
   hipLaunchKernelGGL(k_lay_count, dim3(std::max(1, nbg)), dim3(kLT), 0, s, d_qc, n, nw, B, CG, ngroups, d_tiles,
                      d_cmax);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   std::vector<int> tiles(nbg);
   NFFT4GP_HIP_CHECK(hipMemcpyAsync(tiles.data(), d_tiles, sizeof(int) * nbg, hipMemcpyDeviceToHost, s));
   NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
   std::vector<int> toff(nbg + 1, 0);
   long long acc = 0;
   int Tmax = 1;
   for (int i = 0; i < nbg; i++) {
      toff[i] = (int)acc;
      acc += tiles[i];
      Tmax = std::max(Tmax, tiles[i]);
   }
   toff[nbg] = (int)acc;
   if (Tmax > Tmax_bound || EmitLds(CG, B, Tmax).total > 160 * 1024) {
      (void)hipFree(d_tiles);
      (void)hipFree(d_cmax);
      return -1;
   }
   P.ngroups = ngroups;
   P.nblocks = nblocks;
   P.dl = DevLayout();
   P.dl.cmax = d_cmax;
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&P.dl.tile_off, sizeof(int) * (nbg + 1)));
   NFFT4GP_HIP_CHECK(hipMemcpyAsync(P.dl.tile_off, toff.data(), sizeof(int) * (nbg + 1), hipMemcpyHostToDevice, s));
   const size_t nt = (size_t)std::max<long long>(acc, 1);
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&P.dl.meta, sizeof(uint16_t) * nt * kWave));
   if (rec == 5) NFFT4GP_HIP_CHECK(hipMalloc((void**)&P.dl.lo, sizeof(uint32_t) * nt * (kR / 4) * kWave));
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&P.dl.q, sizeof(uint32_t) * nt * kR * kWave));
   const size_t lds = EmitLds(CG, B, Tmax).total;
   static const bool attr = []() {
      (void)hipFuncSetAttribute((const void*)k_lay_emit<5>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)k_lay_emit<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipGetLastError();
      return true;
   }();
   (void)attr;
   if (nbg > 0)
      hipLaunchKernelGGL(rec == 5 ? k_lay_emit<5> : k_lay_emit<4>, dim3(nbg), dim3(kLT), lds, s, d_qc, n, nw, B, CG,
                         ngroups, Tmax, P.dl.tile_off, P.dl.meta, P.dl.lo, P.dl.q);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
   (void)hipFree(d_tiles);
   P.dl.ntiles = acc;
   P.dl.bytes = (size_t)acc * kWave * (2 + (rec == 5 ? 4 * (kR / 4) : 0) + 4 * kR) + sizeof(int) * (nbg + 1);
   return 0;
}

}  // namespace nfft4gp_amd

extern "C" int Nfft4GPAmdDeviceLayoutRec(const unsigned int* qc, int n, int nw, int B, int CG, int rec,
                                         long long* counts, unsigned short* meta, unsigned int* lo, unsigned int* q,
                                         int* tile_off);
extern "C" int Nfft4GPAmdDeviceLayout(const unsigned int* qc, int n, int nw, int B, int CG, long long* counts,
                                      unsigned short* meta, unsigned int* lo, unsigned int* q, int* tile_off)
{
   return Nfft4GPAmdDeviceLayoutRec(qc, n, nw, B, CG, 5, counts, meta, lo, q, tile_off);
}

extern "C" int Nfft4GPAmdDeviceLayoutRec(const unsigned int* qc, int n, int nw, int B, int CG, int rec,
                                         long long* counts, unsigned short* meta, unsigned int* lo, unsigned int* q,
                                         int* tile_off)
{
   using namespace nfft4gp_amd;
   if (B <= 0 || B > kMaxBlock || CG <= 0 || n < 0 || nw <= 0 || nw > 1023 || !counts || (rec != 4 && rec != 5))
      return -1;
   if (!need_device("Nfft4GPAmdDeviceLayout")) return -1;
   hipStream_t s = current_stream();
   uint32_t* d_qc = nullptr;
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&d_qc, sizeof(uint32_t) * std::max<size_t>(1, (size_t)n * nw)));
   NFFT4GP_HIP_CHECK(hipMemcpy(d_qc, qc, sizeof(uint32_t) * (size_t)n * nw, hipMemcpyHostToDevice));
   AdditivePlan P;
   const int rc = build_layout_dev(d_qc, n, nw, B, CG, P, s, rec);
   (void)hipFree(d_qc);
   if (rc) return -1;
   const int nbg = P.ngroups * P.nblocks;
   counts[0] = P.dl.ntiles;
   counts[1] = P.ngroups;
   counts[2] = P.nblocks;
   const size_t nt = (size_t)P.dl.ntiles;
   int err = 0;
   if (meta && hipMemcpy(meta, P.dl.meta, sizeof(uint16_t) * nt * kWave, hipMemcpyDeviceToHost) != hipSuccess) err = 1;
   if (lo && rec == 5 &&
       hipMemcpy(lo, P.dl.lo, sizeof(uint32_t) * nt * (kR / 4) * kWave, hipMemcpyDeviceToHost) != hipSuccess)
      err = 1;
   if (q && hipMemcpy(q, P.dl.q, sizeof(uint32_t) * nt * kR * kWave, hipMemcpyDeviceToHost) != hipSuccess) err = 1;
   if (tile_off && hipMemcpy(tile_off, P.dl.tile_off, sizeof(int) * (nbg + 1), hipMemcpyDeviceToHost) != hipSuccess)
      err = 1;
   for (void* p : {(void*)P.dl.meta, (void*)P.dl.lo, (void*)P.dl.q, (void*)P.dl.tile_off, (void*)P.dl.cmax})
      (void)hipFree(p);
   return err ? -1 : 0;
}
