// layout.cpp -- cell-bucketed chunk layout of the fixed NFFT nodes (host, built once per handle).
//
// The reference fixes the nodes at the first setup call and only refreshes the kernel
// coefficients afterwards (nfft_interface.c:150 `_scale < 0` test, :216-254).  We exploit that by
// bucketing, once, every block of B consecutive points by oversampled-grid cell, per component:
//
//   block b = points [b*B, (b+1)*B)           (B <= kMaxBlock = 4064: local index and the 32 pad
//                                               entries B .. B+31 used by dummies fit 12 bits)
//   group g = components [g*CG, (g+1)*CG)
//   chunk   = up to R points of ONE (component, cell), padded with dummies (local index B + lane%32,
//             pad entries the kernels hold at zero alpha / discard as output); the points of a chunk
//             are ordered per tile to spread the lanes over LDS banks (balance_tile)
//   tile    = 64 chunks, one per lane (dealt column-wise, see emit_block_group); a lane's words are
//             grouped in 16-byte quads, quads lane-fastest, so each lane loads 16 B per instruction
//             and a wave instruction reads 1 KiB contiguous (quad_index in internal.h):
//               meta [tile][lane]            u16  comp << 6 | cell
//               q    [tile][r/4][lane][r%4]  u32  slot_word (internal.h): the offset in the cell in 2^-32 cell
//                                                  units, its low 4 bits = local index bits 0-3, bit 31 flipped
//               lo   [tile][0][lane][r/4]    u32  byte r%4 = local index bits 4-11
//             5 bytes per (point, window): the chunk's cell lives in meta.  The kernels read the q word as a
//             signed int32: s = (int)q = 2^32 (offset - 1/2), one conversion for the centred offset scaled by 2^32
//             (the 2^-32d are folded into the tap polynomial coefficients); carrying 4 index bits moves a point by
//             at most an eighth of the coordinates' 2^-26-of-a-cell quantum.
//   rec 4 (32-bit precision mode): no lo array; q = slot_word4 (internal.h), the 12-bit index in the low bits.
//   tile_off[b*ngroups + g] = first tile of (b, g); the spread kernel gets one workgroup per (b, g),
//   the interpolation kernel one workgroup per b (all groups).
#include <algorithm>
#include <thread>

#include "internal.h"

namespace nfft4gp_amd {

namespace {

struct ChunkSink {
   // count-only pass when arrays are null
   uint16_t* meta;
   uint32_t* lo;
   uint32_t* q;
};

inline uint32_t lo_word(const uint32_t* loc4)
{
   return lo_byte(loc4[0]) | (lo_byte(loc4[1]) << 8) | (lo_byte(loc4[2]) << 16) | (lo_byte(loc4[3]) << 24);
}

// Order the 16 points of every lane's run so that, at each point slot r, the 64 lanes of a tile hit
// different LDS banks: the spread gathers alpha[loc] with ds_read_b64 (bank pair = loc mod 32 within
// each 32-lane half) and the interpolation adds into y[loc] with ds_add_f64 (loc mod 16 within each
// 16-lane quarter).  Random order costs ~4-way conflicts; a greedy pass per slot gets close to
// conflict-free.  Dummy slots point at pad entry B + lane % 32 (distinct banks, no same-address
// atomics).  Any order is correct: the sums over a run are order-independent up to rounding.
void balance_tile(uint32_t (*loc)[kR], uint32_t (*fr)[kR])
{
   for (int r = 0; r < kR; r++) {
      int c32[2][32] = {};
      int c16[4][16] = {};
      for (int lane = 0; lane < kWave; lane++) {
         int best = r, best_cost = 1 << 30;
         for (int k = r; k < kR; k++) {
            const uint32_t v = loc[lane][k];
            const int cost = 2 * c32[lane >> 5][v & 31] + c16[lane >> 4][v & 15];
            if (cost < best_cost) {
               best_cost = cost;
               best = k;
               if (cost == 0) break;
            }
         }
         std::swap(loc[lane][r], loc[lane][best]);
         std::swap(fr[lane][r], fr[lane][best]);
         c32[lane >> 5][loc[lane][r] & 31]++;
         c16[lane >> 4][loc[lane][r] & 15]++;
      }
   }
}

// enumerate the chunks of (block b, group g) in (component, cell) order; returns the number of
// tiles.  With arrays, writes them into tiles [t0, t0 + T) where T = ntiles: chunk k goes to tile
// t0 + k % T, lane k / T ("dealt" column-wise), so the 64 lanes of a tile hold chunks T apart in the
// sorted order -- different cells -- and their LDS flushes do not collide on one address.
long long emit_block_group(const uint32_t* qc, int n, int nw, int B, int CG, int b, int g,
                           const ChunkSink* out, long long t0, long long T, std::vector<int>& cnt,
                           std::vector<int>& off, std::vector<uint16_t>& sorted, int* cmax = nullptr, int rec = 5)
{
   const int base = b * B;
   const int nloc = std::min(B, n - base);
   const int c0 = g * CG, c1 = std::min(nw, c0 + CG);
   // staging of the group's tiles: [tile][lane][r] local index and offset-in-cell
   std::vector<uint32_t> sloc, sfr;
   if (out) {
      // every slot starts as a dummy chunk of the group's first component
      sloc.resize((size_t)T * kWave * kR);
      sfr.assign((size_t)T * kWave * kR, 0u);
      for (long long tile = 0; tile < T; tile++)
         for (int lane = 0; lane < kWave; lane++) {
            out->meta[(t0 + tile) * kWave + lane] = (uint16_t)(c0 << 6);
            for (int r = 0; r < kR; r++) sloc[((size_t)tile * kWave + lane) * kR + r] = (uint32_t)(B + (lane & 31));
         }
   }
   long long nchunks = 0;
   for (int c = c0; c < c1; c++) {
      const uint32_t* qq = qc + (size_t)c * n + base;
      std::fill(cnt.begin(), cnt.end(), 0);
      for (int j = 0; j < nloc; j++) cnt[qq[j] >> 26]++;
      if (cmax)
         for (int cell = 0; cell < kNos; cell++) *cmax = std::max(*cmax, cnt[cell]);
      off[0] = 0;
      for (int cell = 0; cell < kNos; cell++) off[cell + 1] = off[cell] + cnt[cell];
      if (out) {
         std::vector<int> pos(off.begin(), off.end() - 1);
         for (int j = 0; j < nloc; j++) sorted[pos[qq[j] >> 26]++] = (uint16_t)j;  // stable
      }
      for (int cell = 0; cell < kNos; cell++) {
         for (int s = off[cell]; s < off[cell + 1]; s += kR) {
            if (out) {
               const long long chunk = nchunks;
               const long long tile = chunk % T;
               const int lane = (int)(chunk / T);
               out->meta[(t0 + tile) * kWave + lane] = (uint16_t)((c << 6) | cell);
               for (int r = 0; r < kR; r++) {
                  const int sidx = s + r;
                  const size_t k = ((size_t)tile * kWave + lane) * kR + r;
                  if (sidx < off[cell + 1]) {
                     sloc[k] = sorted[sidx];
                     sfr[k] = qq[sorted[sidx]] & 0x3FFFFFFu;
                  }  // else: stays a dummy (pad entry B + lane % 32: zero alpha / discarded output)
               }
            }
            nchunks++;
         }
      }
   }
   if (out) {
      for (long long tile = 0; tile < T; tile++) {
         auto* L = reinterpret_cast<uint32_t(*)[kR]>(sloc.data() + (size_t)tile * kWave * kR);
         auto* F = reinterpret_cast<uint32_t(*)[kR]>(sfr.data() + (size_t)tile * kWave * kR);
         balance_tile(L, F);
         for (int lane = 0; lane < kWave; lane++) {
            if (rec == 5)
               for (int r4 = 0; r4 < kR / 4; r4++)
                  out->lo[quad_index(t0 + tile, r4, lane, kR / 4)] = lo_word(L[lane] + 4 * r4);
            for (int r = 0; r < kR; r++)
               out->q[quad_index(t0 + tile, r, lane, kR)] =
                   rec == 5 ? slot_word(L[lane][r], F[lane][r]) : slot_word4(L[lane][r], F[lane][r]);
         }
      }
   }
   return (nchunks + kWave - 1) / kWave;
}

template <class F>
void parallel_for(int nitems, F&& f)
{
   unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
   if (nitems < 4) nt = 1;
   std::vector<std::thread> th;
   for (unsigned t = 0; t < nt; t++)
      th.emplace_back([&, t] {
         for (int i = (int)t; i < nitems; i += (int)nt) f(i);
      });
   for (auto& x : th) x.join();
}

}  // namespace

void build_layout(const uint32_t* qc, int n, int nw, int B, int CG, Layout& L, int rec)
{
   L.n = n;
   L.nw = nw;
   L.B = B;
   L.CG = CG;
   L.ngroups = (nw + CG - 1) / CG;
   L.nblocks = (n + B - 1) / B;
   const int nbg = L.nblocks * L.ngroups;
   std::vector<long long> tiles(nbg, 0);
   L.cmax.assign(nbg, 0);
   parallel_for(L.nblocks, [&](int b) {
      std::vector<int> cnt(kNos), off(kNos + 1);
      std::vector<uint16_t> sorted(B);
      for (int g = 0; g < L.ngroups; g++)
         tiles[b * L.ngroups + g] = emit_block_group(qc, n, nw, B, CG, b, g, nullptr, 0, 0, cnt, off, sorted,
                                                     &L.cmax[b * L.ngroups + g]);
   });
   L.tile_off.assign(nbg + 1, 0);
   long long acc = 0;
   for (int i = 0; i < nbg; i++) {
      L.tile_off[i] = (int)acc;
      acc += tiles[i];
   }
   L.tile_off[nbg] = (int)acc;
   L.ntiles = acc;
   L.meta.resize((size_t)acc * kWave);  // every element is written below (emit_block_group)
   L.lo.resize(rec == 5 ? (size_t)acc * (kR / 4) * kWave : 0);
   L.q.resize((size_t)acc * kR * kWave);
   ChunkSink sink{L.meta.data(), L.lo.data(), L.q.data()};
   parallel_for(L.nblocks, [&](int b) {
      std::vector<int> cnt(kNos), off(kNos + 1);
      std::vector<uint16_t> sorted(B);
      for (int g = 0; g < L.ngroups; g++)
         emit_block_group(qc, n, nw, B, CG, b, g, &sink, L.tile_off[b * L.ngroups + g],
                          L.tile_off[b * L.ngroups + g + 1] - L.tile_off[b * L.ngroups + g], cnt, off, sorted,
                          nullptr, rec);
   });
}

}  // namespace nfft4gp_amd
