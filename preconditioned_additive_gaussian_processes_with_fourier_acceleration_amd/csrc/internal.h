// internal.h -- private types of the MI355X NFFT additive-kernel operator.
//
// Algorithm (1-D additive components, the BASELINE configurations B-E):
//   The reference (nfft_interface.c:400-497 -> NFFT3 fastsum_trafo) computes per component
//     f = B diag(1/phihut) F^T [bhat] F diag(1/phihut) B^T alpha
//   with B the 2m+2 = 10-tap Kaiser-Bessel spreading matrix onto a 64-cell periodic grid and F the
//   32-mode DFT.  For one component the middle factor is a real 64x64 circulant W (only Re f is used,
//   nfft_interface.c:436) and each tap is an entire function of the point's offset u in its cell.
//   We write the 10 taps as degree-7 polynomials in u (max error 3.8e-8 of the window peak, the KB window's own
//   truncation level; the band-limited circulant filters the error's high-frequency content, so against the
//   oracle the matvec moves by at most 1.4x the coordinate quantisation's error: DESIGN 3.1), so
//     spread : M[cell][d] = sum_{j in cell} alpha_j u_j^d        (per-cell moments)
//              g[(cell-4+t) mod 64] += sum_d C[t][d] M[cell][d]
//     grid   : h = W g,   H[cell][d] = sum_t h[(cell-4+t) mod 64] C[t][d]
//     interp : f_j = sum_d H[cell_j][d] u_j^d                     (Horner)
//   Points are bucketed by cell at setup (the nodes are fixed after the first setup call,
//   nfft_interface.c:150) so a lane owns a run of R points of one cell: moments accumulate in
//   registers and the interpolation coefficients are loaded once per run.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <utility>
#include <string>
#include <vector>

#include "../../include/nfft4gp_amd.h"

namespace nfft4gp_amd {

constexpr int kNos = 64;            // oversampled grid n_os (nfft_interface.c:25-27)
constexpr int kBand = 32;           // bandwidth N (nfft_interface.c:18)
constexpr int kM = 4;               // window cutoff m (nfft_interface.c:20)
constexpr int kTaps = 2 * kM + 2;   // PRE_PSI taps per dim
constexpr int kDeg = 7;             // tap polynomial degree (round 5: 9 -> 7)
constexpr int kNC = kDeg + 1;       // coefficients per cell
constexpr int kR = 16;              // points per lane-run (chunk)
constexpr int kWave = 64;
constexpr int kPad = 32;            // pad entries after a block's B points (dummy slots, one per bank)
constexpr int kMaxBlock = 4096 - kPad;  // points per block: local index and pad entries fit 12 bits

#define NFFT4GP_HIP_CHECK(expr)                                                                    \
   do {                                                                                            \
      hipError_t _e = (expr);                                                                      \
      if (_e != hipSuccess) {                                                                      \
         fprintf(stderr, "nfft4gp_amd: HIP error %s at %s:%d (%s)\n", hipGetErrorString(_e),      \
                 __FILE__, __LINE__, #expr);                                                       \
         return -1;                                                                                \
      }                                                                                            \
   } while (0)

// ---- host math (window.cpp) --------------------------------------------------------------------
double kb_phi(double t);         // NFFT3 Kaiser-Bessel PHI in grid units
double kb_phi_hut(int k);        // NFFT3 PHI_HUT
// tap polynomial coefficients C[t*kNC + d] (monomials in u = frac - 1/2)
const std::vector<double>& tap_poly_coeffs();
// fastsum kernel Fourier coefficients for a 1-D component, k = -N/2..N/2-1 (index k+N/2)
// kind: 0 gaussian, 1 xx_gaussian, 2 laplacian_rbf, 3 der_laplacian_rbf
void bhat_1d(int kind, double c, double* bhat);
// real circulant first column: w[s] = weight * sum_k bhat_k / phihut_k^2 cos(2 pi k s / n_os)
void circulant_1d(const double* bhat, double weight, double* w);

// ---- layout (layout.cpp) -----------------------------------------------------------------------
// element index of word w (of nwords per lane) of `lane` in tile t: [t][w/4][lane][w%4]
__host__ __device__ inline size_t quad_index(long long t, int w, int lane, int nwords)
{
   return (((size_t)t * (size_t)(nwords / 4) + (size_t)(w >> 2)) * kWave + (size_t)lane) * 4 + (size_t)(w & 3);
}

// std::allocator that leaves trivially constructible elements uninitialised (resize / construction without
// a value): the layout arrays (3.6 GB at config E) are written in full by their builder, zero-filling them
// first cost ~1 s
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
   template <class U>
   struct rebind {
      using other = DefaultInitAlloc<U>;
   };
   DefaultInitAlloc() = default;
   template <class U>
   DefaultInitAlloc(const DefaultInitAlloc<U>&) noexcept {}
   template <class U>
   void construct(U* p) noexcept
   {
      ::new ((void*)p) U;
   }
   template <class U, class... A>
   void construct(U* p, A&&... a)
   {
      ::new ((void*)p) U(std::forward<A>(a)...);
   }
};
template <class T>
using RawVec = std::vector<T, DefaultInitAlloc<T>>;

// the q word of a (point, window) slot (layout.cpp): the offset in the cell in 2^-32 units of a cell, e = 64 frac,
// moved to the nearest value congruent to the low 4 bits of the local index mod 16 (so |move| <= 8, an eighth of
// the 2^-26 quantum), bit 31 flipped so that (int32)q = 2^32 (u = offset - 1/2).  The other 8 index bits are the
// slot's lo byte (lo_byte).
__host__ __device__ inline uint32_t slot_word(uint32_t loc, uint32_t frac)
{
   const uint32_t lo4 = loc & 15u, e = (frac & 0x3FFFFFFu) << 6;
   return ((lo4 >= 8u && e != 0u) ? e - 16u + lo4 : e + lo4) ^ 0x80000000u;
}
__host__ __device__ inline uint32_t lo_byte(uint32_t loc) { return (loc >> 4) & 255u; }
// The 4-byte record of the 32-bit precision mode (Nfft4GPAmdSetPrecision(h, 32), the analogue of the reference's
// NFFT4GP_USING_FLOAT32, SRC/utils/utils.h:28-31): ONE word per (point, window) holding the whole 12-bit local
// index in its low bits -- the offset in the cell is e moved to the nearest value congruent to loc mod 4096, so
// |move| <= 2048 units of 2^-32 of a cell (2^-21 of a cell, 2^-27 of the period: finer than an fp32 coordinate)
__host__ __device__ inline uint32_t slot_word4(uint32_t loc, uint32_t frac)
{
   const uint32_t e = (frac & 0x3FFFFFFu) << 6, L = loc & 4095u;
   const uint32_t v = (e & ~4095u) | L;  // the candidate in e's 4096-unit window; e's low 6 bits are zero
   const int32_t dv = (int32_t)(v - e);  // in (-4096, 4096)
   const uint32_t down = (dv > 2048 && v >= 4096u) ? 4096u : 0u;
   const uint32_t up = (dv < -2048 && v <= 0xFFFFEFFFu) ? 4096u : 0u;
   return (v - down + up) ^ 0x80000000u;
}

struct Layout {
   int n = 0;           // local points
   int nw = 0;          // components
   int B = kMaxBlock;   // block size (points)
   int CG = 8;          // components per spread group
   int rec = 5;         // bytes per (point, window): 5 (slot_word + lo byte) or 4 (slot_word4, no lo array)
   int ngroups = 0;
   int nblocks = 0;
   long long ntiles = 0;
   RawVec<uint16_t> meta;          // [ntiles*64]      comp<<6 | cell
   RawVec<uint32_t> lo;            // [ntiles*R/4*64]  local index bits 4-11, one byte per point
   RawVec<uint32_t> q;             // [ntiles*R*64]    slot_word: offset in the cell, index bits 0-3 below it
   std::vector<int> tile_off;      // [nblocks*ngroups+1]
   std::vector<int> cmax;          // [nblocks*ngroups] the most points any one (window, cell) of (b, g) holds
};
// build from per-component quantized coordinates qc[c*n + j]
void build_layout(const uint32_t* qc, int n, int nw, int B, int CG, Layout& L, int rec = 5);
struct AdditivePlan;
// the same layout from device-resident coordinates into P.dl / P.ngroups / P.nblocks (layout_gpu.hip); -1
// when a (block, group) exceeds the emit kernel's LDS
int build_layout_dev(const uint32_t* d_qc, int n, int nw, int B, int CG, AdditivePlan& P, hipStream_t s, int rec = 5);

// ---- device plan --------------------------------------------------------------------------------
struct DevLayout {
   uint16_t* meta = nullptr;
   uint32_t* lo = nullptr;
   uint32_t* q = nullptr;
   int* tile_off = nullptr;
   int* cmax = nullptr;  // [nblocks*ngroups] the most points of one (window, cell) of each (block, group)
   long long ntiles = 0;
   size_t bytes = 0;
};

// multi-dimensional windows (nfft_md.hip): per-component 64^d grids, dims <= kMdMaxDim
constexpr int kMdMaxDim = 5;     // up to 5-feature windows: 64^5 grids (8.6 GB each, ~77 GB of buffers per
                                 // 5-feature window), the untiled spread / interp from 4 features on
constexpr int kMdTiledMaxDim = 3;  // the tiled kernels' LDS footprint (17^d doubles) fits up to 3 features
struct MdComp {
   int d = 0;
   int hicount = 1;          // kTaps^(d-1): tap rows per point
   long long u_off = 0;      // this component's first entry in u ([point][d]); psi starts at u_off * kTaps
};
struct MdPlan {
   bool on = false;
   bool gfix_per_window = false;  // d_gfix holds one window's fixed-point grid (nfft_md.hip md_spread)
   int maxd = 1;
   long long G = 0;          // 64^maxd: real grid stride per component
   long long Cmax = 0;       // 32 * 64^(maxd-1): complex pass buffer stride per component
   long long M = 0;          // 32^maxd: mode stride per component
   std::vector<MdComp> comps;
   MdComp* d_comps = nullptr;
   int* d_u = nullptr;       // [comp][point][d]  floor(64 x) - m
   double* d_psi = nullptr;  // [comp][point][d][kTaps]  PHI taps (PRE_PSI)
   double* d_grid = nullptr; // [nw][G] spread grid
   double2* d_F[2] = {nullptr, nullptr};  // forward ping-pong [nw][Cmax]
   double2* d_Mo[2] = {nullptr, nullptr}; // modes x bhat (chain 0: K, chain 1: K') [nw][M]
   double2* d_B[4] = {nullptr, nullptr, nullptr, nullptr};  // backward ping-pong, 2 per chain; chain 0's
                                                            // two alias d_F (free once the modes are formed)
   double* d_h[2] = {nullptr, nullptr};   // interpolation grids [nw][G]
   double* d_bh = nullptr;   // [nw][M]  weight * bhat * prod 1/phihut (second deconvolution)
   double* d_bhd = nullptr;  // [nw][M]  the same for the derivative kernel, times dscale
   double* d_dot_part = nullptr;
   unsigned int* d_dot_ticket = nullptr;
   // tiled spread: each component's points sorted by the 8^d tile of their first tap cell; work items
   // (component, tile, first, end) of at most a few thousand points, each summed in LDS then added to the grid
   int* d_perm = nullptr;    // [comp][n] local point indices in tile order
   int4* d_items = nullptr;  // {comp, tile, first, end} (first/end index the component's d_perm)
   int nitems = 0;
   bool lines = false;       // spread by k_md_spread_lines (all windows 3-D, n >= 4e5; NFFT4GP_AMD_MD_SPREAD overrides)
   double* d_part = nullptr; // tiled interpolation: [2][comp][n] per-component values (K, then K')
   // the spread adds in 128-bit fixed point (exact, so the grid does not depend on the order of the atomics):
   // d_gfix [nw][G][lo, hi] 64-bit pairs, d_xmax the bits of max |x| of the launch, psi_max the largest tap
   unsigned long long* d_gfix = nullptr;
   unsigned long long* d_xmax = nullptr;
   double psi_max = 0.0;
};

struct AdditivePlan {
   // geometry
   int n_global = 0, row_begin = 0, row_end = 0, n = 0;  // n = local rows
   int nw = 0, dw = 0, skip_last = 0;
   std::vector<int> comp_dims;
   // per-component cached first-setup state (nfft_interface.c:150-213)
   bool points_ready = false;
   std::vector<double> comp_scale;
   std::vector<double> comp_sigma;
   int kernel = 0;  // 0 gaussian, 1 matern12
   double f = 1.0, l = 1.0, mu = 0.0;
   double weight = 1.0;  // 1/nwindows (1/nwindows of the whole operator on a component shard)
   double diag = 1.0;    // 1: this handle adds the mu x (and grad f^2 x) terms; 0: a component shard without them
   // layout
   int B = kMaxBlock, CG = 3, ngroups = 0, nblocks = 0;  // CG = 3: 3 spread workgroups fit a CU's LDS
   int rec = 5;  // layout record: 5 bytes per (point, window) (fp64 default) or 4 (Nfft4GPAmdSetPrecision 32)
   // -1 (auto): 0 or 3 by the layout's size; 0: the spread; 1: the same with timeline stamps; 2: round-4 moment
   // table (A/B); 3: the next tile loaded before the current one's moments
   int spread_variant = -1;
   // deterministic 1-D matvec: the spread's moment flushes and the interpolation's y adds are rounded to a grid on
   // which every sum is exact, so results do not depend on the order of the LDS atomics (Nfft4GPAmdSetDeterministic)
   bool det = false;
   double* d_hb = nullptr;  // [vector 0, 1][H, Hd][nw] bounds of the interpolation polynomials (k_grid, det)
   int nparts = 0;          // partial grids per window the spread writes (one per block)
   DevLayout dl;
   // device buffers
   double* d_part = nullptr;  // [nblocks][nw][64]
   double* d_w = nullptr;     // [nw][64] circulant, kernel
   double* d_wd = nullptr;    // [nw][64] circulant, derivative kernel
   double* d_H = nullptr;     // [nw][64][kNC]
   double* d_Hd = nullptr;
   double* d_C = nullptr;     // [kTaps][kNC]
   double* d_dot_part = nullptr;         // [nblocks] fused matvec-dot partials
   unsigned int* d_dot_ticket = nullptr; // arrival counters (reduce.hpp)
   double* d_part2 = nullptr; // two-vector matvec: both vectors' partial grids [2][nblocks][nw][64]
   double* d_gsum = nullptr;  // the spread's grids summed by global atomics [nw][64] (launch_spread_grid), zero between
                              // matvecs (k_grid clears what it read)
   double* d_H2 = nullptr;    // [2][nw][64][kNC]
   double* d_xs = nullptr;    // staging (host pointer calls)
   double* d_ys = nullptr;    // staging 3n
   MdPlan md;  // used instead of the 1-D layout when any window has more than one feature
   // timing (Nfft4GPAmdTimingEnable): while on, plan_apply_dev points kev at 6 events and the launchers
   // attach them to the spread / grid / interp dispatches themselves (hipExtLaunchKernelGGL start and stop
   // events = the dispatch packet's begin / end timestamps, the quantity rocprofv3's kernel trace reports)
   bool timing = false;
   hipEvent_t* kev = nullptr;
   double ms[3] = {0, 0, 0};
   long long cnt[3] = {0, 0, 0};
};

// copy the tap polynomial table into constant memory of the current device
int upload_tap_coeffs();
// launchers (nfft_kernels.hip); all enqueue on `stream`
int launch_spread(const AdditivePlan& P, const double* d_x, double* d_part, hipStream_t stream);
int launch_grid(const AdditivePlan& P, const double* d_part, int nparts, int grad, hipStream_t stream);
// a whole handle's spread and grid step: the spread's partial grids summed by k_grid in a fixed order, or (not
// deterministic, few blocks) added by the spread itself into P.d_gsum with global atomics, which k_grid reads and clears
int launch_spread_grid(AdditivePlan& P, const double* d_x, int grad, hipStream_t stream);
int launch_grid_from_sum(const AdditivePlan& P, const double* d_gridsum, int grad, hipStream_t stream);
// the peer-memory exchange of the row split (dist.hip, Nfft4GPAmdDistPeerEnable): every rank's buffer holds
// two grid slots (epoch parity) of slot_doubles entries, each entry two 64-bit words carrying the epoch
// (nfft_kernels.hip).  A rank writes its grids into its own slot; every rank waits until all ranks' entries
// carry the epoch (bounded: `spin` polls, then *err = 1 and the wait gives up) and sums them in rank order, so
// every rank holds the same bits.
constexpr int kPeerInline = 8;  // ranks whose buffer pointers travel in the kernel arguments
struct PeerArgs {
   char* const* bufs = nullptr;  // device array: the ranks' exchange buffers, rank order (own included)
   char* inl[kPeerInline] = {};  // the first kPeerInline of them (scalar loads, no dependent global load)
   char* own = nullptr;          // this rank's buffer
   int world = 0;
   unsigned int epoch = 0;
   unsigned int* err = nullptr;  // device view of the host-mapped error word
   long long slot_doubles = 0;
   long long spin = 0;
};
// gsum = the grids of this shard; with A: into this rank's slot of A.epoch, then the windows' flags published
int launch_reduce_parts(const AdditivePlan& P, const double* d_part, double* d_gridsum, hipStream_t stream,
                        const PeerArgs* A = nullptr);
// row shards with few blocks: grid from the summed grids + y = beta y + alpha f^2 mu x, then the interpolation
// with S workgroups per block adding into y atomically (plain matvec); with A the summed grids come from the
// ranks' slots (the wait overlaps the y initialisation)
// (A and d_part: this rank's partial grids are summed and put into its slot in the same kernel)
int launch_shard_finish_split(const AdditivePlan& P, const double* d_gridsum, double alpha, const double* d_x,
                              double beta, double* d_y, int S, hipStream_t stream, const PeerArgs* A = nullptr,
                              const double* d_part = nullptr);
// d_grid = the rank-order sum of the ranks' slots of A.epoch (after waiting for their flags)
int launch_peer_grid(const AdditivePlan& P, const PeerArgs& A, const double* d_part, hipStream_t stream);
int launch_peer_sum(const AdditivePlan& P, const PeerArgs& A, double* d_grid, hipStream_t stream);
// d_dot != nullptr (non-grad): also writes (y, x) to *d_dot (device), one grid-wide reduction in the launch
int launch_interp(const AdditivePlan& P, int grad, double alpha, const double* d_x, double beta, double* d_y,
                  hipStream_t stream, double* d_dot = nullptr);
// the interpolation of blocks [b0, b1) (plain matvec, no gradient / dot)
int launch_interp_blocks(const AdditivePlan& P, double alpha, const double* d_x, double beta, double* d_y, int b0,
                         int b1, hipStream_t stream);
// y_v = beta y_v + alpha A x_v, v = 0, 1, in one pass over the layout (1-D layouts; -1 for multi-feature windows)
int launch_matvec2(AdditivePlan& P, double alpha, const double* x0, const double* x1, double beta, double* y0,
                   double* y1, hipStream_t stream);
// y_v = beta y_v + alpha A x_v for nv device vectors of this library's additive handle (pairs per layout pass)
int additive_matvec_multi(void* str, int nv, double alpha, const double* const* X, double beta, double* const* Y);
// y = A x (alpha = 1, beta = 0) and *d_dot = (y, x) on device pointers: the matvec + dot of a CG step in
// the matvec's own three launches (used by Nfft4GPSolverPcg when its operator is this library's)
int additive_matvec_dot(void* str, const double* d_x, double* d_y, double* d_dot);
// true when additive_matvec_dot can serve this handle: points set up, whole-row (not a row shard) handle,
// and a 1-D layout whose block count the fused grid reduction can sum (nblocks <= kRedMaxBlocks)
bool additive_fused_dot_ok(void* str);

// Nystrom preconditioner M = U S U^T + eta (I - U U^T) in HBM (nys.c:115-173 apply)
struct NysDev {
   int n = 0, k = 0;
   double eta = 0.0;
   double* U = nullptr;  // n x k column-major, natural row order
   float* Uf = nullptr;  // optional fp32 copy the apply reads instead (Nfft4GPAmdNysSetStorage)
   double* s = nullptr;  // k
   double* w = nullptr;  // apply scratch, k
   double* part = nullptr;
   int nblk = 0;
   // GPU setup only: hipEvent durations of the setup's kernels (ms): panel, U1 = Kp G^T, the Gram
   // U1^T U1 (+ split sum), U = U1 W (Nfft4GPAmdNysSetupTimes)
   double setup_ms[4] = {0.0, 0.0, 0.0, 0.0};
   std::vector<double> hs;  // s on the host (logdet)
   // setups with gradients (nys.c:518-660 with require_grad, for Dvp / Trace / Logdet, nys.c:175-516):
   // Kall = [K | dK/df | dK/dl] (n x 3k, natural row order), dU = K L^{-T} (n x k), G = L^{-1} and G^T,
   // GdKG = [L^{-1} dK11_f L^{-T} | L^{-1} dK11_l L^{-T}] (k x 2k), D = dU^T dU, scratch vk (8k), vn (n)
   bool grad = false;
   double f2 = 0.0;
   double *Kall = nullptr, *dU = nullptr, *G = nullptr, *Gt = nullptr, *GdKG = nullptr, *D = nullptr;
   double *vk = nullptr, *vn = nullptr;
};
void nys_free(NysDev* N);
constexpr int kNysRows = 2048;  // rows per workgroup of the apply's U^T r pass
int nys_alloc_scratch(NysDev* N);
// GPU Nystrom setup (nystrom.hip) from gathered window coordinates xw (n x packed dims, host)
int gemm_f64(bool transA, int M, int N, int K, const double* A, long long lda, const double* B, long long ldb,
             double* C, long long ldc, hipStream_t s);
int sym_eig_host(const std::vector<double>& A, int n, std::vector<double>& w, std::vector<double>& V);
int chol_inverse_host(std::vector<double>& A, int k);
struct Comm;
// a row shard of the Nystrom setup: this process holds rows [row_begin, row_begin + n) of n_global; the
// Gram is all-reduced over comm and rank 0's k x k factors are broadcast (dist.hip)
struct NysShard {
   Comm* comm = nullptr;
   int row_begin = 0, n_global = 0;
};
// xw_host: the gathered window buffer (n rows, or n_global with a shard); perm: at least k entries
NysDev* nys_setup_additive(const double* xw_host, int n, int nw, int dw, int skip_last, int kernel, double f,
                           double l, double mu, const int* perm, int k, int k11_mode, bool with_grad = false,
                           const NysShard* shard = nullptr);

// multi-dimensional windows (nfft_md.hip).  xs[c] = component c's centred, scaled coordinates
// (n_global x d column-major); the plan keeps rows [row_begin, row_end).
int md_build_points(AdditivePlan& P, const std::vector<std::vector<double>>& xs);
int md_setup(AdditivePlan& P);  // kernel coefficients for P.kernel, P.comp_sigma, P.comp_scale
int md_spread(const AdditivePlan& P, const double* d_x, double* d_grid, hipStream_t s);
int md_grid(const AdditivePlan& P, const double* d_grid, int grad, hipStream_t s);
int md_interp(const AdditivePlan& P, int grad, double alpha, const double* d_x, double beta, double* d_y,
              hipStream_t s, double* d_dot = nullptr);
void md_free(AdditivePlan& P);
void bhat_nd(int kind, int d, double c, std::vector<double>& bhat);  // window.cpp, 32^d real

// k x k lower Cholesky of A (+ shift I) and its inverse (rocSOLVER potrf/trtri, host fallback): G = L^{-1}
// (lower, cleaned; may be NULL), Gt = L^{-T}.  A is overwritten.  >0: not positive definite (nystrom.hip)
int chol_inverse_dev(double* A, int k, double shift, double* G, double* Gt, int* d_info, hipStream_t s);
// C (M x N) = A^T B, A K x M (lda), B K x N (ldb), split over K with a fixed-order sum (nystrom.hip)
int gram_tn(int M, int N, int K, const double* A, long long lda, const double* B, long long ldb, double* C, int sym,
            hipStream_t s);
// ascending eigenvalues of a symmetric device matrix (rocSOLVER dsyevd, no vectors; nystrom.hip)
int sym_eigvals_dev(double* A, int n, std::vector<double>& w, hipStream_t s);
// the kernel of a preconditioner setup: plain Gaussian / Matern-1/2 of the points' coordinates
// (Xk == NULL), or the dense additive kernel of the device coordinates Xk (column c of window w at
// c = w*dw + t, ld ldk; the last window has last_dw of them) -- kernel_eval.hpp
struct KernelSpec {
   int kernel = 0;
   double f = 1.0, l = 1.0, mu = 0.0;
   const double* Xk = nullptr;
   long long ldk = 0;
   int nw = 1, dw = 0, last_dw = 0;
};
// FSAI of a kernel matrix (fsai_setup.hip): KNN pattern on dX (n x d, ld ldim), values of the kernel
// K; host CSR out; dW (kw x n): the Schur-complement kernel K - W'W
// With require_grad and dW: dGB (2 kw x n panels L11^{-1} dK12_g) and dGC (3 panels GdK11G_g W) give the
// Schur kernel's gradients (fsai_setup.hip k_fsai_rows)
// keep (no gradients): the CSR stays on the device (keep[0] = ia, keep[1] = ja, keep[2] = aa, owned by the caller);
// only ia comes back to the host then
int fsai_kernel_csr(const double* dX, int n, int ldim, int d, int lfil, const KernelSpec& K, const double* dW, int kw,
                    int require_grad, std::vector<int>& ia, std::vector<int>& ja, std::vector<double>& aa,
                    std::vector<double>& da, hipStream_t s, const double* dGB = nullptr,
                    const double* dGC = nullptr, void** keep = nullptr);
// an Nfft4GPAmdFsaiCreate handle from a CSR already in HBM (fsai_afn.hip): takes ownership of dia / dja / daa; hia
// is the host copy of dia; L^T is formed on the device.  NULL on error (the arrays are freed then)
void* fsai_create_from_device(int n, int* dia, int* dja, double* daa, const std::vector<int>& hia, hipStream_t s);
// the number of non-finite values among count doubles (device)
long long count_nonfinite(const double* d, size_t count, hipStream_t s);
// a row shard's rows of the FSAI (fsai_setup.hip): the pattern of the listed rows (ascending) -- KNN over their
// earlier points only -- and the values of a range of pattern rows, W's column of each entry from dwcol
int fsai_pattern_rows(const double* dX, int n, int ldim, int d, int lfil, const std::vector<int>& rows,
                      std::vector<int>& hia, std::vector<int>& hja, hipStream_t s);
int fsai_values_rows(const KernelSpec& Ks, const double* dX, long long ldim, int d, int lfil, const int* dia,
                     const int* dja, int nrows, const double* dW, int kw, const int* dwcol, double* daa, hipStream_t s);
// a row shard of the AFN apply from one rank's sharded setup (fsai_afn.hip; takes d_Linv, d_LinvT, d_K12)
void* afn_shard_from_parts(int n_local, int k, int n2, Comm* comm, const std::vector<int>& lm_idx,
                           const std::vector<int>& lm_row, const std::vector<int>& nl_pos,
                           const std::vector<int>& nl_row, double* d_Linv, double* d_LinvT, double* d_K12, bool fsai,
                           double schur_scale, const std::vector<int>& gia, const std::vector<int>& gja,
                           const std::vector<double>& gaa);
// the Schur FSAI with gradients as operators (fsai_setup.hip): create from host CSR (+ 3 nnz gradients)
void* fsai_grad_create(int n, const int* ia, const int* ja, const double* aa, const double* da);
void fsai_grad_free(void* F);
// y = G x, G^T x, G^{-1} x, G^{-T} x, dG_g x, dG_g^T x for op = 0..5
int fsai_grad_op(void* F, int op, int g, const double* x, double* y, hipStream_t s);
// sum_i dG_g(i,i) / G(i,i) (g >= 0) or sum_i log(1 / G(i,i)) (g < 0)
double fsai_grad_diag(void* F, int g, hipStream_t s);
// lower Cholesky factor of A (k x k, in place, upper triangle zeroed; rocSOLVER potrf, host fallback);
// returns 0, the failing column + 1, or -1 (nystrom.hip)
int chol_factor_dev(double* A, int k, int* d_info, hipStream_t s);
// the KernelSpec of fkernel_params (this library's additive handle: its window buffer, uploaded to
// *owned; else the plain kernel); 1 additive, 0 plain, -1 error (fsai_setup.hip)
int kernel_spec_of(void* fkernel_params, func_kernel fkernel, int kernel, int n, KernelSpec& K, double** owned);
// The AFN's gradient pieces (MATLAB afn_setup.m with require_grad; afn_dvp.m, afn_trace.m, afn_logdet.m):
// the factors of the apply plus dL_g = L Phi(L^{-1} dK11_g L^{-T}), dK12_g and the Schur FSAI's dG_g
struct AfnGrad {
   int n = 0, k = 0, n2 = 0;
   int* perm = nullptr;                 // device, n
   double *L = nullptr, *Linv = nullptr, *LinvT = nullptr;  // k x k
   double* dL = nullptr;                // 3 k x k (g = f, l, mu)
   const double* K12 = nullptr;         // k x n2, the apply object's
   double* dK12 = nullptr;              // 2 k x n2 (g = f, l; dK12_mu = 0)
   void* S = nullptr;                   // fsai_grad_create handle of the Schur FSAI (n2)
   void* afn = nullptr;                 // the apply (M^{-1}), not owned
   double trace[3] = {0.0, 0.0, 0.0};   // tr(M^{-1} dM/dtheta_g)
   double logdet = 0.0;                 // log det M
   double* work = nullptr;              // 6 n + 8 k scratch
};
void afn_grad_free(AfnGrad* G);
// y_g = M^{-1} (dM/dtheta_g) x for the gradients in mask (all three when NULL), device vectors, y: 3n
int afn_grad_dvp(AfnGrad* G, const int* mask, const double* x, double* y, hipStream_t s);

// AFN apply object from device factors (fsai_afn.hip); owns all of them and S
// S == NULL with n - k > 0: the Schur complement solve is schur_scale * I (schur_opt 0)
void* afn_create_device(int n, int k, int* d_perm, double* d_Linv, double* d_LinvT, double* d_K12, void* S,
                        double schur_scale = 0.0);

hipStream_t current_stream();
bool is_device_ptr(const void* p);
int device_ok();

// ---- libc rand() of the reference (nfft_api.cpp) --------------------------------------------------
// The reference draws libc rand() (Nfft4GPRandPerm, Nfft4GPVecRand, rankest.c), so after the same srand()
// both libraries see the same numbers -- unless something else in the call draws too: the ROCm libraries
// do while they initialise.  An entry point that draws opens a RandScope: the process runs on a private
// random() state for the duration of the call, and each batch of the reference's draws runs inside a
// CallerRandBatch on the caller's state (glibc rand() is random(); initstate / setstate switch its state).
// A scope holds a process-wide recursive lock, so scopes of several host threads do not interleave; a thread
// that calls libc rand() while another thread's library call holds a scope draws from the private state
// (do not call rand() concurrently with this library's setup entry points).  The apply paths (MatSymv,
// GradMatSymv) open no scope.
struct RandScope {
   RandScope();
   ~RandScope();
};
struct CallerRandBatch {
   char* prev = nullptr;
   CallerRandBatch();
   ~CallerRandBatch();
};

// ---- multi-GPU (dist.hip) -----------------------------------------------------------------------
// a process group: in-place sum of count device doubles over the ranks, ordered on stream s
struct Comm {
   int rank = 0, world = 1;
   virtual ~Comm() {}
   virtual int allreduce(double* d_buf, size_t count, hipStream_t s) = 0;
   // the number of ranks the backend itself reports (RCCL: ncclCommCount)
   virtual int ranks() { return world; }
};
// additive handle rows (nfft_api.cpp): local, global, first row; -1 if not an additive handle
int additive_rows(void* str, int* n_local, int* n_global, int* row_begin);
// 1 when a peer exchange of the distributed operator dop timed out (dist.hip; read after a host sync)
int dist_failed(void* dop);
bool shard_fused_dot_ok(void* str);
// row shard: grid (summed over the shards) -> y_local = A x_local and *d_dot = (y_local, x_local) locally
int shard_finish_dot(void* str, const double* grid, const double* x_local, double* y_local, double* d_dot);
// the row split over the peer exchange (1-D windows only: shard_peer_ok): the spread into the partial grids;
// then their sum, the put into this rank's slot, the exchange, the grid and y-init in one kernel (few-block
// shards), or k_reduce_parts + k_peer_sum into d_grid before the usual finish (gradient, dot, many blocks)
bool shard_peer_ok(void* str);
int shard_spread_peer(void* str, const double* x_local, const PeerArgs& A);
int shard_peer_sum(void* str, const PeerArgs& A, double* d_grid);
int shard_finish_dot_peer(void* str, const PeerArgs& A, double* d_grid, const double* x_local, double* y_local,
                          double* d_dot);
int shard_finish_peer(void* str, const PeerArgs& A, double* d_grid, int grad, double alpha, const double* x_local,
                      double beta, double* y_local);
// what Nfft4GPSolverPcg needs to know about a distributed operator (matvec == Nfft4GPAmdDistMatSymv):
// the communicator its dot products are summed over (NULL when the vectors are replicated), the global
// n, and whether q = A p can also form the local (q, p) in its interpolation launch
struct DistPcgInfo {
   Comm* dot_comm = nullptr;
   int n_global = 0;
   int row_begin = 0;  // this rank's first row (0 for replicated vectors)
   bool fused_dot = false;
};
int dist_pcg_info(void* dop, DistPcgInfo& info);
NysDev* nys_setup_shard(void* str, const int* perm, int k, int k11_mode, Comm* comm);  // nfft_api.cpp
// y = alpha A x (beta = 0) of a whole-row 1-D handle with its interpolation split into nchunks launches of
// consecutive blocks; after each, done(r0, r1) is called with the rows that launch wrote (enqueued work
// only, on the current stream).  -1: not a 1-D whole-row handle (the caller runs the plain matvec)
int additive_matvec_chunked(void* str, double alpha, const double* d_x, double* d_y, int nchunks,
                            int (*done)(void* ctx, size_t r0, size_t r1), void* ctx);
// q = A p with the local (q, p) in *d_dot (row shards; the caller all-reduces it)
int dist_matvec_dot(void* dop, const double* d_p, double* d_q, double* d_dot);

}  // namespace nfft4gp_amd
