// nfft_api.cpp -- C ABI of the NFFT additive-kernel operator (drop-in for nfft_interface.c).
//
// Handle model (mirrors nfft_interface.c:3-42, :622-674): a nfft4gp_kernel struct with the
// reference's exact field layout; _iparams[0..2] = nwindows, dwindows, skip_last; _buffer = the
// gathered window columns (host); _dwork = 3n host doubles as in the reference; _external = our
// device plan.  Hyperparameters are read from _params / _noise_level at setup time and cached,
// as the reference caches them in str_adj (nfft_interface.c:219-256).
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <array>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "internal.h"
#include "reduce.hpp"

using namespace nfft4gp_amd;

namespace nfft4gp_amd {

namespace {
// the scope holds this lock for its lifetime: the depth, the saved caller state and the process-wide
// glibc random() state are switched by one host thread at a time (other threads' library calls that
// open a scope wait; libc rand() itself stays unsafe to call concurrently with a scope, see internal.h)
std::recursive_mutex g_rand_mu;
int g_rand_depth = 0;
char* g_caller_rand = nullptr;
char g_private_rand[256];
bool g_private_ready = false;
}  // namespace

// the private state is seeded once and then switched in with setstate (O(1)), so every entry point can
// open a scope
RandScope::RandScope()
{
   g_rand_mu.lock();
   if (g_rand_depth++ == 0) {
      if (!g_private_ready) {
         g_caller_rand = initstate(20240807u, g_private_rand, sizeof(g_private_rand));
         g_private_ready = true;
      } else {
         g_caller_rand = setstate(g_private_rand);
      }
   }
}

RandScope::~RandScope()
{
   if (--g_rand_depth == 0) {
      setstate(g_caller_rand);
      g_caller_rand = nullptr;
   }
   g_rand_mu.unlock();
}

CallerRandBatch::CallerRandBatch()
{
   if (g_rand_depth > 0) prev = setstate(g_caller_rand);
}

CallerRandBatch::~CallerRandBatch()
{
   if (prev) g_caller_rand = setstate(prev);
}

static hipStream_t g_stream = nullptr;

hipStream_t current_stream() { return g_stream; }

int device_ok()
{
   // a positive answer is cached; a negative one is re-queried (and explained) on every call
   static int ok = 0;
   if (!ok) {
      int cnt = 0;
      const hipError_t e = hipGetDeviceCount(&cnt);
      if (e != hipSuccess) {
         fprintf(stderr, "nfft4gp_amd: hipGetDeviceCount failed: %s\n", hipGetErrorString(e));
         cnt = 0;
      }
      (void)hipGetLastError();
      ok = cnt > 0 ? 1 : 0;
   }
   return ok;
}

bool is_device_ptr(const void* p)
{
   if (!p) return false;
   hipPointerAttribute_t attr;
   hipError_t e = hipPointerGetAttributes(&attr, p);
   if (e != hipSuccess) {
      (void)hipGetLastError();
      return false;
   }
   return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

}  // namespace nfft4gp_amd

namespace {

struct TimingRec {
   std::array<hipEvent_t, 6> ev;  // start / stop of the spread, grid and interp dispatches
};

struct PlanExt {
   AdditivePlan P;
   std::vector<TimingRec> pending;
   std::vector<TimingRec> pool;
};

// single-component handle (the reference's str_adj): *Kp of the single-component setup points here.  The
// public str_adj comes first, so a caller that casts *Kp to str_adj* (INC/_external.h:28-51) reads the
// reference's cached scalars.
struct SingleAdj {
   str_adj pub{};
   double sigma_pub = 0.0;  // pub._sigma points here
   nfft4gp_kernel* owner = nullptr;
   int dim = 1;
   int max_n = 0;
   std::vector<double> data;  // first-setup copy of the points (n x dim, column-major)
   PlanExt* plan = nullptr;
};

void dfree(void* p)
{
   if (p) (void)hipFree(p);
}

void free_layout(AdditivePlan& P)
{
   dfree(P.dl.meta);
   dfree(P.dl.lo);
   dfree(P.dl.q);
   dfree(P.dl.tile_off);
   dfree(P.dl.cmax);
   P.dl = DevLayout();
   dfree(P.d_part);
   dfree(P.d_part2);
   dfree(P.d_H2);
   dfree(P.d_dot_part);
   dfree(P.d_dot_ticket);
   P.d_part2 = P.d_H2 = nullptr;
   P.d_part = nullptr;
   P.d_dot_part = nullptr;
   P.d_dot_ticket = nullptr;
}

void free_plan(PlanExt* E)
{
   if (!E) return;
   AdditivePlan& P = E->P;
   free_layout(P);
   md_free(P);
   dfree(P.d_w);
   dfree(P.d_wd);
   dfree(P.d_H);
   dfree(P.d_Hd);
   dfree(P.d_hb);
   dfree(P.d_gsum);
   dfree(P.d_C);
   dfree(P.d_xs);
   dfree(P.d_ys);
   for (auto& r : E->pending)
      for (auto e : r.ev) (void)hipEventDestroy(e);
   for (auto& r : E->pool)
      for (auto e : r.ev) (void)hipEventDestroy(e);
   delete E;
}

template <class T, class A>
int upload(T** dptr, const std::vector<T, A>& h)
{
   if (*dptr) {
      (void)hipFree(*dptr);
      *dptr = nullptr;
   }
   if (h.empty()) return 0;
   NFFT4GP_HIP_CHECK(hipMalloc((void**)dptr, sizeof(T) * h.size()));
   NFFT4GP_HIP_CHECK(hipMemcpy(*dptr, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
   return 0;
}

// nfft_interface.c:150-213: centre by the mean, scale to radius 0.25 unless already in
// [0.125, 0.25], computed once from all n_global points (same operation order as the reference).
double centre_and_scale(const double* col, int n_global, int d, std::vector<double>& xs)
{
   xs.assign(col, col + (size_t)n_global * d);
   for (int i = 0; i < d; i++) {
      double c = 0.0;
      for (int j = 0; j < n_global; j++) c += xs[(size_t)i * n_global + j];
      c /= (double)n_global;
      for (int j = 0; j < n_global; j++) xs[(size_t)i * n_global + j] -= c;
   }
   double radius = 0.0;
   for (int j = 0; j < n_global; j++) {
      double r = 0.0;
      for (int i = 0; i < d; i++) r += xs[(size_t)i * n_global + j] * xs[(size_t)i * n_global + j];
      r = std::sqrt(r);
      if (r > radius) radius = r;
   }
   double scale;
   if (radius == 0.0) return -1.0;  // all points coincide: the reference divides by zero (:190)
   if (radius > 0.25 || radius < 0.125) {
      scale = 0.25 / radius;
      for (auto& v : xs) v *= scale;
   } else {
      scale = 1.0;
   }
   return scale;
}

uint32_t quantize(double x)
{
   // x in [-0.5, 0.5): 32-bit fixed point of x mod 1 (exact power-of-two scaling, one rounding)
   const long long v = std::llround(x * 4294967296.0);
   return (uint32_t)(unsigned long long)v;
}

// first setup: nodes -> layout on the device
int plan_build_points(AdditivePlan& P, const double* buffer)
{
   const int ng = P.n_global;
   RawVec<uint32_t> qc((size_t)P.nw * P.n);  // every entry is written below
   P.comp_scale.assign(P.nw, 1.0);
   std::vector<double> xs;
   if (std::any_of(P.comp_dims.begin(), P.comp_dims.end(), [](int d) { return d != 1; })) {
      // windows of several features: 64^d grids (nfft_md.hip)
      std::vector<std::vector<double>> xsc(P.nw);
      for (int c = 0; c < P.nw; c++) {
         const double* col = buffer + (size_t)c * ng * P.dw;  // nfft_interface.c:703 stride n*dwindows
         P.comp_scale[c] = centre_and_scale(col, ng, P.comp_dims[c], xsc[c]);
         if (P.comp_scale[c] < 0.0) {
            fprintf(stderr, "nfft4gp_amd: all points of window %d coincide (radius 0); the reference's scaling "
                            "0.25/radius (nfft_interface.c:190) is undefined there.\n", c);
            return -1;
         }
      }
      if (md_build_points(P, xsc)) return -1;
      P.points_ready = true;
      return 0;
   }
   // windows are independent: one host thread per window at a time (centre, scale, quantize)
   const auto t0 = std::chrono::steady_clock::now();
   std::atomic<int> next{0};
   auto work = [&]() {
      std::vector<double> xw;
      for (int c = next++; c < P.nw; c = next++) {
         const double* col = buffer + (size_t)c * ng * P.dw;  // nfft_interface.c:703 stride n*dwindows
         P.comp_scale[c] = centre_and_scale(col, ng, 1, xw);
         if (P.comp_scale[c] < 0.0) continue;
         for (int j = 0; j < P.n; j++) qc[(size_t)c * P.n + j] = quantize(xw[(size_t)P.row_begin + j]);
      }
   };
   {
      const int nt = std::max(1, std::min({16, P.nw, (int)std::thread::hardware_concurrency()}));
      std::vector<std::thread> th;
      for (int t = 1; t < nt; t++) th.emplace_back(work);
      work();
      for (auto& t : th) t.join();
   }
   for (int c = 0; c < P.nw; c++)
      if (P.comp_scale[c] < 0.0) {
         fprintf(stderr,
                 "nfft4gp_amd: all points of window %d coincide (radius 0); the reference's scaling "
                 "0.25/radius (nfft_interface.c:190) is undefined there.\n", c);
         return -1;
      }
   const auto t1 = std::chrono::steady_clock::now();
   // the layout is built on the GPU from the quantised coordinates (layout_gpu.hip); layout.cpp builds the
   // same arrays on the host when a (block, group) would not fit the GPU builder's LDS (B > 4064, or CG > 4
   // would need it; neither is a setting the plan uses)
   free_layout(P);
   hipStream_t s = current_stream();
   uint32_t* d_qc = nullptr;
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&d_qc, sizeof(uint32_t) * std::max<size_t>(1, qc.size())));
   NFFT4GP_HIP_CHECK(hipMemcpyAsync(d_qc, qc.data(), sizeof(uint32_t) * qc.size(), hipMemcpyHostToDevice, s));
   const auto t2 = std::chrono::steady_clock::now();
   const int rc_dev = build_layout_dev(d_qc, P.n, P.nw, P.B, P.CG, P, s, P.rec);
   (void)hipStreamSynchronize(s);
   (void)hipFree(d_qc);
   if (rc_dev) {
      Layout L;
      build_layout(qc.data(), P.n, P.nw, P.B, P.CG, L, P.rec);
      P.ngroups = L.ngroups;
      P.nblocks = L.nblocks;
      free_layout(P);
      if (upload(&P.dl.meta, L.meta) || upload(&P.dl.lo, L.lo) || upload(&P.dl.q, L.q) ||
          upload(&P.dl.tile_off, L.tile_off) || upload(&P.dl.cmax, L.cmax))
         return -1;
      P.dl.ntiles = L.ntiles;
      P.dl.bytes = L.meta.size() * 2 + L.lo.size() * 4 + L.q.size() * 4 + L.tile_off.size() * 4;
   }
   if (getenv("NFFT4GP_AMD_VERBOSE")) {
      const auto t3 = std::chrono::steady_clock::now();
      auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
      fprintf(stderr, "nfft4gp_amd: layout setup: centre/scale/quantize %.1f ms, coordinate upload %.1f ms, "
                      "layout (%s) %.1f ms\n", ms(t0, t1), ms(t1, t2), rc_dev ? "host" : "GPU", ms(t2, t3));
   }
   P.nparts = P.nblocks;
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&P.d_part, sizeof(double) * (size_t)std::max(1, P.nparts) * P.nw * kNos));

   dfree(P.d_dot_part);
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&P.d_dot_part, sizeof(double) * (size_t)std::max(1, P.nblocks)));
   if (!P.d_dot_ticket) {
      NFFT4GP_HIP_CHECK(hipMalloc((void**)&P.d_dot_ticket, sizeof(unsigned int) * kTicketWords));
      NFFT4GP_HIP_CHECK(hipMemset(P.d_dot_ticket, 0, sizeof(unsigned int) * kTicketWords));
   }

   if (!P.d_H) NFFT4GP_HIP_CHECK(hipMalloc((void**)&P.d_H, sizeof(double) * (size_t)P.nw * kNos * kNC));
   if (!P.d_Hd) NFFT4GP_HIP_CHECK(hipMalloc((void**)&P.d_Hd, sizeof(double) * (size_t)P.nw * kNos * kNC));
   if (!P.d_hb) NFFT4GP_HIP_CHECK(hipMalloc((void**)&P.d_hb, sizeof(double) * 4 * (size_t)std::max(1, P.nw)));
   if (upload_tap_coeffs()) return -1;
   P.points_ready = true;
   return 0;
}

// every setup: kernel coefficients (nfft_interface.c:216-256)
int plan_setup(AdditivePlan& P, const double* buffer, int kernel, double f, double l, double mu)
{
   if (!device_ok()) {
      fprintf(stderr, "nfft4gp_amd: no HIP device visible; the operator has no CPU fallback.\n");
      return -1;
   }
   if (!P.points_ready && plan_build_points(P, buffer)) return -1;
   P.kernel = kernel;
   P.f = f;
   P.l = l;
   P.mu = mu;
   P.comp_sigma.assign(P.nw, 0.0);
   if (P.md.on) {
      for (int c = 0; c < P.nw; c++)
         P.comp_sigma[c] = (kernel == 0) ? l * P.comp_scale[c] * std::sqrt(2.0) : l * P.comp_scale[c];  // :219/:355
      return md_setup(P);
   }
   std::vector<double> w((size_t)P.nw * kNos), wd((size_t)P.nw * kNos);
   double bh[kBand], bhd[kBand];
   for (int c = 0; c < P.nw; c++) {
      const double sc = P.comp_scale[c];
      const double sig = (kernel == 0) ? l * sc * std::sqrt(2.0) : l * sc;  // :219 / :355
      P.comp_sigma[c] = sig;
      bhat_1d(kernel == 0 ? 0 : 2, sig, bh);
      bhat_1d(kernel == 0 ? 1 : 3, sig, bhd);
      const double dscale = (kernel == 0) ? 2.0 * sc * std::sqrt(2.0) / sig : sc / sig;  // :536
      circulant_1d(bh, P.weight, w.data() + (size_t)c * kNos);
      circulant_1d(bhd, P.weight * dscale, wd.data() + (size_t)c * kNos);
   }
   if (upload(&P.d_w, w) || upload(&P.d_wd, wd)) return -1;
   return 0;
}

TimingRec get_rec(PlanExt* E)
{
   if (!E->pool.empty()) {
      TimingRec r = E->pool.back();
      E->pool.pop_back();
      return r;
   }
   TimingRec r;
   for (auto& e : r.ev) (void)hipEventCreate(&e);
   return r;
}

// y = beta*y + alpha*(op) x  on device pointers
int plan_apply_dev(PlanExt* E, int grad, double alpha, const double* d_x, double beta, double* d_y)
{
   AdditivePlan& P = E->P;
   hipStream_t s = current_stream();
   TimingRec rec;
   if (P.timing) {
      rec = get_rec(E);
      if (!P.md.on) P.kev = rec.ev.data();  // 1-D launchers attach the events to the dispatches
   }
   const bool mdt = P.timing && P.md.on;  // multi-feature windows: events recorded around each launch
   int rc = 0;
   if (mdt) (void)hipEventRecord(rec.ev[0], s);
   if (P.md.on) {
      rc = md_spread(P, d_x, P.md.d_grid, s);
      if (mdt) {
         (void)hipEventRecord(rec.ev[1], s);
         (void)hipEventRecord(rec.ev[2], s);
      }
      if (!rc) rc = md_grid(P, P.md.d_grid, grad, s);
   } else {
      rc = launch_spread_grid(P, d_x, grad, s);
   }
   if (mdt) {
      (void)hipEventRecord(rec.ev[3], s);
      (void)hipEventRecord(rec.ev[4], s);
   }
   if (!rc)
      rc = P.md.on ? md_interp(P, grad, alpha, d_x, beta, d_y, s) : launch_interp(P, grad, alpha, d_x, beta, d_y, s);
   if (mdt) (void)hipEventRecord(rec.ev[5], s);
   P.kev = nullptr;
   if (P.timing) {
      if (rc)
         E->pool.push_back(rec);
      else
         E->pending.push_back(rec);
   }
   return rc ? -1 : 0;
}

int plan_apply(PlanExt* E, int n, int grad, double alpha, const double* x, double beta, double* y)
{
   AdditivePlan& P = E->P;
   if (!P.points_ready) {
      fprintf(stderr, "nfft4gp_amd: matvec called before the kernel setup (func_kernel) call.\n");
      return -1;
   }
   if (n != P.n) {
      fprintf(stderr, "nfft4gp_amd: matvec size %d does not match the handle (%d).\n", n, P.n);
      return -1;
   }
   if (P.row_begin != 0 || P.row_end != P.n_global) {
      // a row shard holds only its rows' share of the grids: its operator is the split-phase pair
      // Nfft4GPAmdShardSpread -> (sum over shards) -> Nfft4GPAmdShardFinish, never a whole matvec
      fprintf(stderr, "nfft4gp_amd: rows [%d, %d) of %d form a row shard; use Nfft4GPAmdShardSpread/ShardFinish.\n",
              P.row_begin, P.row_end, P.n_global);
      return -1;
   }
   const size_t ny = (size_t)n * (grad ? 3 : 1);
   const bool dx = is_device_ptr(x), dy = is_device_ptr(y);
   if (dx && dy) return plan_apply_dev(E, grad, alpha, x, beta, y);
   // host staging (PCIe), synchronous
   hipStream_t s = current_stream();
   if (!P.d_xs) NFFT4GP_HIP_CHECK(hipMalloc((void**)&P.d_xs, sizeof(double) * (size_t)n));
   if (!P.d_ys) NFFT4GP_HIP_CHECK(hipMalloc((void**)&P.d_ys, sizeof(double) * (size_t)n * 3));
   const double* xd = x;
   double* yd = y;
   if (!dx) {
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(P.d_xs, x, sizeof(double) * n, hipMemcpyHostToDevice, s));
      xd = P.d_xs;
   }
   if (!dy) {
      yd = P.d_ys;
      if (beta != 0.0) NFFT4GP_HIP_CHECK(hipMemcpyAsync(yd, y, sizeof(double) * ny, hipMemcpyHostToDevice, s));
   }
   if (plan_apply_dev(E, grad, alpha, xd, beta, yd)) return -1;
   if (!dy) NFFT4GP_HIP_CHECK(hipMemcpyAsync(y, yd, sizeof(double) * ny, hipMemcpyDeviceToHost, s));
   NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
   return 0;
}

PlanExt* additive_plan(void* str)
{
   if (!str) return nullptr;
   return (PlanExt*)((nfft4gp_kernel*)str)->_external;
}


// kernels.c:404-441: _ldwork = max_n, or max_n * omp_get_max_threads() for an OpenMP handle.  This library
// has no OpenMP of its own, but when the reference's dense kernels share the process (its kernels.c calls
// this function through the dynamic linker once libnfft4gp_amd precedes it) they index _dwork per thread:
// ask the OpenMP runtime already in the process, if any.
int omp_threads_in_process()
{
   using fn_t = int (*)();
   static fn_t f = (fn_t)dlsym(RTLD_DEFAULT, "omp_get_max_threads");
   return f ? std::max(1, f()) : 1;
}

nfft4gp_kernel* kernel_struct_create(int max_n, int omp = 0)
{
   nfft4gp_kernel* k = (nfft4gp_kernel*)calloc(1, sizeof(nfft4gp_kernel));
   k->_max_n = max_n;
   k->_omp = omp;
   k->_ldwork = (size_t)max_n * (size_t)(omp ? omp_threads_in_process() : 1);
   k->_dwork = (double*)malloc(sizeof(double) * std::max<size_t>(1, k->_ldwork));
   return k;
}

int setup_common(void* str, int kernel, int n, int ldim, double** Kp, double** dKp)
{
   if (Kp == NULL || dKp == NULL) {
      printf("Error: NFFT kernel requires Kp and dKp to be not NULL.\n");
      return -1;
   }
   nfft4gp_kernel* kd = (nfft4gp_kernel*)str;
   PlanExt* E = additive_plan(str);
   if (!E) return -1;
   (void)n;
   (void)ldim;
   if (plan_setup(E->P, kd->_buffer, kernel, kd->_params[0], kd->_params[1], kd->_noise_level)) return -1;
   *Kp = (double*)str;
   *dKp = (double*)str;
   return 0;
}

// Points per block B: the interpolation runs one workgroup per block and the spread one per (block, window
// group), so a handle with few points (a small problem, or a row shard of several GPUs) needs smaller
// blocks to fill the 256 CUs, at the price of more partial grids and per-workgroup folds.  Measured per
// matvec (32 windows; n: B = 4064 / 2032 / 1016): 1e6: 85.6 / 104.4 / 146.9 us; 5e5: 59.7 / 57.0 / -;
// 2.5e5: 45.6 / 39.7 / 41.5; 1.25e5: 39.1 / 29.9 / 29.1; 1e5 (8 windows): 21.6 / 17.1 / 16.9.
// Every block size is a multiple of 16 (so are the row shards' first rows, dist.row_range): a point's local index
// is then its global index mod 16 in its low 4 bits whatever the layout, and so is the sub-quantum offset those
// bits set in its q word (slot_word) -- the operator does not depend on the block size or the row split.
int default_block(int n)
{
   if (n >= 200 * kMaxBlock) return kMaxBlock;
   if (n >= 40 * 2032) return 2032;
   return 1024;
}

// tuning overrides (layout only; results are independent of them up to rounding)
void env_layout(AdditivePlan& P)
{
   P.B = default_block(P.n);
   // windows per spread workgroup: at most 4 (with the [window][degree][cell] moment table three 4-window
   // workgroups of a 4064-point block fit a CU's LDS: config C's spread 40.8 -> 38.7 us, the matvec 78.9 -> 78.4,
   // profiles/r05_spread_ab.txt; 5 / 6 / 8 windows: spread 34.0 -> 36.4 / 40.8 / 37.9 us,
   // profiles/r05_spread_cg_ab.txt), spread evenly over the fewest groups -- a one-window workgroup pays the whole
   // alpha staging and fold (round 4: 4 windows as 2 + 2 took 22.3 against 24.2 us as 3 + 1 per rank of
   // BASELINE configs[3]'s component split, profiles/r04_component_cg_sweep.txt)
   // ... unless that leaves fewer than 384 spread workgroups (1.5 per CU): then at most 3 per group, as in round 4
   // (BASELINE configs[3]'s component shard, 4 windows x 247 blocks: one 4-window group is 247 workgroups, 23.3 us
   // per rank against 22.3 us as 2 + 2, profiles/r05_mid_shard_components8.json)
   {
      const int nw = std::max(P.nw, 1), nblocks = std::max(1, (P.n + P.B - 1) / P.B);
      auto pick = [&](int cgmax) {
         const int ngroups = (nw + cgmax - 1) / cgmax;
         P.CG = (nw + ngroups - 1) / ngroups;
         return ngroups;
      };
      if ((long long)pick(4) * nblocks < 384) pick(3);
   }
   if (const char* e = getenv("NFFT4GP_AMD_BLOCK")) {
      const int v = atoi(e);
      if (v >= 256) P.B = std::min(v, kMaxBlock) & ~15;  // a multiple of 16 (default_block)
   }
   if (const char* e = getenv("NFFT4GP_AMD_CG")) {
      const int v = atoi(e);
      if (v >= 1 && v <= 64) P.CG = v;
   }
   if (const char* e = getenv("NFFT4GP_AMD_SPREAD_VARIANT")) P.spread_variant = atoi(e);
   if (const char* e = getenv("NFFT4GP_AMD_DET")) P.det = atoi(e) != 0;
   if (const char* e = getenv("NFFT4GP_AMD_PRECISION")) P.rec = atoi(e) == 32 ? 4 : 5;
}

void* additive_create(double* data, int n_global, int ldim, int* windows, int nwindows, int dwindows, int rb, int re)
{
   nfft4gp_kernel* kd = kernel_struct_create(3 * n_global);  // nfft_interface.c:624
   kd->_iparams[0] = nwindows;
   kd->_iparams[1] = dwindows;
   int skip_window = 1;
   kd->_iparams[2] = 0;
   while (skip_window < dwindows && windows[nwindows * dwindows - skip_window] < 0) {  // :630-636
      skip_window++;
      kd->_iparams[2]++;
   }
   kd->_ibufferp = (int**)malloc(sizeof(int*));
   kd->_ibufferp[0] = windows;
   kd->_buffer = (double*)malloc(sizeof(double) * (size_t)n_global * nwindows * dwindows);
   kd->_own_buffer = 1;
   PlanExt* E = new PlanExt();
   AdditivePlan& P = E->P;
   P.n_global = n_global;
   P.row_begin = rb;
   P.row_end = re;
   P.n = re - rb;
   P.nw = nwindows;
   P.dw = dwindows;
   P.skip_last = kd->_iparams[2];
   P.weight = 1.0 / (double)nwindows;  // nfft_interface.c:806
   env_layout(P);
   double* dst = kd->_buffer;
   const int* fw = windows;
   for (int i = 0; i < nwindows; i++) {  // :648-670
      int actual = 0;
      for (int j = 0; j < dwindows; j++) {
         if (fw[0] >= 0) {
            memcpy(dst, data + (size_t)fw[0] * ldim, sizeof(double) * n_global);
            fw++;
            dst += n_global;
            actual++;
         }
      }
      P.comp_dims.push_back(actual);
   }
   kd->_external = E;
   return kd;
}

}  // namespace

namespace nfft4gp_amd {
bool additive_fused_dot_ok(void* str)
{
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready) return false;
   const AdditivePlan& P = E->P;
   if (P.row_begin != 0 || P.row_end != P.n_global) return false;
   return P.md.on || P.nblocks <= kRedMaxBlocks;
}

int additive_matvec_dot(void* str, const double* d_x, double* d_y, double* d_dot)
{
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready) return -1;
   AdditivePlan& P = E->P;
   hipStream_t s = current_stream();
   if (P.md.on) {
      if (md_spread(P, d_x, P.md.d_grid, s) || md_grid(P, P.md.d_grid, 0, s)) return -1;
      return md_interp(P, 0, 1.0, d_x, 0.0, d_y, s, d_dot);
   }
   if (launch_spread_grid(P, d_x, 0, s)) return -1;
   return launch_interp(P, 0, 1.0, d_x, 0.0, d_y, s, d_dot);
}
}  // namespace nfft4gp_amd

namespace nfft4gp_amd {
// y_v = beta y_v + alpha A x_v for nv device vectors: two per pass over the layout (launch_matvec2), an odd
// last vector (and multi-feature-window handles) through the single-vector matvec
int additive_matvec_multi(void* str, int nv, double alpha, const double* const* X, double beta, double* const* Y)
{
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready) return -1;
   AdditivePlan& P = E->P;
   if (P.row_begin != 0 || P.row_end != P.n_global) return -1;
   hipStream_t s = current_stream();
   int v = 0;
   if (!P.md.on && !P.timing)
      for (; v + 1 < nv; v += 2)
         if (launch_matvec2(P, alpha, X[v], X[v + 1], beta, Y[v], Y[v + 1], s)) return -1;
   for (; v < nv; v++)
      if (plan_apply_dev(E, 0, alpha, X[v], beta, Y[v])) return -1;
   return 0;
}

int additive_matvec_chunked(void* str, double alpha, const double* d_x, double* d_y, int nchunks,
                            int (*done)(void* ctx, size_t r0, size_t r1), void* ctx)
{
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready) return -1;
   AdditivePlan& P = E->P;
   if (P.md.on || P.timing || P.row_begin != 0 || P.row_end != P.n_global || P.nblocks == 0) return -1;
   hipStream_t s = current_stream();
   if (launch_spread_grid(P, d_x, 0, s)) return -1;
   nchunks = std::max(1, std::min(nchunks, P.nblocks));
   for (int c = 0; c < nchunks; c++) {
      const int b0 = (int)((long long)P.nblocks * c / nchunks), b1 = (int)((long long)P.nblocks * (c + 1) / nchunks);
      if (launch_interp_blocks(P, alpha, d_x, 0.0, d_y, b0, b1, s)) return -1;
      if (done(ctx, (size_t)b0 * P.B, std::min((size_t)b1 * P.B, (size_t)P.n))) return -1;
   }
   return 0;
}

// rows of an additive handle: local (this shard) and global; -1 when str is not an additive handle
int additive_rows(void* str, int* n_local, int* n_global, int* row_begin)
{
   PlanExt* E = additive_plan(str);
   if (!E) return -1;
   *n_local = E->P.n;
   *n_global = E->P.n_global;
   if (row_begin) *row_begin = E->P.row_begin;
   return 0;
}

// interpolation workgroups per block of a row shard's split finish (Nfft4GPAmdShardFinish)
// (deterministic mode: 1 unless NFFT4GP_AMD_SHARD_SPLIT asks -- the split interpolation's y-slices add with
// unrounded atomics)
static int shard_split(const AdditivePlan& P)
{
   int S = (P.nblocks <= 64 && !P.det) ? 4 : 1;
   if (const char* e = getenv("NFFT4GP_AMD_SHARD_SPLIT")) S = std::max(1, std::min(16, atoi(e)));
   return std::min(S, std::max(1, P.ngroups));
}

// the row-sharded matvec's local interpolation with the fused (y, x) partial dot of these rows
// (not yet summed over the shards): the q = A p, (q, p) step of a distributed CG
bool shard_fused_dot_ok(void* str)
{
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready) return false;
   return E->P.md.on || E->P.nblocks <= kRedMaxBlocks;
}

bool shard_peer_ok(void* str)
{
   PlanExt* E = additive_plan(str);
   return E && E->P.points_ready && !E->P.md.on;
}

int shard_spread_peer(void* str, const double* x_local, const PeerArgs& A)
{
   (void)A;  // the put into this rank's slot happens in the finish (or shard_peer_sum)
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready || E->P.md.on) return -1;
   AdditivePlan& P = E->P;
   hipStream_t s = current_stream();
   return (P.nblocks > 0 && launch_spread(P, x_local, P.d_part, s)) ? -1 : 0;
}

int shard_peer_sum(void* str, const PeerArgs& A, double* d_grid)
{
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready || E->P.md.on) return -1;
   hipStream_t s = current_stream();
   if (launch_reduce_parts(E->P, E->P.d_part, nullptr, s, &A)) return -1;
   return launch_peer_sum(E->P, A, d_grid, s);
}

int shard_finish_peer(void* str, const PeerArgs& A, double* d_grid, int grad, double alpha, const double* x_local,
                      double beta, double* y_local)
{
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready || E->P.md.on) return -1;
   AdditivePlan& P = E->P;
   hipStream_t s = current_stream();
   const int S = shard_split(P);
   if (!grad && S > 1 && !P.timing)
      return launch_shard_finish_split(P, nullptr, alpha, x_local, beta, y_local, S, s, &A, P.d_part);
   // unsplit, not deterministic (k_grid's blocked H sum): the partial-grid sum, put, gather and H in one
   // launch, then k_interp as on the all-reduce path (same grid_tail arithmetic: bitwise equal results)
   if (!grad && !P.timing && !P.det)
      return (launch_peer_grid(P, A, P.d_part, s) || launch_interp(P, 0, alpha, x_local, beta, y_local, s)) ? -1 : 0;
   if (shard_peer_sum(str, A, d_grid) || launch_grid_from_sum(P, d_grid, grad, s)) return -1;
   return launch_interp(P, grad, alpha, x_local, beta, y_local, s);
}

int shard_finish_dot(void* str, const double* grid, const double* x_local, double* y_local, double* d_dot)
{
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready) return -1;
   AdditivePlan& P = E->P;
   hipStream_t s = current_stream();
   if (P.n == 0) {  // a shard without rows contributes 0 to the dot
      NFFT4GP_HIP_CHECK(hipMemsetAsync(d_dot, 0, sizeof(double), s));
      return 0;
   }
   if (P.md.on) {
      if (md_grid(P, grid, 0, s)) return -1;
      return md_interp(P, 0, 1.0, x_local, 0.0, y_local, s, d_dot);
   }
   if (launch_grid_from_sum(P, grid, 0, s)) return -1;
   return launch_interp(P, 0, 1.0, x_local, 0.0, y_local, s, d_dot);
}

// shard_finish_dot over the peer exchange: the one-launch grid step (sum, put, gather, H) where the plan allows
// it (as shard_finish_peer), else the gather into d_grid and shard_finish_dot
int shard_finish_dot_peer(void* str, const PeerArgs& A, double* d_grid, const double* x_local, double* y_local,
                          double* d_dot)
{
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready || E->P.md.on) return -1;
   AdditivePlan& P = E->P;
   hipStream_t s = current_stream();
   if (P.n > 0 && !P.det && !P.timing)
      return (launch_peer_grid(P, A, P.d_part, s) || launch_interp(P, 0, 1.0, x_local, 0.0, y_local, s, d_dot)) ? -1
                                                                                                            : 0;
   if (shard_peer_sum(str, A, d_grid)) return -1;
   return shard_finish_dot(str, d_grid, x_local, y_local, d_dot);
}
}  // namespace nfft4gp_amd

namespace nfft4gp_amd {
// the gathered window buffer of an additive handle (kernels.h:65-95 _buffer / _iparams) and its plan's
// kernel type (-1 before the first kernel setup); returns -1 for a handle that is not an additive one
int additive_buffer_info(void* str, const double** xw, int* n, int* nw, int* dw, int* skip_last, int* kernel)
{
   nfft4gp_kernel* kd = (nfft4gp_kernel*)str;
   PlanExt* E = additive_plan(str);
   if (!kd || !E || !kd->_buffer) return -1;
   const AdditivePlan& P = E->P;
   if (P.row_begin != 0 || P.row_end != P.n_global) return -1;
   *xw = kd->_buffer;
   *n = P.n_global;
   *nw = kd->_iparams[0];
   *dw = kd->_iparams[1];
   *skip_last = kd->_iparams[2];
   *kernel = P.points_ready ? P.kernel : -1;
   return 0;
}
}  // namespace nfft4gp_amd

extern "C" {

static const char* kVersion = "nfft4gp_amd 0.1.0 (gfx950)";

const char* Nfft4GPAmdVersion(void) { return kVersion; }
int Nfft4GPAmdDeviceAvailable(void) { return device_ok(); }
void Nfft4GPAmdSetStream(void* s) { g_stream = (hipStream_t)s; }
void* Nfft4GPAmdGetStream(void) { return (void*)g_stream; }

void* Nfft4GPKernelParamCreate(int max_n, int omp) { return kernel_struct_create(max_n, omp); }

void Nfft4GPKernelParamFree(void* str)
{
   nfft4gp_kernel* k = (nfft4gp_kernel*)str;
   if (!k) return;
   free(k->_dwork);
   if (k->_own_buffer) free(k->_buffer);
   if (k->_own_dbuffer) free(k->_dbuffer);
   free(k->_ibufferp);
   if (k->_own_fkernel_buffer_params) Nfft4GPKernelParamFree(k->_fkernel_buffer_params);
   free(k);
}

/* ------------------------------- additive ----------------------------------------------------- */
void* Nfft4GPNFFTAdditiveKernelParamCreate(double* data, int n, int ldim, int d, int* windows, int nwindows,
                                           int dwindows)
{
   (void)d;
   RandScope rand_scope;  // HIP's first use may draw rand(); the reference's NFFT entry points draw none
   return additive_create(data, n, ldim, windows, nwindows, dwindows, 0, n);
}

void* Nfft4GPAmdAdditiveShardCreate(double* data, int n_global, int ldim, int d, int* windows, int nwindows,
                                    int dwindows, int row_begin, int row_end)
{
   (void)d;
   if (row_begin < 0 || row_end > n_global || row_begin > row_end) {
      fprintf(stderr, "nfft4gp_amd: invalid shard rows [%d, %d) of %d\n", row_begin, row_end, n_global);
      return NULL;
   }
   return additive_create(data, n_global, ldim, windows, nwindows, dwindows, row_begin, row_end);
}

int Nfft4GPNFFTAdditiveKernelGaussianKernel(void* str, double* data, int n, int ldim, int d, int* permr, int kr,
                                            int* permc, int kc, double** Kp, double** dKp)
{
   (void)data, (void)d, (void)permr, (void)kr, (void)permc, (void)kc;
   RandScope rand_scope;
   return setup_common(str, 0, n, ldim, Kp, dKp);
}

int Nfft4GPNFFTAdditiveKernelMatern12Kernel(void* str, double* data, int n, int ldim, int d, int* permr, int kr,
                                            int* permc, int kc, double** Kp, double** dKp)
{
   (void)data, (void)d, (void)permr, (void)kr, (void)permc, (void)kc;
   RandScope rand_scope;
   return setup_common(str, 1, n, ldim, Kp, dKp);
}

int Nfft4GPAdditiveNFFTMatSymv(void* data, int n, double alpha, double* x, double beta, double* y)
{
   PlanExt* E = additive_plan(data);
   if (!E) return -1;
   // no RandScope on the apply path: HIP was initialised by the handle's create / setup
   return plan_apply(E, n, 0, alpha, x, beta, y);
}

int Nfft4GPAmdAdditiveMatSymvMulti(void* data, int n, int nrhs, double alpha, const double* X, long long ldx,
                                   double beta, double* Y, long long ldy)
{
   PlanExt* E = additive_plan(data);
   if (!E || !E->P.points_ready || n != E->P.n || nrhs < 0 || ldx < n || ldy < n) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAdditiveMatSymvMulti: handle not set up, or n / ld mismatch\n");
      return -1;
   }
   if (nrhs == 0) return 0;
   if (!is_device_ptr(X) || !is_device_ptr(Y)) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAdditiveMatSymvMulti takes device arrays\n");
      return -1;
   }
   std::vector<const double*> xs(nrhs);
   std::vector<double*> ys(nrhs);
   for (int v = 0; v < nrhs; v++) {
      xs[v] = X + (size_t)v * ldx;
      ys[v] = Y + (size_t)v * ldy;
   }
   return additive_matvec_multi(data, nrhs, alpha, xs.data(), beta, ys.data());
}

int Nfft4GPAdditiveNFFTGradMatSymv(void* data, int n, double alpha, double* x, double beta, double* y)
{
   PlanExt* E = additive_plan(data);
   if (!E) return -1;
   return plan_apply(E, n, 1, alpha, x, beta, y);
}

void Nfft4GPAdditiveNFFTKernelFree(void* str)
{
   if (!str) return;
   free_plan(additive_plan(str));
   ((nfft4gp_kernel*)str)->_external = NULL;
   Nfft4GPKernelParamFree(str);
}

double* Nfft4GPNFFTAppendData(double* X1, int n1, int ldim1, int d, double* X2, int n2, int ldim2)
{
   double* X = (double*)malloc(sizeof(double) * (size_t)(n1 + n2) * d);
   for (int i = 0; i < d; i++) {
      memcpy(X + (size_t)i * (n1 + n2), X1 + (size_t)i * ldim1, sizeof(double) * n1);
      memcpy(X + (size_t)i * (n1 + n2) + n1, X2 + (size_t)i * ldim2, sizeof(double) * n2);
   }
   return X;
}

int Nfft4GPAmdAdditiveLayoutInfo(void* str, long long* out, int nout)
{
   PlanExt* E = additive_plan(str);
   if (!E || !out) return -1;
   const AdditivePlan& P = E->P;
   long long v[10] = {P.n, P.nw, P.B, P.nblocks, P.dl.ntiles, P.dl.ntiles * kWave * kR, kR, P.CG, P.ngroups,
                      (long long)P.dl.bytes};
   for (int i = 0; i < nout && i < 10; i++) out[i] = v[i];
   return 0;
}

int Nfft4GPAmdSetPrecision(void* str, int bits)
{
   PlanExt* E = additive_plan(str);
   if (!E || (bits != 32 && bits != 64)) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdSetPrecision needs an additive handle and bits 32 or 64\n");
      return -1;
   }
   AdditivePlan& P = E->P;
   const int rec = bits == 32 ? 4 : 5;
   if (rec == P.rec) return 0;
   (void)hipStreamSynchronize(current_stream());
   P.rec = rec;
   if (!P.points_ready || P.md.on) return 0;  // multi-feature windows keep their fp64 coordinates
   // the layout is rebuilt from the handle's points, and the kernel's coefficients with it
   const double* buffer = ((nfft4gp_kernel*)str)->_buffer;
   P.points_ready = false;
   if (plan_build_points(P, buffer)) return -1;
   return plan_setup(P, buffer, P.kernel, P.f, P.l, P.mu);
}

int Nfft4GPAmdSetDeterministic(void* str, int on)
{
   PlanExt* E = additive_plan(str);
   if (!E) return -1;
   (void)hipStreamSynchronize(current_stream());
   E->P.det = on != 0;
   return 0;
}

int Nfft4GPAmdTimingEnable(void* str, int enable)
{
   PlanExt* E = additive_plan(str);
   if (!E) return -1;
   E->P.timing = enable != 0;
   if (enable) {
      (void)hipStreamSynchronize(current_stream());
      for (auto& r : E->pending) E->pool.push_back(r);
      E->pending.clear();
      for (int i = 0; i < 3; i++) {
         E->P.ms[i] = 0;
         E->P.cnt[i] = 0;
      }
   }
   return 0;
}

int Nfft4GPAmdTimingQuery(void* str, double* ms, long long* cnt)
{
   PlanExt* E = additive_plan(str);
   if (!E) return -1;
   AdditivePlan& P = E->P;
   for (auto& r : E->pending) {
      NFFT4GP_HIP_CHECK(hipEventSynchronize(r.ev[5]));
      for (int i = 0; i < 3; i++) {
         float t = 0.f;
         NFFT4GP_HIP_CHECK(hipEventElapsedTime(&t, r.ev[2 * i], r.ev[2 * i + 1]));
         P.ms[i] += t;
         P.cnt[i]++;
      }
      E->pool.push_back(r);
   }
   E->pending.clear();
   for (int i = 0; i < 3; i++) {
      if (ms) ms[i] = P.ms[i];
      if (cnt) cnt[i] = P.cnt[i];
   }
   return 0;
}

int Nfft4GPAmdKernelBench(void* str, int which, int grad, int reps, const double* x, double* y, double* ms_avg)
{
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready || reps <= 0 || !ms_avg) return -1;
   AdditivePlan& P = E->P;
   if (!is_device_ptr(x) || !is_device_ptr(y)) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdKernelBench needs device vectors\n");
      return -1;
   }
   hipStream_t s = current_stream();
   hipEvent_t e0, e1;
   NFFT4GP_HIP_CHECK(hipEventCreate(&e0));
   NFFT4GP_HIP_CHECK(hipEventCreate(&e1));
   // one warm launch, then `reps` back-to-back launches of the one kernel between a single event pair
   for (int rep = -1; rep < reps; rep++) {
      if (rep == 0) NFFT4GP_HIP_CHECK(hipEventRecord(e0, s));
      int rc = 0;
      if (P.md.on)
         rc = which == 0 ? md_spread(P, x, P.md.d_grid, s)
              : which == 1 ? md_grid(P, P.md.d_grid, grad, s)
                           : md_interp(P, grad, 1.0, x, 0.0, y, s);
      else if (which == 0)
         rc = launch_spread(P, x, P.d_part, s);
      else if (which == 1)
         rc = launch_grid(P, P.d_part, P.nparts, grad, s);
      else
         rc = launch_interp(P, grad, 1.0, x, 0.0, y, s);
      if (rc) return -1;
   }
   NFFT4GP_HIP_CHECK(hipEventRecord(e1, s));
   NFFT4GP_HIP_CHECK(hipEventSynchronize(e1));
   float t = 0.f;
   NFFT4GP_HIP_CHECK(hipEventElapsedTime(&t, e0, e1));
   *ms_avg = (double)t / reps;
   (void)hipEventDestroy(e0);
   (void)hipEventDestroy(e1);
   return 0;
}


void* Nfft4GPAmdNysSetupAdditive(void* str, const int* perm, int k, int k11_mode)
{
   if (!device_ok()) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdNysSetupAdditive: no HIP device visible (no CPU fallback).\n");
      return nullptr;
   }
   nfft4gp_kernel* kd = (nfft4gp_kernel*)str;
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready || !perm) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdNysSetupAdditive needs an additive handle after its kernel setup\n");
      return nullptr;
   }
   const AdditivePlan& P = E->P;
   if (P.row_begin != 0 || P.row_end != P.n_global) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdNysSetupAdditive: row-sharded handles are not supported\n");
      return nullptr;
   }
   return nys_setup_additive(kd->_buffer, P.n_global, P.nw, P.dw, P.skip_last, P.kernel, kd->_params[0],
                             kd->_params[1], kd->_noise_level, perm, k, k11_mode);
}

}  // extern "C"

namespace nfft4gp_amd {
// the row-sharded Nystrom setup of a row-shard handle (its gathered buffer holds all n_global rows): the
// panel, U1 and U of its own rows, the Gram all-reduced over comm (dist.hip Nfft4GPAmdNysShardSetupAdditive)
NysDev* nys_setup_shard(void* str, const int* perm, int k, int k11_mode, Comm* comm)
{
   nfft4gp_kernel* kd = (nfft4gp_kernel*)str;
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready || !perm || !comm) {
      fprintf(stderr, "nfft4gp_amd: the sharded Nystrom setup needs a row-shard handle after its kernel setup\n");
      return nullptr;
   }
   const AdditivePlan& P = E->P;
   NysShard sh;
   sh.comm = comm;
   sh.row_begin = P.row_begin;
   sh.n_global = P.n_global;
   return nys_setup_additive(kd->_buffer, P.n, P.nw, P.dw, P.skip_last, P.kernel, kd->_params[0], kd->_params[1],
                             kd->_noise_level, perm, k, k11_mode, false, &sh);
}
}  // namespace nfft4gp_amd

extern "C" {

int Nfft4GPAmdAdditiveComponentShard(void* str, int nw_global, int own_diag)
{
   PlanExt* E = additive_plan(str);
   if (!E || nw_global < E->P.nw || E->P.row_begin != 0 || E->P.row_end != E->P.n_global) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdAdditiveComponentShard needs a whole-row additive handle and "
                      "nw_global >= its %d windows\n", E ? E->P.nw : 0);
      return -1;
   }
   E->P.weight = 1.0 / (double)nw_global;  // the whole operator's 1/nwindows (nfft_interface.c:806)
   E->P.diag = own_diag ? 1.0 : 0.0;
   // after a kernel setup the weight is already folded into the circulants: rebuild them with the new one
   AdditivePlan& P = E->P;
   if (P.points_ready) return plan_setup(P, ((nfft4gp_kernel*)str)->_buffer, P.kernel, P.f, P.l, P.mu);
   return 0;
}

int Nfft4GPAmdShardSpread(void* str, const double* x_local, double* grid)
{
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready) return -1;
   AdditivePlan& P = E->P;
   hipStream_t s = current_stream();
   if (P.md.on) return md_spread(P, x_local, grid, s);
   if (P.nblocks == 0) {
      NFFT4GP_HIP_CHECK(hipMemsetAsync(grid, 0, sizeof(double) * P.nw * kNos, s));
      return 0;
   }
   // the blocks' partial grids summed by k_reduce_parts into the grid the caller all-reduces
   if (launch_spread(P, x_local, P.d_part, s)) return -1;
   return launch_reduce_parts(P, P.d_part, grid, s);
}

int Nfft4GPAmdShardFinish(void* str, const double* grid, int grad, double alpha, const double* x_local, double beta,
                          double* y_local)
{
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready) return -1;
   AdditivePlan& P = E->P;
   hipStream_t s = current_stream();
   if (P.md.on) {
      if (md_grid(P, grid, grad, s)) return -1;
      return md_interp(P, grad, alpha, x_local, beta, y_local, s);
   }
   // few blocks (a row shard of many GPUs): S interpolation workgroups per block so the launch fills more
   // CUs.  Measured per-rank matvec at config C (tools/shard_probe.py, S = 1 / 2 / 4 / 8): 8 GPUs (62 blocks)
   // 31.1 / 31.3 / 29.3 / 32.1 us; 4 GPUs (123 blocks) 41.0 / 43.0 / 45.2 / 50.5; 2 GPUs 59.7 / 66.8 / ...
   // so S = 4 at <= 64 blocks, else 1 (NFFT4GP_AMD_SHARD_SPLIT overrides S)
   const int S = shard_split(P);
   if (!grad && S > 1 && !P.timing) return launch_shard_finish_split(P, grid, alpha, x_local, beta, y_local, S, s);
   if (launch_grid_from_sum(P, grid, grad, s)) return -1;
   return launch_interp(P, grad, alpha, x_local, beta, y_local, s);
}

// debugging: the circulant coefficients H ([nw][64][kNC]) of the last grid pass into out (count doubles at
// most); returns the number copied, or -1
long long Nfft4GPAmdDebugShardH(void* str, double* out, long long count)
{
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready || E->P.md.on || !out || !E->P.d_H) return -1;
   const long long m = std::min(count, (long long)E->P.nw * kNos * kNC);
   if (hipStreamSynchronize(current_stream()) != hipSuccess ||
       hipMemcpy(out, E->P.d_H, sizeof(double) * (size_t)m, hipMemcpyDeviceToHost) != hipSuccess)
      return -1;
   return m;
}

long long Nfft4GPAmdShardGridSize(void* str)
{
   PlanExt* E = additive_plan(str);
   if (!E || !E->P.points_ready) return -1;
   const AdditivePlan& P = E->P;
   return P.md.on ? (long long)P.nw * P.md.G : (long long)P.nw * kNos;
}

/* ------------------------------- host-only helpers -------------------------------------------- */
int Nfft4GPAmdHostTapPoly(double* C)
{
   if (C) {
      const std::vector<double>& T = tap_poly_coeffs();
      memcpy(C, T.data(), sizeof(double) * T.size());
   }
   return kNC;
}

int Nfft4GPAmdHostCirculant(int kind, double c, double weight, double* bhat, double* w)
{
   double bh[kBand];
   bhat_1d(kind, c, bh);
   if (bhat) memcpy(bhat, bh, sizeof(bh));
   if (w) circulant_1d(bh, weight, w);
   return 0;
}

double Nfft4GPAmdHostPrepare(const double* col, int n, unsigned int* q)
{
   std::vector<double> xs;
   const double sc = centre_and_scale(col, n, 1, xs);
   if (sc < 0.0) return sc;
   for (int j = 0; j < n; j++) q[j] = quantize(xs[j]);
   return sc;
}

int Nfft4GPAmdHostLayout(const unsigned int* qc, int n, int nw, int B, int CG, long long* counts,
                         unsigned short* meta, unsigned int* lo, unsigned int* q, int* tile_off)
{
   return Nfft4GPAmdHostLayoutRec(qc, n, nw, B, CG, 5, counts, meta, lo, q, tile_off);
}

int Nfft4GPAmdHostLayoutRec(const unsigned int* qc, int n, int nw, int B, int CG, int rec, long long* counts,
                            unsigned short* meta, unsigned int* lo, unsigned int* q, int* tile_off)
{
   if (B <= 0 || B > kMaxBlock || CG <= 0 || n < 0 || nw <= 0 || nw > 1023 || (rec != 4 && rec != 5)) return -1;
   Layout L;
   build_layout(qc, n, nw, B, CG, L, rec);
   counts[0] = L.ntiles;
   counts[1] = L.ngroups;
   counts[2] = L.nblocks;
   if (meta) memcpy(meta, L.meta.data(), L.meta.size() * sizeof(uint16_t));
   if (lo && !L.lo.empty()) memcpy(lo, L.lo.data(), L.lo.size() * sizeof(uint32_t));
   if (q) memcpy(q, L.q.data(), L.q.size() * sizeof(uint32_t));
   if (tile_off) memcpy(tile_off, L.tile_off.data(), L.tile_off.size() * sizeof(int));
   return 0;
}

/* ------------------------------- single component --------------------------------------------- */
void* Nfft4GPNFFTKernelParamCreate(int max_n, int dim)
{
   nfft4gp_kernel* kd = kernel_struct_create(max_n);  // nfft_interface.c:5
   SingleAdj* adj = new SingleAdj();
   adj->owner = kd;
   adj->dim = dim;
   adj->max_n = max_n;
   kd->_external = adj;
   return kd;
}

int Nfft4GPNFFTKernelParamRemovePoints(void* kernel)
{
   nfft4gp_kernel* kd = (nfft4gp_kernel*)kernel;
   SingleAdj* adj = kd ? (SingleAdj*)kd->_external : nullptr;
   if (adj && adj->plan) {
      free_layout(adj->plan->P);
      adj->plan->P.points_ready = false;
   }
   return 0;
}

int Nfft4GPNFFTKernelParamFreeNFFTKernel(void* kernel) { return Nfft4GPNFFTKernelParamRemovePoints(kernel); }

void Nfft4GPNFFTKernelParamFree(void* kernel)
{
   nfft4gp_kernel* kd = (nfft4gp_kernel*)kernel;
   if (!kd) return;
   SingleAdj* adj = (SingleAdj*)kd->_external;
   if (adj) {
      free_plan(adj->plan);
      delete adj;
   }
   kd->_external = NULL;
   Nfft4GPKernelParamFree(kd);
}

void Nfft4GPNFFTKernelFree(void* str) { (void)str; }

static int single_setup(void* str, int kernel, double* data, int n, int ldim, int d, double** Kp, double** dKp)
{
   nfft4gp_kernel* kd = (nfft4gp_kernel*)str;
   SingleAdj* adj = (SingleAdj*)kd->_external;
   if (Kp == NULL || dKp == NULL) {
      printf("Error: NFFT kernel requires Kp and dKp to be not NULL.\n");
      return -1;
   }
   if (n != ldim) {
      printf("Error: NFFT kernel requires n == ldim.\n");
      return -1;
   }
   if (!adj->plan) {
      adj->data.assign(data, data + (size_t)n * d);  // first call fixes the points (:150-153)
      adj->plan = new PlanExt();
      AdditivePlan& P = adj->plan->P;
      P.n_global = n;
      P.row_begin = 0;
      P.row_end = n;
      P.n = n;
      P.nw = 1;
      P.dw = d;
      P.weight = 1.0;
      P.comp_dims.assign(1, d);
      env_layout(P);
   }
   AdditivePlan& P = adj->plan->P;
   if (plan_setup(P, adj->data.data(), kernel, kd->_params[0], kd->_params[1], kd->_noise_level)) return -1;
   // the reference's str_adj scalars (nfft_interface.c:14-28, :150-231)
   str_adj& A = adj->pub;
   A._kernel = kernel;
   A._d = d;
   adj->sigma_pub = P.comp_sigma.empty() ? 0.0 : P.comp_sigma[0];
   A._sigma = &adj->sigma_pub;
   A._mu = kd->_noise_level;
   A._N = kBand;
   A._p = 1;
   A._m = kM;
   A._eps = 0.0;
   A._n = n;
   A._NN = kNos;
   A._x = nullptr;
   A._scale = P.comp_scale.empty() ? 1.0 : P.comp_scale[0];
   A._kernel_scale = kd->_params[0];
   A._fastsum_original = nullptr;
   A._fastsum_derivative = nullptr;
   *Kp = (double*)adj;
   *dKp = (double*)adj;
   return 0;
}

int Nfft4GPNFFTKernelGaussianKernel(void* str, double* data, int n, int ldim, int d, int* permr, int kr, int* permc,
                                    int kc, double** Kp, double** dKp)
{
   (void)permr, (void)kr, (void)permc, (void)kc;
   RandScope rand_scope;
   return single_setup(str, 0, data, n, ldim, d, Kp, dKp);
}

int Nfft4GPNFFTKernelMatern12Kernel(void* str, double* data, int n, int ldim, int d, int* permr, int kr, int* permc,
                                    int kc, double** Kp, double** dKp)
{
   (void)permr, (void)kr, (void)permc, (void)kc;
   RandScope rand_scope;
   return single_setup(str, 1, data, n, ldim, d, Kp, dKp);
}

int Nfft4GPNFFTMatSymv(void* data, int n, double alpha, double* x, double beta, double* y)
{
   SingleAdj* adj = (SingleAdj*)data;
   if (!adj || !adj->plan) return -1;
   return plan_apply(adj->plan, n, 0, alpha, x, beta, y);
}

int Nfft4GPNFFTGradMatSymv(void* data, int n, double alpha, double* x, double beta, double* y)
{
   SingleAdj* adj = (SingleAdj*)data;
   if (!adj || !adj->plan) return -1;
   return plan_apply(adj->plan, n, 1, alpha, x, beta, y);
}

}  // extern "C"
