// callbacks.hpp -- host/device vector views and the operator/preconditioner callback adapter shared by
// the Krylov solvers (solvers.hip: PCG; krylov.hip: FGMRES, Lanczos, the GP loss).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdio>

#include "internal.h"

namespace nfft4gp_amd {

// host-or-device view of a vector: host pointers are staged through device memory
struct Vec {
   double* d = nullptr;
   double* h = nullptr;
   size_t n = 0;
   bool staged = false;
   int open(double* p, size_t nn, bool copy_in)
   {
      n = nn;
      if (is_device_ptr(p)) {
         d = p;
         return 0;
      }
      h = p;
      staged = true;
      NFFT4GP_HIP_CHECK(hipMalloc((void**)&d, sizeof(double) * (n ? n : 1)));
      if (copy_in && n) NFFT4GP_HIP_CHECK(hipMemcpy(d, h, sizeof(double) * n, hipMemcpyHostToDevice));
      return 0;
   }
   int close(bool copy_out)
   {
      if (staged) {
         hipStream_t s = current_stream();
         NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
         if (copy_out && n) NFFT4GP_HIP_CHECK(hipMemcpy(h, d, sizeof(double) * n, hipMemcpyDeviceToHost));
         NFFT4GP_HIP_CHECK(hipFree(d));
         d = nullptr;
      }
      return 0;
   }
};

inline bool need_device(const char* who)
{
   if (!device_ok()) {
      fprintf(stderr, "nfft4gp_amd: %s: no HIP device visible (no CPU fallback).\n", who);
      return false;
   }
   return true;
}

// ---- operator / preconditioner callbacks of Nfft4GPSolverPcg ----------------------------------
// The library's own operators take device pointers.  Any other callback (e.g. the reference's
// Nfft4GPDenseMatSymv on a host matrix) is called the reference's way, with HOST vectors: the
// adapter stages its input and output through pinned host buffers around the call.  Mode -1 (auto)
// decides per function pointer; 0 forces host staging, 1 forces device pointers.

struct Callbacks {
   func_symmatvec matvec;
   void* mat;
   func_solve prec;
   void* pdata;
   bool mv_dev, pc_dev;
   size_t n;
   size_t out_mult = 1;  // 3 for the gradient operators (y has 3n entries)
   // a distributed operator (dist.hip): row shards sum every dot over `comm` and hold rows
   // [row_begin, row_begin + n) of n_global; replicated vectors (component shards, one GPU) have comm == NULL
   Comm* comm = nullptr;
   size_t n_global = 0, row_begin = 0;
   double *h_in = nullptr, *h_out = nullptr;
   int ensure_host()
   {
      if (!h_in) {
         NFFT4GP_HIP_CHECK(hipHostMalloc((void**)&h_in, sizeof(double) * (n ? n : 1)));
         NFFT4GP_HIP_CHECK(hipHostMalloc((void**)&h_out, sizeof(double) * (n ? n * out_mult : 1)));
      }
      return 0;
   }
   ~Callbacks()
   {
      if (h_in) (void)hipHostFree(h_in);
      if (h_out) (void)hipHostFree(h_out);
   }
   // y = alpha A x + beta y on device vectors
   int apply(double alpha, double* dx, double beta, double* dy)
   {
      if (mv_dev) return matvec(mat, (int)n, alpha, dx, beta, dy);
      if (ensure_host()) return -1;
      hipStream_t s = current_stream();
      const size_t no = n * out_mult;
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(h_in, dx, sizeof(double) * n, hipMemcpyDeviceToHost, s));
      if (beta != 0.0) NFFT4GP_HIP_CHECK(hipMemcpyAsync(h_out, dy, sizeof(double) * no, hipMemcpyDeviceToHost, s));
      NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
      if (matvec(mat, (int)n, alpha, h_in, beta, h_out)) return -1;
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(dy, h_out, sizeof(double) * no, hipMemcpyHostToDevice, s));
      return 0;
   }
   // z = M^{-1} r on device vectors
   int solve(double* dz, double* dr)
   {
      if (pc_dev) return prec(pdata, (int)n, dz, dr);
      if (ensure_host()) return -1;
      hipStream_t s = current_stream();
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(h_in, dr, sizeof(double) * n, hipMemcpyDeviceToHost, s));
      NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
      if (prec(pdata, (int)n, h_out, h_in)) return -1;
      NFFT4GP_HIP_CHECK(hipMemcpyAsync(dz, h_out, sizeof(double) * n, hipMemcpyHostToDevice, s));
      return 0;
   }
};

// fills cb.comm / n_global / row_begin from the operator (after cb.matvec, cb.mat, cb.n, cb.mv_dev are set)
inline int bind_dist(Callbacks& cb)
{
   cb.comm = nullptr;
   cb.n_global = cb.n;
   cb.row_begin = 0;
   if (!cb.mv_dev || (cb.matvec != &Nfft4GPAmdDistMatSymv && cb.matvec != &Nfft4GPAmdDistGradMatSymv)) return 0;
   DistPcgInfo info;
   if (dist_pcg_info(cb.mat, info)) return -1;
   cb.comm = info.dot_comm;
   cb.n_global = (size_t)info.n_global;
   cb.row_begin = (size_t)info.row_begin;
   return 0;
}

// a solver's last host sync before it reports success: a peer exchange of its distributed operator whose wait
// gave up during the solve (dist.hip) fails the solve instead of returning numbers summed from stale words
inline int dist_final_check(const Callbacks& cb)
{
   if (!cb.mv_dev || (cb.matvec != &Nfft4GPAmdDistMatSymv && cb.matvec != &Nfft4GPAmdDistGradMatSymv)) return 0;
   NFFT4GP_HIP_CHECK(hipStreamSynchronize(current_stream()));
   if (dist_failed(cb.mat)) {
      fprintf(stderr, "nfft4gp_amd: a peer exchange timed out during the solve; its result is discarded\n");
      return -1;
   }
   return 0;
}

// the library's own func_symmatvec / func_solve entry points (these take device pointers)
bool library_operator(const void* fn);
extern int g_cb_mode;  // Nfft4GPAmdSetCallbackPointerMode

}  // namespace nfft4gp_amd
