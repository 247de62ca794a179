// dist.hip -- the additive operator and the Nystrom apply split over one process per GPU.
//
// The reference is one process: Nfft4GPAdditiveNFFTMatSymv runs its components one after another into
// _dwork (nfft_interface.c:796-817) and Nfft4GPSolverPcg (pcg.c:3-206) works on whole vectors.  The sum
// over components and the sum over points are both independent, so the operator splits two ways
// (DESIGN 6):
//   rows        each rank spreads its own points for every window, the nw x 64 grids (16 KB at config D;
//               nw x 64^d for multi-feature windows) are all-reduced, each rank interpolates its rows.
//               PCG vectors stay row-sharded, so Nfft4GPSolverPcg sums its dots over the communicator.
//   components  each rank holds a subset of the windows for all points; y (n doubles) is all-reduced and
//               the vectors are replicated (the dots need no communication).
// Communicators: RCCL (librccl.so.1 dlopen'ed -- the copy PyTorch maps -- one ncclComm per process, every
// all-reduce enqueued on the library stream, no host synchronisation), or a caller's all-reduce callback
// on a device staging buffer (the gloo process group of the one-GPU tests).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types and prototypes only: the library is dlopen'ed on first use

#include <dlfcn.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "internal.h"

using namespace nfft4gp_amd;

namespace {

struct RcclApi {
   bool ok = false;
   decltype(&ncclGetUniqueId) get_id = nullptr;
   decltype(&ncclCommInitRank) init_rank = nullptr;
   decltype(&ncclAllReduce) all_reduce = nullptr;
   decltype(&ncclCommDestroy) destroy = nullptr;
   decltype(&ncclGetErrorString) err = nullptr;
   decltype(&ncclCommCount) count = nullptr;
};

RcclApi& rccl()
{
   static RcclApi R;
   static bool tried = false;
   if (tried) return R;
   tried = true;
   // the soname first: it matches the copy PyTorch's nccl process group already mapped (one RCCL per process)
   static const char* const names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1", nullptr};
   std::string why;
   void* h = nullptr;
   for (const char* const* p = names; *p && !h; ++p) {
      h = dlopen(*p, RTLD_NOW | RTLD_GLOBAL);
      if (!h) {
         const char* e = dlerror();
         why += std::string("\n  ") + (e ? e : *p);
      }
   }
   if (h) {
      R.get_id = (decltype(&ncclGetUniqueId))dlsym(h, "ncclGetUniqueId");
      R.init_rank = (decltype(&ncclCommInitRank))dlsym(h, "ncclCommInitRank");
      R.all_reduce = (decltype(&ncclAllReduce))dlsym(h, "ncclAllReduce");
      R.destroy = (decltype(&ncclCommDestroy))dlsym(h, "ncclCommDestroy");
      R.err = (decltype(&ncclGetErrorString))dlsym(h, "ncclGetErrorString");
      R.count = (decltype(&ncclCommCount))dlsym(h, "ncclCommCount");
      R.ok = R.get_id && R.init_rank && R.all_reduce && R.destroy && R.err && R.count;
      if (!R.ok) why += "\n  an RCCL entry point is missing";
   }
   if (!R.ok) fprintf(stderr, "nfft4gp_amd: RCCL could not be loaded:%s\n", why.c_str());
   return R;
}

struct CommRccl : Comm {
   ncclComm_t c = nullptr;
   int ranks() override
   {
      int k = -1;
      if (!c || rccl().count(c, &k) != ncclSuccess) return -1;
      return k;
   }
   int allreduce(double* d_buf, size_t count, hipStream_t s) override
   {
      if (count == 0) return 0;
      const ncclResult_t r = rccl().all_reduce(d_buf, d_buf, count, ncclDouble, ncclSum, c, s);
      if (r != ncclSuccess) {
         fprintf(stderr, "nfft4gp_amd: ncclAllReduce: %s\n", rccl().err(r));
         return -1;
      }
      return 0;
   }
   ~CommRccl() override
   {
      if (c) rccl().destroy(c);
   }
};

struct CommCallback : Comm {
   int ranks() override { return world; }
   Nfft4GPAmdAllreduceFn fn = nullptr;
   void* ctx = nullptr;
   double* stage = nullptr;  // the caller's device buffer
   size_t cap = 0;
   int allreduce(double* d_buf, size_t count, hipStream_t s) override
   {
      for (size_t off = 0; off < count; off += cap) {
         const size_t m = std::min(cap, count - off);
         NFFT4GP_HIP_CHECK(hipMemcpyAsync(stage, d_buf + off, sizeof(double) * m, hipMemcpyDeviceToDevice, s));
         // the callback may read the staging buffer on another stream (or from the host): the copy must
         // have landed before it runs
         NFFT4GP_HIP_CHECK(hipStreamSynchronize(s));
         if (fn(ctx, stage, (long long)m)) {
            fprintf(stderr, "nfft4gp_amd: the all-reduce callback failed\n");
            return -1;
         }
         // the callback may have written the sum on the library stream (torch's current stream); s may be
         // another one (the component split's chunk stream)
         if (s != current_stream()) NFFT4GP_HIP_CHECK(hipStreamSynchronize(current_stream()));
         NFFT4GP_HIP_CHECK(hipMemcpyAsync(d_buf + off, stage, sizeof(double) * m, hipMemcpyDeviceToDevice, s));
      }
      return 0;
   }
};

// y = beta y + t  (component shards with beta != 0)
__global__ void k_axpby_add(double beta, double* __restrict__ y, const double* __restrict__ t, size_t n)
{
   for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
      y[i] = (beta == 0.0 ? 0.0 : beta * y[i]) + t[i];
}

// the peer-memory exchange of a row-sharded operator (Nfft4GPAmdDistPeerEnable): this rank's exported buffer,
// the peers' opened ones, the device pointer table and the host-mapped error word the waits set
constexpr int kPeerMaxWorld = 256;  // the grid kernels' threads: one polls each rank's flag

constexpr int kPeerScal = 4096;  // scalars per peer all-reduce (larger ones go to the communicator)

// rank r's buffer (nfft_kernels.hip's peer_buf: the first kPeerInline from the kernel arguments)
__device__ __forceinline__ char* peer_rank_buf(const PeerArgs& A, int r)
{
   char* b = A.inl[0];
#pragma unroll
   for (int k = 1; k < kPeerInline; k++)
      if (r == k) b = A.inl[k];
   return r < kPeerInline ? b : A.bufs[r];
}

// The solvers' small all-reduces (dots, norms, Hessenberg columns) over the same IPC buffers as the grid exchange:
// each rank puts its `count` values into its scalar slot of exchange e (two epoch-stamped 64-bit words per value,
// system scope, as the grid entries), then a thread per (rank, value) polls that rank's entry until it carries e,
// and the values are summed in rank order -- the same bits on every rank, and for two ranks the same as any
// all-reduce.  Slot parity e & 1: a rank writes exchange e + 2's slot only after it has read every rank's e + 1,
// which every rank published after reading e.  A wait that gives up sets *A.err (the next operator call fails).
__global__ __launch_bounds__(1024) void k_peer_scalars(PeerArgs A, long long off, unsigned int e,
                                                       double* __restrict__ v, int count)
{
   __shared__ double s_v[1024];
   const unsigned long long stamp = (unsigned long long)e << 32;
   const size_t slot = (size_t)off + (size_t)(e & 1u) * kPeerScal * 16;
   for (int i = threadIdx.x; i < count; i += 1024) {
      unsigned long long* p = (unsigned long long*)(A.own + slot) + 2 * i;
      const unsigned long long bits = (unsigned long long)__double_as_longlong(v[i]);
      __hip_atomic_store(p, (bits & 0xffffffffull) | stamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(p + 1, (bits >> 32) | stamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
   }
   __syncthreads();  // every thread's reads of v are done before any sum overwrites it
   const int W = A.world;
   const int per = 1024 / W;
   for (int i0 = 0; i0 < count; i0 += per) {
      const int r = threadIdx.x % W, k = threadIdx.x / W, i = i0 + k;
      if (k < per && i < count) {
         const unsigned long long* p = (const unsigned long long*)(peer_rank_buf(A, r) + slot) + 2 * i;
         unsigned long long w0 = 0, w1 = 0;
         for (long long it = 0;; it++) {
            w0 = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            w1 = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((unsigned int)(w0 >> 32) == e && (unsigned int)(w1 >> 32) == e) break;
            if (it >= A.spin) {
               __hip_atomic_store(A.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
               break;
            }
            __builtin_amdgcn_s_sleep(2);
         }
         s_v[k * W + r] = __longlong_as_double((long long)((w0 & 0xffffffffull) | (w1 << 32)));
      }
      __syncthreads();
      if (threadIdx.x < per && i0 + (int)threadIdx.x < count) {
         double sum = 0.0;
         for (int q = 0; q < W; q++) sum = q == 0 ? s_v[threadIdx.x * W] : sum + s_v[threadIdx.x * W + q];
         v[i0 + threadIdx.x] = sum;
      }
      __syncthreads();
   }
}

struct PeerState;
// the communicator the solvers see while the peer exchange is on: small all-reduces through the IPC buffers,
// larger ones through the operator's own communicator
struct PeerComm : Comm {
   PeerState* P = nullptr;
   Comm* base = nullptr;
   int ranks() override { return base->ranks(); }
   int allreduce(double* d_buf, size_t count, hipStream_t s) override;
};

struct PeerState {
   PeerArgs a;
   char* local = nullptr;
   std::vector<char*> opened;  // peers' buffers from hipIpcOpenMemHandle (closed at free)
   char** d_bufs = nullptr;
   unsigned int* h_err = nullptr;
   long long scal_off = 0;     // bytes: the scalar slots after the two grid slots
   unsigned int sepoch = 0;    // scalar exchanges so far (the stamp of the next is sepoch + 1)
   PeerComm pcomm;
};

int PeerComm::allreduce(double* d_buf, size_t count, hipStream_t s)
{
   if (count == 0) return 0;
   if (count > (size_t)kPeerScal) return base->allreduce(d_buf, count, s);
   // 0 is the zeroed buffer's stamp; on wrap skip to 2, which keeps the slot parity alternating (e / e + 2 reuse)
   if (++P->sepoch == 0u) P->sepoch = 2u;
   hipLaunchKernelGGL(k_peer_scalars, dim3(1), dim3(1024), 0, s, P->a, P->scal_off, P->sepoch, d_buf, (int)count);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return 0;
}

struct DistOp {
   // first member: a distributed operator is also the kernel data of the loss (gp_loss.c:143-150 writes
   // _params[0] = f, _params[1] = l and _noise_level = mu into it before calling the kernel setup,
   // Nfft4GPAmdDistGaussianKernel / ...Matern12Kernel, which hands them to the local handle)
   nfft4gp_kernel hdr{};
   int kind = 0;  // 0 rows, 1 components
   void* h = nullptr;
   Comm* comm = nullptr;
   int n_local = 0, n_global = 0, row_begin = 0;
   double* d_grid = nullptr;
   size_t grid_count = 0;
   double* d_tmp = nullptr;  // components, beta != 0: 3 n
   // components: y is all-reduced in `chunks` pieces on a stream of its own, each piece as soon as the
   // interpolation launch that writes it is done, so the all-reduce of piece i overlaps the interpolation
   // of piece i + 1; chunks = 1: one all-reduce after the whole matvec
   int chunks = 4;
   hipStream_t cs = nullptr;
   std::vector<hipEvent_t> ev;
   // timing (Nfft4GPAmdDistTimingEnable): per matvec, event pairs around this rank's kernels before the
   // exchange, the all-reduce(s) and the kernels after it; summed by Nfft4GPAmdDistTimingQuery
   bool timing = false;
   std::vector<hipEvent_t> tpool;        // every timed event, released at the query
   std::vector<std::pair<int, int>> tpairs[3];  // indices into tpool: [0] local before, [1] all-reduce, [2] after
   long long tcount = 0;
   PeerState* peer = nullptr;  // row split: the peer exchange instead of comm->allreduce of the grids
};

void peer_free(PeerState* P)
{
   if (!P) return;
   for (char* b : P->opened)
      if (b) (void)hipIpcCloseMemHandle(b);
   if (P->local) (void)hipFree(P->local);
   if (P->d_bufs) (void)hipFree(P->d_bufs);
   if (P->h_err) (void)hipHostFree(P->h_err);
   delete P;
}

// collective: no rank unmaps or frees its buffer while another's last exchange may still read it
void peer_release(DistOp* D)
{
   if (!D->peer) return;
   (void)hipStreamSynchronize(current_stream());
   double one = 1.0, *d_one = nullptr;
   if (hipMalloc((void**)&d_one, sizeof(double)) == hipSuccess &&
       hipMemcpy(d_one, &one, sizeof(double), hipMemcpyHostToDevice) == hipSuccess)
      (void)D->comm->allreduce(d_one, 1, current_stream());
   (void)hipStreamSynchronize(current_stream());
   (void)hipFree(d_one);
   peer_free(D->peer);
   D->peer = nullptr;
}

// a wait of an earlier exchange gave up (a peer never published): every later call fails
int peer_check(DistOp* D)
{
   if (D->peer && __atomic_load_n(D->peer->h_err, __ATOMIC_ACQUIRE)) {
      fprintf(stderr, "nfft4gp_amd: a peer exchange timed out (a rank did not publish its grids); the distributed "
                      "operator is unusable\n");
      return -1;
   }
   return 0;
}

hipEvent_t timing_event(DistOp* D, int* idx)
{
   hipEvent_t e = nullptr;
   if (hipEventCreate(&e) != hipSuccess) return nullptr;
   *idx = (int)D->tpool.size();
   D->tpool.push_back(e);
   return e;
}

// record an event on stream s (timing on); returns its pool index, or -1
int timing_mark(DistOp* D, hipStream_t s)
{
   if (!D->timing) return -1;
   int i = -1;
   hipEvent_t e = timing_event(D, &i);
   if (!e || hipEventRecord(e, s) != hipSuccess) return -1;
   return i;
}

void timing_pair(DistOp* D, int which, int a, int b)
{
   if (a >= 0 && b >= 0) D->tpairs[which].push_back({a, b});
}

struct ChunkCtx {
   DistOp* D;
   double* y;
   hipStream_t s;
   int i;
};

// after the interpolation of rows [r0, r1): the comm stream waits for it, then all-reduces those rows
int chunk_done(void* vctx, size_t r0, size_t r1)
{
   ChunkCtx* C = (ChunkCtx*)vctx;
   DistOp* D = C->D;
   if ((size_t)C->i + 1 >= D->ev.size()) return -1;
   hipEvent_t e = D->ev[C->i++];
   NFFT4GP_HIP_CHECK(hipEventRecord(e, C->s));
   NFFT4GP_HIP_CHECK(hipStreamWaitEvent(D->cs, e, 0));
   const int a = timing_mark(D, D->cs);
   if (D->comm->allreduce(C->y + r0, r1 - r0, D->cs)) return -1;
   timing_pair(D, 1, a, timing_mark(D, D->cs));
   return 0;
}

int ensure_chunk_stream(DistOp* D)
{
   if (!D->cs) NFFT4GP_HIP_CHECK(hipStreamCreateWithFlags(&D->cs, hipStreamNonBlocking));
   while (D->ev.size() < (size_t)D->chunks + 1) {
      hipEvent_t e;
      NFFT4GP_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      D->ev.push_back(e);
   }
   return 0;
}

int grid_ready(DistOp* D)
{
   const long long g = Nfft4GPAmdShardGridSize(D->h);
   if (g < 0) {
      fprintf(stderr, "nfft4gp_amd: distributed matvec before the kernel setup\n");
      return -1;
   }
   if (D->d_grid && D->grid_count == (size_t)g) return 0;
   if (D->d_grid) (void)hipFree(D->d_grid);
   D->d_grid = nullptr;
   NFFT4GP_HIP_CHECK(hipMalloc((void**)&D->d_grid, sizeof(double) * std::max<size_t>(1, (size_t)g)));
   D->grid_count = (size_t)g;
   return 0;
}

int dist_apply(DistOp* D, int n, int grad, double alpha, double* x, double beta, double* y)
{
   if (!D) return -1;
   const int want = D->kind == 0 ? D->n_local : D->n_global;
   if (n != want) {
      fprintf(stderr, "nfft4gp_amd: distributed matvec size %d, this rank holds %d\n", n, want);
      return -1;
   }
   if ((n > 0 && (!is_device_ptr(x) || !is_device_ptr(y)))) {
      fprintf(stderr, "nfft4gp_amd: the distributed operators take device vectors\n");
      return -1;
   }
   hipStream_t s = current_stream();
   if (D->timing) D->tcount++;
   if (D->kind == 0 && D->peer) {
      if (grid_ready(D) || peer_check(D)) return -1;
      PeerArgs& A = D->peer->a;
      A.epoch++;
      const int e0 = timing_mark(D, s);
      if (shard_spread_peer(D->h, x, A)) return -1;
      const int e1 = timing_mark(D, s);
      if (shard_finish_peer(D->h, A, D->d_grid, grad, alpha, x, beta, y)) return -1;
      const int e3 = timing_mark(D, s);
      timing_pair(D, 0, e0, e1);
      timing_pair(D, 2, e1, e3);  // the exchange is inside the grid kernel: the all-reduce slot stays empty
      return 0;
   }
   if (D->kind == 0) {
      if (grid_ready(D)) return -1;
      const int e0 = timing_mark(D, s);
      if (Nfft4GPAmdShardSpread(D->h, x, D->d_grid)) return -1;
      const int e1 = timing_mark(D, s);
      if (D->comm->allreduce(D->d_grid, D->grid_count, s)) return -1;
      const int e2 = timing_mark(D, s);
      if (Nfft4GPAmdShardFinish(D->h, D->d_grid, grad, alpha, x, beta, y)) return -1;
      const int e3 = timing_mark(D, s);
      timing_pair(D, 0, e0, e1);
      timing_pair(D, 1, e1, e2);
      timing_pair(D, 2, e2, e3);
      return 0;
   }
   const int c0 = timing_mark(D, s);
   const size_t ny = (size_t)n * (grad ? 3 : 1);
   double* out = y;
   if (beta != 0.0) {
      if (!D->d_tmp) NFFT4GP_HIP_CHECK(hipMalloc((void**)&D->d_tmp, sizeof(double) * 3 * std::max<size_t>(1, n)));
      out = D->d_tmp;
   }
   bool chunked = false;
   if (!grad && D->chunks > 1 && n > 0) {
      if (ensure_chunk_stream(D)) return -1;
      ChunkCtx C{D, out, s, 0};
      const int rc = additive_matvec_chunked(D->h, alpha, x, out, D->chunks, &chunk_done, &C);
      if (rc == 0) {
         timing_pair(D, 0, c0, timing_mark(D, s));
         // the stream's later work (the caller's reads of y, the next matvec) waits for the last piece
         NFFT4GP_HIP_CHECK(hipEventRecord(D->ev[C.i], D->cs));
         NFFT4GP_HIP_CHECK(hipStreamWaitEvent(s, D->ev[C.i], 0));
         chunked = true;
      } else if (C.i > 0) {
         return -1;  // failed after some pieces were enqueued
      }
   }
   if (!chunked) {
      const int rc = grad ? Nfft4GPAdditiveNFFTGradMatSymv(D->h, n, alpha, x, 0.0, out)
                          : Nfft4GPAdditiveNFFTMatSymv(D->h, n, alpha, x, 0.0, out);
      if (rc) return -1;
      const int e1 = timing_mark(D, s);
      timing_pair(D, 0, c0, e1);
      if (D->comm->allreduce(out, ny, s)) return -1;
      timing_pair(D, 1, e1, timing_mark(D, s));
   }
   if (beta != 0.0) {
      const int g = (int)std::min<size_t>(4096, (ny + 255) / 256);
      hipLaunchKernelGGL(k_axpby_add, dim3(std::max(g, 1)), dim3(256), 0, s, beta, y, (const double*)D->d_tmp, ny);
      NFFT4GP_HIP_CHECK(hipGetLastError());
   }
   return 0;
}

// ---- row-sharded Nystrom apply ----------------------------------------------------------------------
__global__ void k_dnys_scale(double* __restrict__ w, const double* __restrict__ s, int k, double eta)
{
   const int j = blockIdx.x * blockDim.x + threadIdx.x;
   if (j < k) {
      const double t = w[j];
      w[j] = s[j] * t - t / eta;  // the expression of the one-GPU apply (solvers.hip k_nys_w)
   }
}

struct DistNys {
   NysDev* N = nullptr;  // this rank's rows of U (n = local rows), s, eta, scratch
   Comm* comm = nullptr;
};

}  // namespace

namespace nfft4gp_amd {
// a peer exchange's wait gave up during the work enqueued so far (read after a host sync): the operator's
// results, and a solver's that used it, are not to be trusted
int dist_failed(void* dop)
{
   DistOp* D = (DistOp*)dop;
   return D && peer_check(D) ? 1 : 0;
}

int dist_pcg_info(void* dop, DistPcgInfo& info)
{
   DistOp* D = (DistOp*)dop;
   if (!D) return -1;
   info.n_global = D->n_global;
   info.row_begin = D->kind == 0 ? D->row_begin : 0;
   // with the peer exchange on, the solvers' small all-reduces go through it too (PeerComm)
   // (not under NFFT4GP_AMD_PEER_FAKE_WORLD, whose sums are wrong by design)
   const bool peer_dots = D->peer && D->peer->a.world == D->comm->world;
   info.dot_comm = D->kind == 0 ? (peer_dots ? (Comm*)&D->peer->pcomm : D->comm) : nullptr;
   info.fused_dot = D->kind == 0 && shard_fused_dot_ok(D->h);
   return 0;
}

int dist_matvec_dot(void* dop, const double* d_p, double* d_q, double* d_dot)
{
   DistOp* D = (DistOp*)dop;
   if (!D || D->kind != 0 || grid_ready(D)) return -1;
   if (D->peer) {
      if (peer_check(D)) return -1;
      PeerArgs& A = D->peer->a;
      A.epoch++;
      if (shard_spread_peer(D->h, d_p, A)) return -1;
      return shard_finish_dot_peer(D->h, A, D->d_grid, d_p, d_q, d_dot);
   }
   if (Nfft4GPAmdShardSpread(D->h, d_p, D->d_grid)) return -1;
   if (D->comm->allreduce(D->d_grid, D->grid_count, current_stream())) return -1;
   return shard_finish_dot(D->h, D->d_grid, d_p, d_q, d_dot);
}

// the row-sharded apply (nys.c:115-173 over row shards); implemented with the one-GPU apply's kernels
int nys_apply_rows(NysDev* N, Comm* comm, double* x, const double* rhs, hipStream_t s);
}  // namespace nfft4gp_amd

extern "C" {

int Nfft4GPAmdCommUniqueId(void* id128)
{
   RcclApi& R = rccl();
   if (!R.ok || !id128) return -1;
   ncclUniqueId id;
   const ncclResult_t r = R.get_id(&id);
   if (r != ncclSuccess) {
      fprintf(stderr, "nfft4gp_amd: ncclGetUniqueId: %s\n", R.err(r));
      return -1;
   }
   static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
   memcpy(id128, &id, sizeof(id));
   return 0;
}

// every rank asks this before any rank enters ncclCommInitRank (dist.py all-reduces the answers): a rank
// that would return before the collective init (no device, RCCL not loadable) must not leave the others
// blocked inside it
int Nfft4GPAmdCommRcclAvailable(void)
{
   return (device_ok() && rccl().ok) ? 1 : 0;
}

void* Nfft4GPAmdCommCreateRccl(int rank, int world, const void* id128)
{
   if (!device_ok() || !id128 || world < 1 || rank < 0 || rank >= world) return nullptr;
   RcclApi& R = rccl();
   if (!R.ok) return nullptr;
   ncclUniqueId id;
   memcpy(&id, id128, sizeof(id));
   CommRccl* C = new CommRccl();
   C->rank = rank;
   C->world = world;
   const ncclResult_t r = R.init_rank(&C->c, world, id, rank);
   if (r != ncclSuccess) {
      fprintf(stderr, "nfft4gp_amd: ncclCommInitRank (rank %d of %d): %s\n", rank, world, R.err(r));
      C->c = nullptr;
      delete C;
      return nullptr;
   }
   return C;
}

void* Nfft4GPAmdCommCreateCallback(int rank, int world, Nfft4GPAmdAllreduceFn fn, void* ctx, double* d_stage,
                                   long long capacity)
{
   if (!fn || !d_stage || capacity <= 0 || world < 1 || rank < 0 || rank >= world) return nullptr;
   if (!is_device_ptr(d_stage)) {
      fprintf(stderr, "nfft4gp_amd: the all-reduce staging buffer must be device memory\n");
      return nullptr;
   }
   CommCallback* C = new CommCallback();
   C->rank = rank;
   C->world = world;
   C->fn = fn;
   C->ctx = ctx;
   C->stage = d_stage;
   C->cap = (size_t)capacity;
   return C;
}

int Nfft4GPAmdCommAllreduce(void* comm, double* d_buf, long long count)
{
   if (!comm || count < 0) return -1;
   return ((Comm*)comm)->allreduce(d_buf, (size_t)count, current_stream());
}

void Nfft4GPAmdCommFree(void* comm)
{
   if (!comm) return;
   (void)hipStreamSynchronize(current_stream());
   delete (Comm*)comm;
}

void* Nfft4GPAmdDistCreate(void* handle, int kind, void* comm)
{
   int nl = 0, ng = 0, rb = 0;
   if (!comm || (kind != 0 && kind != 1) || additive_rows(handle, &nl, &ng, &rb)) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdDistCreate needs an additive handle, kind 0 or 1 and a communicator\n");
      return nullptr;
   }
   if (kind == 1 && nl != ng) {
      fprintf(stderr, "nfft4gp_amd: a component-sharded operator needs a whole-row handle\n");
      return nullptr;
   }
   DistOp* D = new DistOp();
   D->kind = kind;
   D->h = handle;
   D->comm = (Comm*)comm;
   D->n_local = nl;
   D->n_global = ng;
   D->row_begin = rb;
   if (kind == 0 && rb % 16 != 0)
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdDistCreate: row shard starts at %d, not a multiple of 16: the 1-D layout's "
                      "offset words then differ from the whole handle's, so the operator depends on the split by "
                      "rounding (dist.row_range's shards start at multiples of 16)\n", rb);
   const nfft4gp_kernel* kd = (const nfft4gp_kernel*)handle;
   D->hdr._params[0] = kd->_params[0];
   D->hdr._params[1] = kd->_params[1];
   D->hdr._noise_level = kd->_noise_level;
   return D;
}

void Nfft4GPAmdDistFree(void* dop)
{
   DistOp* D = (DistOp*)dop;
   if (!D) return;
   (void)hipStreamSynchronize(current_stream());
   if (D->cs) (void)hipStreamSynchronize(D->cs);
   peer_release(D);
   if (D->d_grid) (void)hipFree(D->d_grid);
   if (D->d_tmp) (void)hipFree(D->d_tmp);
   for (hipEvent_t e : D->ev) (void)hipEventDestroy(e);
   for (hipEvent_t e : D->tpool) (void)hipEventDestroy(e);
   if (D->cs) (void)hipStreamDestroy(D->cs);
   delete D;
}

// func_kernel of a distributed operator (kernels.h:49): the hyperparameters written into its header go to
// the local handle, whose own setup runs (nfft_interface.c:676-794); *Kp = *dKp = the operator, so the
// loss's matvec / grad-matvec calls reach Nfft4GPAmdDistMatSymv / ...GradMatSymv with it
static int dist_kernel_setup(void* str, int kernel, double** Kp, double** dKp)
{
   DistOp* D = (DistOp*)str;
   if (!D || !Kp || !dKp) {
      printf("Error: NFFT kernel requires Kp and dKp to be not NULL.\n");
      return -1;
   }
   nfft4gp_kernel* kd = (nfft4gp_kernel*)D->h;
   kd->_params[0] = D->hdr._params[0];
   kd->_params[1] = D->hdr._params[1];
   kd->_noise_level = D->hdr._noise_level;
   double *K = nullptr, *dK = nullptr;
   const int rc = kernel == 0 ? Nfft4GPNFFTAdditiveKernelGaussianKernel(D->h, nullptr, D->n_local, D->n_local, 0,
                                                                        nullptr, 0, nullptr, 0, &K, &dK)
                              : Nfft4GPNFFTAdditiveKernelMatern12Kernel(D->h, nullptr, D->n_local, D->n_local, 0,
                                                                        nullptr, 0, nullptr, 0, &K, &dK);
   if (rc) return -1;
   *Kp = (double*)D;
   *dKp = (double*)D;
   return 0;
}

int Nfft4GPAmdDistGaussianKernel(void* str, double* data, int n, int ldim, int d, int* permr, int kr, int* permc,
                                 int kc, double** Kp, double** dKp)
{
   (void)data, (void)n, (void)ldim, (void)d, (void)permr, (void)kr, (void)permc, (void)kc;
   return dist_kernel_setup(str, 0, Kp, dKp);
}

int Nfft4GPAmdDistMatern12Kernel(void* str, double* data, int n, int ldim, int d, int* permr, int kr, int* permc,
                                 int kc, double** Kp, double** dKp)
{
   (void)data, (void)n, (void)ldim, (void)d, (void)permr, (void)kr, (void)permc, (void)kc;
   return dist_kernel_setup(str, 1, Kp, dKp);
}

int Nfft4GPAmdCommRanks(void* comm)
{
   if (!comm) return -1;
   return ((Comm*)comm)->ranks();
}

static void dist_timing_reset(DistOp* D)
{
   for (hipEvent_t e : D->tpool) (void)hipEventDestroy(e);
   D->tpool.clear();
   for (auto& v : D->tpairs) v.clear();
   D->tcount = 0;
}

int Nfft4GPAmdDistTimingEnable(void* dop, int enable)
{
   DistOp* D = (DistOp*)dop;
   if (!D) return -1;
   NFFT4GP_HIP_CHECK(hipStreamSynchronize(current_stream()));
   if (D->cs) NFFT4GP_HIP_CHECK(hipStreamSynchronize(D->cs));
   if (enable) dist_timing_reset(D);
   D->timing = enable != 0;
   return 0;
}

int Nfft4GPAmdDistTimingQuery(void* dop, double* ms, long long* cnt)
{
   DistOp* D = (DistOp*)dop;
   if (!D || !ms) return -1;
   NFFT4GP_HIP_CHECK(hipStreamSynchronize(current_stream()));
   if (D->cs) NFFT4GP_HIP_CHECK(hipStreamSynchronize(D->cs));
   for (int w = 0; w < 3; w++) {
      double t = 0.0;
      for (const auto& p : D->tpairs[w]) {
         float f = 0.0f;
         NFFT4GP_HIP_CHECK(hipEventElapsedTime(&f, D->tpool[p.first], D->tpool[p.second]));
         t += f;
      }
      ms[w] = t;
   }
   if (cnt) *cnt = D->tcount;
   return 0;
}

// The peer-memory exchange for a row-sharded operator (collective): each rank exports one
// buffer (two grid slots + a flag per window) with hipIpcGetMemHandle, the handles travel over the
// communicator (one byte per double, so the sum is exact), every rank opens the others'.  From then on a
// matvec publishes its grids into its own slot and the grid kernel sums all ranks' slots in rank order (every
// rank holds the same bits) -- no all-reduce.  Returns 0 (on), 1 (not applicable: component split or
// multi-feature windows -- the same answer on every rank) or -1 (a rank could not allocate, export or open:
// every rank keeps the communicator's all-reduce).
int Nfft4GPAmdDistPeerEnable(void* dop)
{
   DistOp* D = (DistOp*)dop;
   if (!D) return -1;
   if (D->peer) return 0;
   if (D->kind != 0 || !shard_peer_ok(D->h)) return 1;
   if (grid_ready(D)) return -1;
   Comm* C = D->comm;
   const int world = C->world, rank = C->rank;
   if (world < 1 || world > kPeerMaxWorld) return 1;
   hipStream_t s = current_stream();
   PeerState* P = new PeerState();
   const size_t gcount = D->grid_count;
   // two grid slots of (low, high) words with the epoch (nfft_kernels.hip), then two scalar slots (k_peer_scalars)
   const size_t bytes = 2 * gcount * 16 + 2 * (size_t)kPeerScal * 16;
   constexpr size_t HB = sizeof(hipIpcMemHandle_t);
   // uncached device memory (hipDeviceMallocUncached, MTYPE UC): every store and load of the exchange words, the
   // owner's and the peers' over xGMI, goes to the owning device's memory, so no cache level of either device can
   // hold a stale epoch word; the coherence of the exchange then needs no rule about which caches a system-scope
   // access bypasses on coarse-grained memory.  NFFT4GP_AMD_PEER_CACHED=1: plain hipMalloc (A/B)
   static const bool cached = getenv("NFFT4GP_AMD_PEER_CACHED") && atoi(getenv("NFFT4GP_AMD_PEER_CACHED")) != 0;
   bool ok = (cached ? hipMalloc((void**)&P->local, bytes)
                     : hipExtMallocWithFlags((void**)&P->local, bytes, hipDeviceMallocUncached)) == hipSuccess &&
             hipMemsetAsync(P->local, 0, bytes, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
   hipIpcMemHandle_t mine;
   memset(&mine, 0, sizeof(mine));
   if (ok && world > 1 && hipIpcGetMemHandle(&mine, P->local) != hipSuccess) {
      fprintf(stderr, "nfft4gp_amd: hipIpcGetMemHandle refused the exchange buffer\n");
      ok = false;
   }
   ok = ok && hipHostMalloc((void**)&P->h_err, sizeof(unsigned int), hipHostMallocMapped) == hipSuccess;
   if (ok) *P->h_err = 0u;
   ok = ok && hipMalloc((void**)&P->d_bufs, sizeof(char*) * world) == hipSuccess;
   // round 1: the handles and whether every rank got this far
   std::vector<double> hx((size_t)world * HB + 1, 0.0);
   for (size_t b = 0; b < HB; b++) hx[(size_t)rank * HB + b] = (double)((const unsigned char*)&mine)[b];
   hx.back() = ok ? 0.0 : 1.0;
   double* dx = nullptr;
   // every rank enters both all-reduces whatever failed locally (a rank that skipped one would leave the
   // others waiting in it); only a rank that cannot even hold the few-KB exchange buffer returns early
   if (hipMalloc((void**)&dx, sizeof(double) * hx.size()) != hipSuccess) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdDistPeerEnable: no device memory for the handle exchange\n");
      peer_free(P);
      return -1;
   }
   auto agree = [&](std::vector<double>& v) {
      bool ok = hipMemcpy(dx, v.data(), sizeof(double) * v.size(), hipMemcpyHostToDevice) == hipSuccess;
      if (!ok) (void)hipMemset(dx + v.size() - 1, 0, sizeof(double));  // still the same collective
      ok = C->allreduce(dx, v.size(), s) == 0 && ok;
      ok = hipMemcpyAsync(v.data(), dx, sizeof(double) * v.size(), hipMemcpyDeviceToHost, s) == hipSuccess &&
           hipStreamSynchronize(s) == hipSuccess && ok;
      if (!ok) v.back() = 1.0;  // this rank's copy of the answer is unusable: report a failure
      return true;
   };
   bool all = agree(hx) && hx.back() == 0.0;
   std::vector<char*> bufs(world, nullptr);
   P->opened.assign(world, nullptr);
   bool mine_ok = all;
   for (int r = 0; r < world && mine_ok; r++) {
      if (r == rank) {
         bufs[r] = P->local;
         continue;
      }
      hipIpcMemHandle_t h;
      for (size_t b = 0; b < HB; b++) ((unsigned char*)&h)[b] = (unsigned char)hx[(size_t)r * HB + b];
      void* ptr = nullptr;
      if (hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
         fprintf(stderr, "nfft4gp_amd: hipIpcOpenMemHandle refused rank %d's exchange buffer\n", r);
         mine_ok = false;
         break;
      }
      P->opened[r] = (char*)ptr;
      bufs[r] = (char*)ptr;
   }
   // timing probe only (one process): the exchange kernels read this rank's own slot `k` times, as k ranks would
   int fake = 0;
   if (world == 1 && mine_ok)
      if (const char* e = getenv("NFFT4GP_AMD_PEER_FAKE_WORLD")) fake = std::max(0, std::min(kPeerMaxWorld, atoi(e)));
   if (fake > 1) {
      fprintf(stderr, "nfft4gp_amd: NFFT4GP_AMD_PEER_FAKE_WORLD=%d: the exchange sums this rank's slot %d times "
                      "(timing only; the results are wrong)\n", fake, fake);
      bufs.assign(fake, P->local);
   }
   mine_ok = mine_ok && hipMemcpy(P->d_bufs, bufs.data(), sizeof(char*) * std::min<size_t>(bufs.size(), world),
                                  hipMemcpyHostToDevice) == hipSuccess;
   if (fake > 1) {
      (void)hipFree(P->d_bufs);
      P->d_bufs = nullptr;
      mine_ok = hipMalloc((void**)&P->d_bufs, sizeof(char*) * fake) == hipSuccess &&
                hipMemcpy(P->d_bufs, bufs.data(), sizeof(char*) * fake, hipMemcpyHostToDevice) == hipSuccess;
   }
   // round 2: every rank opened every buffer
   std::vector<double> ok2(hx.size(), 0.0);
   ok2.back() = mine_ok ? 0.0 : 1.0;
   all = agree(ok2) && ok2.back() == 0.0;
   (void)hipFree(dx);
   if (!all) {
      peer_free(P);
      return -1;
   }
   unsigned int* d_err = nullptr;
   if (hipHostGetDevicePointer((void**)&d_err, P->h_err, 0) != hipSuccess) d_err = P->h_err;
   // ~16 s of polls (each a system-scope load and an s_sleep): far above the host-side skew of ranks that
   // enqueue the same solve, short enough that a dead peer ends the call
   long long spin = 1ll << 23;
   if (const char* e = getenv("NFFT4GP_AMD_PEER_SPIN")) spin = std::max(1ll, atoll(e));
   P->a.bufs = P->d_bufs;
   for (int r = 0; r < kPeerInline && r < (int)bufs.size(); r++) P->a.inl[r] = bufs[r];
   P->a.own = P->local;
   P->a.world = fake > 1 ? fake : world;
   P->a.epoch = 0u;
   P->a.err = d_err;
   P->a.slot_doubles = (long long)gcount;
   P->a.spin = spin;
   P->scal_off = (long long)(2 * gcount * 16);
   P->pcomm.P = P;
   P->pcomm.base = C;
   P->pcomm.rank = C->rank;
   P->pcomm.world = C->world;
   D->peer = P;
   return 0;
}

// back to the communicator's all-reduce (collective); the operator is usable again after a timed-out wait
int Nfft4GPAmdDistPeerDisable(void* dop)
{
   DistOp* D = (DistOp*)dop;
   if (!D) return -1;
   peer_release(D);
   return 0;
}

int Nfft4GPAmdDistPeerActive(void* dop)
{
   DistOp* D = (DistOp*)dop;
   return D ? (D->peer ? 1 : 0) : -1;
}

int Nfft4GPAmdDistSetChunks(void* dop, int chunks)
{
   DistOp* D = (DistOp*)dop;
   if (!D || chunks < 1 || chunks > 256) return -1;
   (void)hipStreamSynchronize(current_stream());
   D->chunks = chunks;
   return 0;
}

int Nfft4GPAmdDistCheck(void* dop)
{
   if (!dop) return -1;
   NFFT4GP_HIP_CHECK(hipStreamSynchronize(current_stream()));
   return peer_check((DistOp*)dop);
}

int Nfft4GPAmdDistMatSymv(void* dop, int n, double alpha, double* x, double beta, double* y)
{
   return dist_apply((DistOp*)dop, n, 0, alpha, x, beta, y);
}

int Nfft4GPAmdDistGradMatSymv(void* dop, int n, double alpha, double* x, double beta, double* y)
{
   return dist_apply((DistOp*)dop, n, 1, alpha, x, beta, y);
}

void* Nfft4GPAmdNysShard(void* nys, int row_begin, int row_end, void* comm)
{
   NysDev* S = (NysDev*)nys;
   if (!S || !comm || row_begin < 0 || row_end > S->n || row_begin > row_end) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdNysShard: invalid rows [%d, %d)\n", row_begin, row_end);
      return nullptr;
   }
   hipStream_t s = current_stream();
   NysDev* N = new NysDev();
   N->n = row_end - row_begin;
   N->k = S->k;
   N->eta = S->eta;
   const size_t nl = (size_t)N->n;
   if (hipMalloc((void**)&N->U, sizeof(double) * std::max<size_t>(1, nl * N->k)) != hipSuccess ||
       hipMalloc((void**)&N->s, sizeof(double) * std::max(1, N->k)) != hipSuccess || nys_alloc_scratch(N)) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdNysShard: allocation failed\n");
      nys_free(N);
      return nullptr;
   }
   // rows [row_begin, row_end) of every column of the n x k column-major U
   if ((nl && hipMemcpy2DAsync(N->U, sizeof(double) * nl, S->U + row_begin, sizeof(double) * (size_t)S->n,
                               sizeof(double) * nl, (size_t)N->k, hipMemcpyDeviceToDevice, s) != hipSuccess) ||
       hipMemcpyAsync(N->s, S->s, sizeof(double) * N->k, hipMemcpyDeviceToDevice, s) != hipSuccess ||
       hipStreamSynchronize(s) != hipSuccess) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdNysShard: copy failed\n");
      nys_free(N);
      return nullptr;
   }
   DistNys* D = new DistNys();
   D->N = N;
   D->comm = (Comm*)comm;
   return D;
}

// Nfft4GPPrecondNysSetupWithKernel (nys.c:518-660, K11 on the landmarks) split over the row shards of a
// distributed operator: every rank forms the panel of its own rows, U1 = Kp L^{-T} and its partial Gram
// U1^T U1; ONE k x k all-reduce sums the Gram (matops.c:65-137 is a sum over rows); rank 0's k x k factors
// (L^{-T}, the eigenbasis) are broadcast so every rank scales its rows alike.  No rank holds more than its
// n/N rows of the n x k panel.
void* Nfft4GPAmdNysShardSetupAdditive(void* dop, const int* perm, int k, int k11_mode)
{
   DistOp* D = (DistOp*)dop;
   if (!D || D->kind != 0 || !perm || (k11_mode != 0 && k11_mode != 1)) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdNysShardSetupAdditive needs a row-sharded operator (kind 0), the "
                      "landmark order and k11_mode 0 or 1\n");
      return nullptr;
   }
   NysDev* N = nys_setup_shard(D->h, perm, k, k11_mode, D->comm);
   if (!N) return nullptr;
   DistNys* R = new DistNys();
   R->N = N;
   R->comm = D->comm;
   return R;
}

int Nfft4GPAmdDistNysSolve(void* dnys, int n, double* x, double* rhs)
{
   DistNys* D = (DistNys*)dnys;
   if (!D || n != D->N->n) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdDistNysSolve: size %d, this rank holds %d rows\n", n,
              D ? D->N->n : -1);
      return -1;
   }
   if (n > 0 && (!is_device_ptr(x) || !is_device_ptr(rhs))) {
      fprintf(stderr, "nfft4gp_amd: Nfft4GPAmdDistNysSolve takes device vectors\n");
      return -1;
   }
   return nys_apply_rows(D->N, D->comm, x, rhs, current_stream());
}

void Nfft4GPAmdDistNysFree(void* dnys)
{
   DistNys* D = (DistNys*)dnys;
   if (!D) return;
   nys_free(D->N);
   delete D;
}

}  // extern "C"

namespace nfft4gp_amd {
// k_dnys_scale is this file's; the U passes are solvers.hip's (nys_gemv_t_local / nys_u_local)
int nys_ut_local(NysDev* N, const double* rhs, double* w, hipStream_t s);
int nys_u_local(NysDev* N, const double* w, const double* rhs, double* x, hipStream_t s);

int nys_apply_rows(NysDev* N, Comm* comm, double* x, const double* rhs, hipStream_t s)
{
   // w = U_loc^T r_loc (k), summed over the row shards, then w = s w - w / eta, then x = U_loc w + r / eta
   if (nys_ut_local(N, rhs, N->w, s)) return -1;
   if (comm->allreduce(N->w, (size_t)N->k, s)) return -1;
   hipLaunchKernelGGL(k_dnys_scale, dim3((N->k + 255) / 256), dim3(256), 0, s, N->w, (const double*)N->s, N->k, N->eta);
   NFFT4GP_HIP_CHECK(hipGetLastError());
   return nys_u_local(N, N->w, rhs, x, s);
}
}  // namespace nfft4gp_amd
