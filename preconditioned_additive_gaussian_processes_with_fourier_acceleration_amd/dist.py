"""Multi-GPU additive operator, Nystrom apply and CG (one process per GPU).

The reference is single-process (SRC/external/nfft_interface.c:796-817 runs the components one after
another; SRC/solvers/pcg.c works on whole vectors).  The operator splits two ways:

* rows (``partition="rows"``): every rank spreads its own n/N points for all windows, the nw x 64
  oversampled grids (16 KB at nw = 32) are summed with ONE all-reduce, every rank interpolates its rows;
  CG vectors stay row-sharded and every dot is summed over the ranks.
* components (``partition="components"``, the split BASELINE configs[3] names): every rank holds a
  contiguous block of the windows for all points, y (n doubles) is all-reduced, vectors are replicated.

``DistributedAdditiveKernel`` / ``RowShardedNystrom`` are the library's distributed operators
(dist.hip): the all-reduces are enqueued by the C++ code on the library stream (RCCL) and
``solvers.pcg`` drives them through the reference's own Nfft4GPSolverPcg entry point, with the
scalars and control decisions on the device (no per-iteration host synchronisation).

``RowShardedAdditiveKernel`` is the host-controlled mirror of the same CG over any engine with
``shard_spread`` / ``shard_finish`` (the CPU tests drive it with the numpy replay of the HIP kernels).
"""
from __future__ import annotations

import math

import numpy as np


def row_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous row block of `rank` (ceil-divided and rounded up to a multiple of 16, so every shard starts
    at a multiple of 16 and its points keep their low 4 local-index bits -- and the sub-quantum offsets the layout
    derives from them -- exactly as in the whole handle; the last ranks may get fewer or zero rows)."""
    per = (n + world - 1) // world
    per = (per + 15) // 16 * 16
    return min(n, rank * per), min(n, (rank + 1) * per)


def component_range(nw: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block of windows of `rank` (balanced: sizes differ by at most one; every rank gets at
    least one window when nw >= world).  Config D: 32 windows on 8 GPUs -> 4 per GPU."""
    return rank * nw // world, (rank + 1) * nw // world


class Communicator:
    """The process group of the library's distributed operators (Nfft4GPAmdComm*).

    ``Communicator.rccl()``: RCCL over xGMI, one communicator per process created from an id that rank 0
    makes and torch.distributed broadcasts; all-reduces are enqueued on the library stream.
    ``Communicator.callback()``: the all-reduce of a torch.distributed group through a device staging
    buffer -- gloo (several ranks on one GPU, which RCCL refuses) sums a host copy, nccl sums the staging
    buffer itself with torch's own RCCL communicator; it synchronises -- a test and fallback path, not a
    fast one."""

    def __init__(self, h, rank, world, keep=()):
        self.h, self.rank, self.world, self._keep = h, rank, world, keep

    @staticmethod
    def _bind_stream():
        import torch
        from . import _lib
        _lib.lib().Nfft4GPAmdSetStream(torch.cuda.current_stream().cuda_stream)

    @classmethod
    def rccl(cls, group=None):
        import torch
        import torch.distributed as dist
        from . import _lib
        L = _lib.lib()
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        on_device = dist.get_backend(group) == "nccl"
        dev = "cuda" if on_device else "cpu"
        # every rank learns whether every rank can create a communicator BEFORE any of them enters
        # ncclCommInitRank: a rank that cannot (no device, RCCL not loadable) would otherwise return early
        # while the others wait inside the collective init for it
        notready = torch.tensor([0.0 if L.Nfft4GPAmdCommRcclAvailable() == 1 else 1.0], dtype=torch.float64,
                                device=dev)
        dist.all_reduce(notready, group=group)
        if float(notready.item()) != 0.0:
            raise RuntimeError("RCCL is not available on %d rank(s) (see stderr)" % int(notready.item()))
        # the 128-byte id plus a status byte, so that a failure on rank 0 reaches every rank through the same
        # broadcast (no rank is left waiting in a collective the others never enter)
        buf = np.zeros(129, dtype=np.uint8)
        if rank == 0:
            buf[128] = 1 if L.Nfft4GPAmdCommUniqueId(buf.ctypes.data) == 0 else 0
        t = torch.from_numpy(buf)
        if on_device:
            t = t.cuda()
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        buf = np.ascontiguousarray(t.cpu().numpy())
        if buf[128] != 1:
            raise RuntimeError("Nfft4GPAmdCommUniqueId failed on rank 0 (RCCL not loadable, see its stderr)")
        cls._bind_stream()
        h = L.Nfft4GPAmdCommCreateRccl(rank, world, buf.ctypes.data)
        # every rank learns whether every rank has a communicator before any of them uses one
        ok = torch.tensor([0.0 if h else 1.0], dtype=torch.float64, device=dev)
        dist.all_reduce(ok, group=group)
        if float(ok.item()) != 0.0:
            if h:
                L.Nfft4GPAmdCommFree(h)
            raise RuntimeError("Nfft4GPAmdCommCreateRccl failed on %d rank(s) (see stderr)" % int(ok.item()))
        return cls(h, rank, world)

    @classmethod
    def callback(cls, group=None, capacity: int = 1 << 20):
        import torch
        import torch.distributed as dist
        from . import _lib
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        stage = torch.zeros(capacity, dtype=torch.float64, device="cuda")
        on_device = dist.get_backend(group) == "nccl"

        def _allreduce(ctx, ptr, count):
            try:
                if on_device:  # torch's RCCL communicator, in place, on torch's current stream
                    dist.all_reduce(stage[:count], group=group)
                    torch.cuda.current_stream().synchronize()
                    return 0
                host = stage[:count].cpu()  # on torch's current stream = the library stream
                dist.all_reduce(host, group=group)
                stage[:count].copy_(host)
                return 0
            except Exception:  # a C caller cannot take a Python exception
                return -1

        fn = _lib.ALLREDUCE(_allreduce)
        cls._bind_stream()
        h = _lib.lib().Nfft4GPAmdCommCreateCallback(rank, world, fn, None, stage.data_ptr(), capacity)
        if not h:
            raise RuntimeError("Nfft4GPAmdCommCreateCallback failed")
        return cls(h, rank, world, keep=(stage, fn))

    def allreduce(self, t):
        """In-place sum of a float64 device tensor over the ranks."""
        from . import _lib
        if _lib.lib().Nfft4GPAmdCommAllreduce(self.h, t.data_ptr(), t.numel()) != 0:
            raise RuntimeError("Nfft4GPAmdCommAllreduce failed")
        return t

    def ranks(self) -> int:
        """The ranks the backend itself reports (ncclCommCount for RCCL; the group size for a callback)."""
        from . import _lib
        return int(_lib.lib().Nfft4GPAmdCommRanks(self.h))

    def free(self):
        if getattr(self, "h", None):
            from . import _lib
            _lib.lib().Nfft4GPAmdCommFree(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DistributedAdditiveKernel:
    """The additive operator split over a Communicator (Nfft4GPAmdDist*, dist.hip).

    rows:       x, y hold this rank's rows [row_begin, row_end); ``n`` is their count.
    components: this rank's windows [comp_begin, comp_end) for all n points, x and y whole (replicated).
    ``solvers.pcg(self, b, x)`` runs Nfft4GPSolverPcg on it (device-controlled, dots summed over the ranks
    for rows); ``solvers.fgmres``, ``solvers.logdet`` and ``gp.gp_loss(..., op=self)`` run the reference's
    FGMRES, Lanczos quadrature and GP loss on it the same way (krylov.hip, every rank collectively)."""

    def __init__(self, data, windows, nwindows: int, dwindows: int, comm: Communicator, partition: str = "rows"):
        from . import _lib
        from .nfft import NFFTAdditiveKernel
        data = np.asfortranarray(np.asarray(data, dtype=np.float64))
        n = data.shape[0]
        self.comm, self.partition = comm, partition
        self.n_global, self.nwindows = n, nwindows
        L = _lib.lib()
        if partition == "rows":
            self.row_begin, self.row_end = row_range(n, comm.rank, comm.world)
            self.comp_begin, self.comp_end = 0, nwindows
            self.local = NFFTAdditiveKernel(data, windows, nwindows, dwindows, shard=(self.row_begin, self.row_end))
            kind = 0
        elif partition == "components":
            if nwindows < comm.world:
                raise ValueError(f"{nwindows} windows cannot be split over {comm.world} ranks")
            self.row_begin, self.row_end = 0, n
            self.comp_begin, self.comp_end = component_range(nwindows, comm.rank, comm.world)
            win = np.asarray(windows, dtype=np.int32).reshape(nwindows, dwindows)[self.comp_begin:self.comp_end]
            self.local = NFFTAdditiveKernel(data, win, self.comp_end - self.comp_begin, dwindows)
            if L.Nfft4GPAmdAdditiveComponentShard(self.local.h, nwindows, int(comm.rank == 0)) != 0:
                raise RuntimeError("Nfft4GPAmdAdditiveComponentShard failed")
            kind = 1
        else:
            raise ValueError("partition is 'rows' or 'components'")
        self.n = self.row_end - self.row_begin
        self.h = L.Nfft4GPAmdDistCreate(self.local.h, kind, comm.h)
        if not self.h:
            raise RuntimeError("Nfft4GPAmdDistCreate failed")

    def setup(self, kernel=0, f=None, l=None, mu=None) -> int:
        return self.local.setup(kernel, f, l, mu)

    def _apply(self, name, x, alpha, beta, y, mult):
        from . import _lib
        from .nfft import _check_len, _empty_like, _ptr
        _check_len("x", x, self.n)
        if y is None:
            y = _empty_like(x, mult * self.n)
        _check_len("y", y, mult * self.n)
        if getattr(_lib.lib(), name)(self.h, self.n, float(alpha), _ptr(x)[0], float(beta), _ptr(y)[0]) != 0:
            raise RuntimeError(f"{name} failed")
        return y

    def matsymv(self, x, alpha=1.0, beta=0.0, y=None):
        return self._apply("Nfft4GPAmdDistMatSymv", x, alpha, beta, y, 1)

    def gradmatsymv(self, x, alpha=1.0, beta=0.0, y=None):
        return self._apply("Nfft4GPAmdDistGradMatSymv", x, alpha, beta, y, 3)

    def enable_peer(self) -> bool:
        """Row split, 1-D windows: exchange the grids through peer memory instead of the communicator's
        all-reduce (Nfft4GPAmdDistPeerEnable; collective, after setup).  False when it does not apply or some
        rank could not export / open its buffer (then every rank keeps the all-reduce).  With it on, free() is
        collective."""
        from . import _lib
        return _lib.lib().Nfft4GPAmdDistPeerEnable(self.h) == 0

    def disable_peer(self):
        """Back to the communicator's all-reduce (collective)."""
        from . import _lib
        if _lib.lib().Nfft4GPAmdDistPeerDisable(self.h) != 0:
            raise RuntimeError("Nfft4GPAmdDistPeerDisable failed")

    def check(self):
        """Synchronise and raise if a peer exchange of this operator timed out in the work enqueued so far
        (Nfft4GPAmdDistCheck): its results are then not to be used."""
        from . import _lib
        if _lib.lib().Nfft4GPAmdDistCheck(self.h) != 0:
            raise RuntimeError("a peer exchange of the distributed operator timed out (Nfft4GPAmdDistCheck)")

    @property
    def peer_active(self) -> bool:
        from . import _lib
        return bool(self.h) and _lib.lib().Nfft4GPAmdDistPeerActive(self.h) == 1

    def timing(self, on: bool = True):
        """Per-rank hipEvent timing of every matvec (Nfft4GPAmdDistTimingEnable; enabling resets)."""
        from . import _lib
        if _lib.lib().Nfft4GPAmdDistTimingEnable(self.h, int(bool(on))) != 0:
            raise RuntimeError("Nfft4GPAmdDistTimingEnable failed")

    def timing_query(self) -> dict:
        """Milliseconds per timed matvec of this rank's kernels before the exchange, the all-reduce(s) and the
        kernels after it, and the number of matvecs timed."""
        import ctypes as C
        from . import _lib
        ms = (C.c_double * 3)()
        cnt = C.c_longlong()
        if _lib.lib().Nfft4GPAmdDistTimingQuery(self.h, ms, C.byref(cnt)) != 0:
            raise RuntimeError("Nfft4GPAmdDistTimingQuery failed")
        k = max(cnt.value, 1)
        return {"local_before_ms": ms[0] / k, "allreduce_ms": ms[1] / k, "local_after_ms": ms[2] / k,
                "matvecs": cnt.value}

    @property
    def matvec_fnptr(self) -> int:
        from . import _lib
        return _lib.fnptr("Nfft4GPAmdDistMatSymv")

    @property
    def gradmatvec_fnptr(self) -> int:
        from . import _lib
        return _lib.fnptr("Nfft4GPAmdDistGradMatSymv")

    def free(self):
        from . import _lib
        if getattr(self, "h", None):
            _lib.lib().Nfft4GPAmdDistFree(self.h)
            self.h = None
        if getattr(self, "local", None) is not None:
            self.local.free()
            self.local = None

    def __del__(self):
        try:
            # with the peer exchange on, the free is collective: never from the collector of one rank alone
            if not self.peer_active:
                self.free()
        except Exception:
            pass


class RowShardedNystrom:
    """Rows [row_begin, row_end) of a NystromPrecond's U (Nfft4GPAmdNysShard): the apply of nys.c:115-173
    as a local U^T r, a k-vector all-reduce and a local U w + r / eta."""

    def __init__(self, nys, row_begin: int, row_end: int, comm: Communicator):
        from . import _lib
        self.n, self.k, self.comm = row_end - row_begin, nys.k, comm
        self.h = _lib.lib().Nfft4GPAmdNysShard(nys.h, int(row_begin), int(row_end), comm.h)
        if not self.h:
            raise RuntimeError("Nfft4GPAmdNysShard failed")

    @classmethod
    def setup(cls, op: "DistributedAdditiveKernel", perm, k: int, k11: str = "landmarks"):
        """The setup itself split over the rows (Nfft4GPAmdNysShardSetupAdditive, nys.c:518-660): every rank
        forms the panel of its own rows and its partial Gram, one k x k all-reduce sums the Gram, and no
        rank holds more than its rows of U.  ``op``: a row-partitioned operator after its kernel setup;
        ``perm``: the global landmark order (its first k entries), the same on every rank."""
        from . import _lib
        if op.partition != "rows":
            raise ValueError("the sharded Nystrom setup splits rows: use a partition='rows' operator")
        self = cls.__new__(cls)
        self.n, self.k, self.comm = op.n, int(k), op.comm
        p = np.ascontiguousarray(np.asarray(perm, dtype=np.int32))
        self.h = _lib.lib().Nfft4GPAmdNysShardSetupAdditive(op.h, p.ctypes.data, int(k),
                                                            {"reference": 0, "landmarks": 1}[k11])
        if not self.h:
            raise RuntimeError("Nfft4GPAmdNysShardSetupAdditive failed (see stderr)")
        return self

    def solve(self, x, rhs):
        from . import _lib
        from .nfft import _check_len, _ptr
        _check_len("x", x, self.n)
        _check_len("rhs", rhs, self.n)
        if _lib.lib().Nfft4GPAmdDistNysSolve(self.h, self.n, _ptr(x)[0], _ptr(rhs)[0]) != 0:
            raise RuntimeError("Nfft4GPAmdDistNysSolve failed")
        return x

    @property
    def solve_fnptr(self) -> int:
        from . import _lib
        return _lib.fnptr("Nfft4GPAmdDistNysSolve")

    def free(self):
        from . import _lib
        if getattr(self, "h", None):
            _lib.lib().Nfft4GPAmdDistNysFree(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class RowShardedAfn:
    """Rows [row_begin, row_end) of an AFN apply (Nfft4GPAmdAfnShard, afn.c:82-143 over row shards): this rank's
    landmarks, the K12 columns of its Schur points and their rows of the Schur FSAI; an apply exchanges two
    k-vectors (and, with the Schur FSAI, the Schur vector before each sparse product).  ``afn``: an
    AfnPrecond, or a PrecondAFN whose estimate built the AFN itself."""

    def __init__(self, afn, row_begin: int, row_end: int, comm: Communicator):
        import ctypes as C
        from . import _lib
        L = _lib.lib()
        h = afn.h
        if hasattr(afn, "KINDS"):  # a PrecondAFN: its AFN apply object, if that is what it built
            a = C.c_void_p()
            L.Nfft4GPAmdPrecondAFNInfo(afn.h, None, None, C.byref(a), None)
            if not a.value:
                raise ValueError(f"the PrecondAFN built a {afn.kind}, not an AFN")
            h = a.value
        self.n, self.comm = row_end - row_begin, comm
        self.h = L.Nfft4GPAmdAfnShard(h, int(row_begin), int(row_end), comm.h)
        if not self.h:
            raise RuntimeError("Nfft4GPAmdAfnShard failed (see stderr)")

    @classmethod
    def setup(cls, X, k: int, comm: Communicator, row_begin: int, row_end: int, perm_opt: str = "fps", perm=None,
              schur: str = "fsai", schur_lfil: int = 20, kernel: int = 0, op=None, f: float = 1.0, l: float = 1.0,
              mu: float = 0.01):
        """Nfft4GPAmdAfnShardSetup: the same row shard set up on this rank alone, every rank collectively, with
        no full AFN on any rank (afn.c:161-489 split by rows): the ordering and L11^{-1} replicated, K12 only at
        this rank's Schur points, the Schur FSAI's KNN and values only for this rank's rows.  X (n x d) and
        ``op`` (an NFFTAdditiveKernel of all n points after its setup: the dense additive kernel) are the same
        on every rank; perm_opt "identity" / "fps" / "perm" (``perm`` given); schur "fsai" / "noise"."""
        from . import _lib
        L = _lib.lib()
        X = np.asfortranarray(np.asarray(X, dtype=np.float64))
        n, d = X.shape
        opt = {"identity": 0, "fps": 1, "perm": 2}[perm_opt]
        p = None if perm is None else np.ascontiguousarray(np.asarray(perm, dtype=np.int32))
        if opt == 2 and (p is None or p.size != n):
            raise ValueError("perm_opt 'perm' needs a permutation of the n points")
        params = op.h if op is not None else _lib.kernel_params(f, l, mu, n)
        self = cls.__new__(cls)
        self.n, self.comm = row_end - row_begin, comm
        self.h = L.Nfft4GPAmdAfnShardSetup(X.ctypes.data, n, n, d, int(k), opt, None if p is None else p.ctypes.data,
                                           {"fsai": 3, "noise": 0}[schur], int(schur_lfil), int(kernel), params,
                                           int(row_begin), int(row_end), comm.h)
        if op is None:
            L.Nfft4GPKernelParamFree(params)
        if not self.h:
            raise RuntimeError("Nfft4GPAmdAfnShardSetup failed (see stderr)")
        return self

    def info(self) -> dict:
        """Landmarks m1 and Schur points m2 of this rank, the K12 doubles it holds (k m2) and its G entries."""
        import ctypes as C
        from . import _lib
        m1, m2 = C.c_int(), C.c_int()
        k12, nnz = C.c_longlong(), C.c_longlong()
        _lib.lib().Nfft4GPAmdAfnShardInfo(self.h, C.byref(m1), C.byref(m2), C.byref(k12), C.byref(nnz))
        return {"m1": m1.value, "m2": m2.value, "k12_doubles": k12.value, "g_nnz": nnz.value}

    def solve(self, x, rhs):
        from . import _lib
        from .nfft import _check_len, _ptr
        _check_len("x", x, self.n)
        _check_len("rhs", rhs, self.n)
        if _lib.lib().Nfft4GPAmdDistAfnSolve(self.h, self.n, _ptr(x)[0], _ptr(rhs)[0]) != 0:
            raise RuntimeError("Nfft4GPAmdDistAfnSolve failed")
        return x

    @property
    def solve_fnptr(self) -> int:
        from . import _lib
        return _lib.fnptr("Nfft4GPAmdDistAfnSolve")

    def free(self):
        from . import _lib
        if getattr(self, "h", None):
            _lib.lib().Nfft4GPAmdDistAfnFree(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class GpuVecOps:
    """BLAS-1 on device tensors through this library's HIP kernels (Nfft4GPVec*, vecops.c:3-155)."""

    def __init__(self):
        from . import _lib
        self.L = _lib.lib()

    def dot(self, a, b) -> float:
        return float(self.L.Nfft4GPVecDdot(a.data_ptr(), a.numel(), b.data_ptr()))

    def axpy(self, alpha, x, y):
        self.L.Nfft4GPVecAxpy(float(alpha), x.data_ptr(), x.numel(), y.data_ptr())

    def scale(self, x, s):
        self.L.Nfft4GPVecScale(x.data_ptr(), x.numel(), float(s))

    def copy(self, dst, src):
        dst.copy_(src)


class NumpyVecOps:
    """The same four operations on numpy arrays (CPU tests of the distributed control flow)."""

    def dot(self, a, b) -> float:
        return float(np.dot(a, b))

    def axpy(self, alpha, x, y):
        if alpha == 0.0:
            return
        y += alpha * x

    def scale(self, x, s):
        if s == 0.0:
            x[:] = 0.0
        else:
            x *= s

    def copy(self, dst, src):
        dst[:] = src


class RowShardedAdditiveKernel:
    """y_local = beta*y_local + alpha*f^2*((1/nw) sum_c K_c + mu I) x, rows sharded over a process group."""

    def __init__(self, engine, nwindows: int, n_global: int, row_begin: int, row_end: int, group=None,
                 grid=None):
        import torch
        import torch.distributed as dist
        self.engine = engine
        self.dist = dist
        self.group = group
        self.nw = nwindows
        self.n_global = n_global
        self.row_begin, self.row_end = row_begin, row_end
        self.n = row_end - row_begin
        if grid is None:
            # the HIP shard handle writes the grid from a kernel: keep it in HBM (RCCL reduces it in
            # place); a host engine (the numpy replay in the tests) keeps it in host memory
            dev = "cuda" if hasattr(engine, "h") else "cpu"
            size = engine.shard_grid_size() if hasattr(engine, "shard_grid_size") else nwindows * 64
            if size <= 0:
                raise RuntimeError("run the kernel setup on the shard handle before sharding its matvec")
            grid = torch.zeros(size, dtype=torch.float64, device=dev)
        self.grid = grid
        if hasattr(engine, "h"):
            # the HIP kernels and the collectives must be ordered on torch's current stream
            from . import _lib
            _lib.lib().Nfft4GPAmdSetStream(torch.cuda.current_stream().cuda_stream)
        self._grid_np = grid.numpy() if grid.device.type == "cpu" else None

    def _reduce_grid(self):
        self.dist.all_reduce(self.grid, group=self.group)

    def matsymv(self, x_local, alpha=1.0, beta=0.0, y_local=None, grad=False):
        g = self._grid_np if self._grid_np is not None else self.grid
        self.engine.shard_spread(x_local, g)
        self._reduce_grid()
        return self.engine.shard_finish(g, x_local, alpha, beta, y_local, grad)

    # ---- CG (pcg.c:3-206) with row-sharded vectors ----------------------------------------------
    def _gdot(self, vec, a, b) -> float:
        import torch
        dev = self.grid.device
        t = torch.tensor([vec.dot(a, b)], dtype=torch.float64, device=dev)
        self.dist.all_reduce(t, group=self.group)
        return float(t.item())

    def pcg(self, b, x, maxits=1000, tol=1e-6, atol=False, vec=None, precond=None):
        """Distributed mirror of Nfft4GPSolverPcg: same early exits, breakdown tests, true-residual
        recheck and reporting (rel_res_v, iter = 0 when not converged).  ``precond(z, r)`` acts on
        local rows.  Returns (x, rel_res, rel_res_v, iters)."""
        vec = vec or NumpyVecOps()
        EPS = np.finfo(np.float64).eps
        normb = math.sqrt(self._gdot(vec, b, b))
        if normb < EPS:  # pcg.c:32-41
            vec.scale(x, 0.0)
            return x, 0.0, np.zeros(1), 0
        tolb = tol if atol else tol * normb
        maxits = min(maxits, self.n_global)
        r = b.copy() if isinstance(b, np.ndarray) else b.clone()
        self.matsymv(x, -1.0, 1.0, r)
        normr = math.sqrt(self._gdot(vec, r, r))
        if normr < tolb:  # pcg.c:70-84
            return x, normr / normb, np.array([normr / normb]), 0
        normr2 = normr
        hist = np.zeros(maxits + 1)
        hist[0] = normr / normb
        z = r.copy() if isinstance(r, np.ndarray) else r.clone()
        p = z.copy() if isinstance(z, np.ndarray) else z.clone()
        q = z.copy() if isinstance(z, np.ndarray) else z.clone()
        rho = 1.0
        it = 0
        for ii in range(1, maxits + 1):
            if precond is not None:
                precond(z, r)
            else:
                vec.copy(z, r)
            rho1 = rho
            rho = self._gdot(vec, z, r)
            if rho == 0.0:
                break
            if ii == 1:
                vec.copy(p, z)
            else:
                beta = rho / rho1
                if beta == 0.0:
                    break
                vec.scale(p, beta)
                vec.axpy(1.0, z, p)
            self.matsymv(p, 1.0, 0.0, q)
            pq = self._gdot(vec, q, p)
            if pq <= 0:
                break
            alpha = rho / pq
            vec.axpy(alpha, p, x)
            vec.axpy(-alpha, q, r)
            normr = math.sqrt(self._gdot(vec, r, r))
            normr2 = normr
            hist[ii] = normr / normb
            if normr <= tolb:  # pcg.c:181-193
                vec.copy(r, b)
                self.matsymv(x, -1.0, 1.0, r)
                normr2 = math.sqrt(self._gdot(vec, r, r))
                hist[ii] = normr2
                if normr2 <= tolb:
                    it = ii
                    break
        return x, normr2 / normb, hist, it
