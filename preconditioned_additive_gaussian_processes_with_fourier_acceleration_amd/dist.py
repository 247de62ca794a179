"""Row-sharded multi-GPU operator and CG over torch.distributed (one process per GPU, RCCL).

The reference is single-process (SRC/external/nfft_interface.c, SRC/solvers/pcg.c).  Across GPUs the
additive matvec shards by ROWS: every rank spreads its own n/N points for all
windows into the nw x 64 oversampled grids, the grids (16 KB at nw = 32) are summed with ONE
all-reduce, and every rank interpolates its own rows.  CG keeps x, r, p, q row-sharded, so each dot
product becomes a local dot plus a scalar all-reduce.

``engine`` is anything with ``shard_spread(x_local, grid)`` / ``shard_finish(grid, x_local, alpha,
beta, y_local, grad)`` -- the HIP shard handle (NFFTAdditiveKernel(..., shard=...)) in production; the
CPU tests plug in the numpy replay of the same kernels to exercise the gloo path.
"""
from __future__ import annotations

import math

import numpy as np


def row_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous row block of `rank` (ceil-divided, the last ranks may get fewer or zero rows)."""
    per = (n + world - 1) // world
    return min(n, rank * per), min(n, (rank + 1) * per)


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
