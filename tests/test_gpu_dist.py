"""Multi-GPU path on one GPU: two gloo ranks driving the library's distributed
operators (dist.hip, Nfft4GPAmdDist*) -- row-sharded and component-sharded additive matvecs, the gradient
matvec, the row-sharded Nystrom apply, and the device-controlled Nfft4GPSolverPcg on both -- against the
oracle and the one-GPU operator; plus the RCCL communicator itself (one rank: RCCL refuses two ranks on
one device) through the same operators.

Reference behaviour being split: nfft_interface.c:796-817 (components summed one after another, weight
1/nw, mu term once), pcg.c:3-206 (whole-vector CG), nys.c:115-173 (Nystrom apply).
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def problem(kind, seed=77):
    """(X, windows, nw, dw, x): 1-D windows (configs B-D shape) or TEST1-style multi-feature windows."""
    rng = np.random.default_rng(seed)
    if kind == "1d":
        n, d = 20000, 8
        X = rng.random((n, d))
        return X, np.arange(d, dtype=np.int32), d, 1, rng.random(n) - 0.5
    n = 6000
    X = rng.random((n, 5))
    win = np.array([0, 1, 2, 3, 4, -1], dtype=np.int32)  # 3-D window and a padded 2-D last window
    return X, win, 2, 3, rng.random(n) - 0.5


def _worker(rank, world, port, outdir, backend):
    for p in (ROOT, HERE, os.path.join(ROOT, "oracle")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    from preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd.dist import (
        Communicator, DistributedAdditiveKernel, RowShardedAfn, RowShardedNystrom)
    torch.cuda.set_device(0)
    # "nccl_callback": torch's own RCCL process group behind the callback communicator (bench.py's fallback)
    dist.init_process_group("nccl" if backend == "nccl_callback" else "gloo", rank=rank, world_size=world)
    comm = Communicator.rccl() if backend == "rccl" else Communicator.callback()
    out = {}
    for kind in ("1d", "md"):
        X, win, nw, dw, x = problem(kind)
        n = X.shape[0]
        for part in ("rows", "components"):
            op = DistributedAdditiveKernel(X, win, nw, dw, comm, partition=part)
            assert op.setup(amd.GAUSSIAN, f=1.3, l=0.1, mu=0.1) == 0
            rb, re = op.row_begin, op.row_end
            xd = torch.tensor(x[rb:re], device="cuda")
            y = op.matsymv(xd)
            y0 = torch.full_like(y, 0.25)
            yb = op.matsymv(xd, 0.7, -1.5, y0.clone())
            g = op.gradmatsymv(xd)
            if part == "components":
                # y all-reduced in one piece instead of 4 overlapped pieces: the same sums, bit for bit
                L = amd.lib()
                assert L.Nfft4GPAmdDistSetChunks(op.h, 1) == 0
                out[f"{kind}_{part}_y1"] = op.matsymv(xd).cpu().numpy()
                out[f"{kind}_{part}_yb1"] = op.matsymv(xd, 0.7, -1.5, y0.clone()).cpu().numpy()
                assert L.Nfft4GPAmdDistSetChunks(op.h, 7) == 0
                out[f"{kind}_{part}_y7"] = op.matsymv(xd).cpu().numpy()
                assert L.Nfft4GPAmdDistSetChunks(op.h, 4) == 0
            b = torch.tensor(x[rb:re], device="cuda")
            xs = torch.zeros_like(b)
            _, rr, hist, it = amd.pcg(op, b, xs, maxits=2000, tol=1e-6)
            key = f"{kind}_{part}"
            out.update({key + "_y": y.cpu().numpy(), key + "_yb": yb.cpu().numpy(), key + "_g": g.cpu().numpy(),
                        key + "_x": xs.cpu().numpy(), key + "_rr": rr, key + "_it": it, key + "_rb": rb,
                        key + "_re": re})
            if kind == "1d" and part == "rows":
                # row-sharded Nystrom: the full setup on every rank (deterministic), then this rank's rows
                full = amd.NFFTAdditiveKernel(X, win, nw, dw)
                assert full.setup(amd.GAUSSIAN, f=1.3, l=0.1, mu=0.1) == 0
                perm = np.random.default_rng(5).permutation(n).astype(np.int32)
                nys = amd.NystromPrecond.from_additive(full, perm, 64, k11="landmarks")
                dn = RowShardedNystrom(nys, rb, re, comm)
                r = torch.tensor(np.random.default_rng(6).random(n)[rb:re], device="cuda")
                z = torch.zeros_like(r)
                dn.solve(z, r)
                # the setup itself split over the rows (one k x k all-reduce of the Gram)
                ds = RowShardedNystrom.setup(op, perm, 64, k11="landmarks")
                zs = torch.zeros_like(r)
                ds.solve(zs, r)
                xs3 = torch.zeros_like(b)
                _, _, _, it3 = amd.pcg(op, b, xs3, maxits=2000, tol=1e-6, precond=ds)
                out.update({"nys_shard_z": zs.cpu().numpy(), "nys_shard_x": xs3.cpu().numpy(), "nys_shard_it": it3})
                ds.free()
                # the AFN apply split over the rows (both Schur solves), from a full setup on every rank
                for schur in ("fsai", "noise"):
                    afn = amd.AfnPrecond.setup(X, 64, 0, 0, 0, perm_opt="perm", perm=perm, schur_lfil=10, op=full,
                                               schur=schur)
                    da = RowShardedAfn(afn, rb, re, comm)
                    za = torch.zeros_like(r)
                    da.solve(za, r)
                    xs4 = torch.zeros_like(b)
                    _, _, _, it4 = amd.pcg(op, b, xs4, maxits=2000, tol=1e-6, precond=da)
                    out.update({f"afn_{schur}_z": za.cpu().numpy(), f"afn_{schur}_x": xs4.cpu().numpy(),
                                f"afn_{schur}_it": it4})
                    da.free()
                    afn.free()
                    # the same shard set up on this rank alone (no full AFN anywhere): K12 at its Schur points
                    # only, the Schur FSAI's KNN and values for its rows only
                    ds_a = RowShardedAfn.setup(X, 64, comm, rb, re, perm_opt="perm", perm=perm, schur=schur,
                                               schur_lfil=10, op=full)
                    zs_a = torch.zeros_like(r)
                    ds_a.solve(zs_a, r)
                    xs5 = torch.zeros_like(b)
                    _, _, _, it5 = amd.pcg(op, b, xs5, maxits=2000, tol=1e-6, precond=ds_a)
                    inf = ds_a.info()
                    out.update({f"afn_{schur}_sz": zs_a.cpu().numpy(), f"afn_{schur}_sx": xs5.cpu().numpy(),
                                f"afn_{schur}_sit": it5, f"afn_{schur}_m2": inf["m2"],
                                f"afn_{schur}_k12": inf["k12_doubles"], f"afn_{schur}_gnnz": inf["g_nnz"]})
                    ds_a.free()
                # a failure on ONE rank's rows (a local Schur FSAI breakdown left the other rank in
                # PCG's collectives): every rank must return NULL and none may wait forever
                if rank == 1:
                    os.environ["NFFT4GP_AMD_FAULT_AFN_SHARD"] = "1"
                try:
                    RowShardedAfn.setup(X, 64, comm, rb, re, perm_opt="perm", perm=perm, schur="fsai", schur_lfil=10,
                                        op=full)
                    out["afn_fault_raised"] = 0
                except RuntimeError:
                    out["afn_fault_raised"] = 1
                os.environ.pop("NFFT4GP_AMD_FAULT_AFN_SHARD", None)
                xs2 = torch.zeros_like(b)
                _, rr2, _, it2 = amd.pcg(op, b, xs2, maxits=2000, tol=1e-6, precond=dn)
                out.update({"nys_z": z.cpu().numpy(), "nys_x": xs2.cpu().numpy(), "nys_rr": rr2, "nys_it": it2})
                dn.free()
                nys.free()
                full.free()
            op.free()
    torch.cuda.synchronize()
    comm.free()
    np.savez(os.path.join(outdir, f"{backend}_rank{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


def _run(tmp_path_factory, backend, world):
    import torch.multiprocessing as mp
    out = tmp_path_factory.mktemp(backend)
    mp.spawn(_worker, args=(world, _free_port(), str(out), backend), nprocs=world, join=True)
    return [dict(np.load(os.path.join(out, f"{backend}_rank{r}.npz"))) for r in range(world)]


@pytest.fixture(scope="module")
def gloo2(tmp_path_factory):
    return _run(tmp_path_factory, "callback", 2)


@pytest.fixture(scope="module")
def rccl1(tmp_path_factory):
    return _run(tmp_path_factory, "rccl", 1)


@pytest.fixture(scope="module")
def nccl_cb1(tmp_path_factory):
    return _run(tmp_path_factory, "nccl_callback", 1)


@pytest.fixture(scope="module")
def single(torch_cuda):
    """The one-GPU operator and PCG on the same problems (the reference's whole-vector semantics)."""
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    torch = torch_cuda
    res = {}
    for kind in ("1d", "md"):
        X, win, nw, dw, x = problem(kind)
        op = amd.NFFTAdditiveKernel(X, win, nw, dw)
        assert op.setup(amd.GAUSSIAN, f=1.3, l=0.1, mu=0.1) == 0
        xd = torch.tensor(x, device="cuda")
        res[kind + "_y"] = op.matsymv(xd).cpu().numpy()
        res[kind + "_yb"] = op.matsymv(xd, 0.7, -1.5, torch.full_like(xd, 0.25)).cpu().numpy()
        res[kind + "_g"] = op.gradmatsymv(xd).cpu().numpy()
        xs = torch.zeros_like(xd)
        _, rr, _, it = amd.pcg(op, xd.clone(), xs, maxits=2000, tol=1e-6)
        res[kind + "_x"], res[kind + "_it"] = xs.cpu().numpy(), it
        if kind == "1d":
            perm = np.random.default_rng(5).permutation(X.shape[0]).astype(np.int32)
            nys = amd.NystromPrecond.from_additive(op, perm, 64, k11="landmarks")
            r = torch.tensor(np.random.default_rng(6).random(X.shape[0]), device="cuda")
            res["nys_z"] = nys.solve(torch.zeros_like(r), r).cpu().numpy()
            xs2 = torch.zeros_like(xd)
            _, _, _, res["nys_it"] = amd.pcg(op, xd.clone(), xs2, maxits=2000, tol=1e-6, precond=nys)
            res["nys_x"] = xs2.cpu().numpy()
            nys.free()
            for schur in ("fsai", "noise"):
                afn = amd.AfnPrecond.setup(X, 64, 0, 0, 0, perm_opt="perm", perm=perm, schur_lfil=10, op=op,
                                           schur=schur)
                res[f"afn_{schur}_z"] = afn.solve(torch.zeros_like(r), r).cpu().numpy()
                xs4 = torch.zeros_like(xd)
                _, _, _, res[f"afn_{schur}_it"] = amd.pcg(op, xd.clone(), xs4, maxits=2000, tol=1e-6, precond=afn)
                res[f"afn_{schur}_x"] = xs4.cpu().numpy()
                afn.free()
        op.free()
    return res


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(b), 1e-300))


def gather(ranks, key, part, mult=1):
    """Whole vector from the ranks' pieces: rows concatenate (per output block of the gradient), replicated
    components must agree between ranks."""
    if part == "components":
        for r in ranks[1:]:
            np.testing.assert_array_equal(r[key], ranks[0][key])
        return ranks[0][key]
    blocks = []
    for m in range(mult):
        for r in ranks:
            nl = int(r[key.rsplit("_", 1)[0] + "_re"]) - int(r[key.rsplit("_", 1)[0] + "_rb"])
            blocks.append(r[key][m * nl:(m + 1) * nl])
    return np.concatenate(blocks)


@pytest.mark.parametrize("kind", ["1d", "md"])
@pytest.mark.parametrize("part", ["rows", "components"])
def test_distributed_matvec_matches_single_gpu_and_oracle(gloo2, single, kind, part):
    from oracle import OracleAdditiveNFFT
    key = f"{kind}_{part}"
    y = gather(gloo2, key + "_y", part)
    yb = gather(gloo2, key + "_yb", part)
    g = gather(gloo2, key + "_g", part, 3)
    # the split sums the same terms in another order: rounding-level differences
    assert rel(y, single[kind + "_y"]) < 1e-12
    assert rel(yb, single[kind + "_yb"]) < 1e-12
    assert rel(g, single[kind + "_g"]) < 1e-12
    X, win, nw, dw, x = problem(kind)
    o = OracleAdditiveNFFT(X, win, nw, dw)
    o.setup(0, 1.3, 0.1, 0.1)
    tol = 1e-8 if kind == "1d" else 1e-10
    assert rel(y, o.matsymv(x)) < tol
    assert rel(g, o.gradmatsymv(x)) < tol


@pytest.mark.parametrize("kind", ["1d", "md"])
@pytest.mark.parametrize("part", ["rows", "components"])
def test_distributed_pcg_matches_single_gpu(gloo2, single, kind, part):
    key = f"{kind}_{part}"
    its = [int(r[key + "_it"]) for r in gloo2]
    assert len(set(its)) == 1, its  # every rank took the same device-side decisions
    it, it1 = its[0], int(single[kind + "_it"])
    assert it > 0 and float(gloo2[0][key + "_rr"]) <= 1e-6
    # LDS-atomic accumulation order moves CG's count by a few iterations run to run
    assert abs(it - it1) <= max(3, it1 // 20), (it, it1)
    assert rel(gather(gloo2, key + "_x", part), single[kind + "_x"]) < 1e-4


@pytest.mark.parametrize("kind", ["1d", "md"])
def test_component_split_chunked_allreduce_is_bitwise(gloo2, kind):
    """the component split all-reduces y in pieces on its own stream, each overlapping the
    next piece's interpolation.  The pieces are disjoint slices summed element for element, so 1, 4 (default)
    and 7 pieces compute the same sums; the interpolation's ds_add_f64 order follows the wave schedule, so
    two matvecs of the same x differ at rounding level anyway: compared to 1e-14, and every
    rank holds the same bits (multi-feature windows keep the single all-reduce)."""
    for r in gloo2:
        assert rel(r[f"{kind}_components_y1"], r[f"{kind}_components_y"]) < 1e-14
        assert rel(r[f"{kind}_components_y7"], r[f"{kind}_components_y"]) < 1e-14
        assert rel(r[f"{kind}_components_yb1"], r[f"{kind}_components_yb"]) < 1e-14
    for key in ("y", "y1", "y7", "yb", "yb1"):
        np.testing.assert_array_equal(gloo2[0][f"{kind}_components_{key}"], gloo2[1][f"{kind}_components_{key}"])


def test_row_sharded_nystrom_setup(gloo2, single):
    """Nfft4GPAmdNysShardSetupAdditive: panel, U1 and U per row shard, the Gram summed
    with one k x k all-reduce; the apply equals the one-GPU setup's (the Gram's sum is regrouped, so its
    eigenbasis moves at rounding level) and PCG with it takes the one-GPU iteration count."""
    z = np.concatenate([r["nys_shard_z"] for r in gloo2])
    assert rel(z, single["nys_z"]) < 1e-9
    its = [int(r["nys_shard_it"]) for r in gloo2]
    assert len(set(its)) == 1 and its[0] > 0
    assert abs(its[0] - int(single["nys_it"])) <= max(3, int(single["nys_it"]) // 20), (its, single["nys_it"])
    assert rel(np.concatenate([r["nys_shard_x"] for r in gloo2]), single["nys_x"]) < 1e-4


@pytest.mark.parametrize("schur", ["fsai", "noise"])
def test_row_sharded_afn_apply_and_pcg(gloo2, single, schur):
    """Nfft4GPAmdAfnShard: each rank keeps its landmarks, the K12 columns of its Schur
    points and their FSAI rows; the apply equals the one-GPU apply (the K12 y2 sum is regrouped over the
    ranks) and PCG with it matches the one-GPU iteration count."""
    z = np.concatenate([r[f"afn_{schur}_z"] for r in gloo2])
    assert rel(z, single[f"afn_{schur}_z"]) < 1e-12
    its = [int(r[f"afn_{schur}_it"]) for r in gloo2]
    it1 = int(single[f"afn_{schur}_it"])
    assert len(set(its)) == 1 and its[0] > 0
    assert abs(its[0] - it1) <= max(3, it1 // 20), (its, it1)
    assert rel(np.concatenate([r[f"afn_{schur}_x"] for r in gloo2]), single[f"afn_{schur}_x"]) < 1e-4


@pytest.mark.parametrize("schur", ["fsai", "noise"])
def test_row_sharded_afn_setup(gloo2, single, schur):
    """Nfft4GPAmdAfnShardSetup: each rank sets up its own shard -- the K12 columns of its
    Schur points only (k x m2 with m2 ~ (n - k) / N), the Schur FSAI's KNN and values for its rows only -- and
    the apply equals the one-GPU AFN apply (afn.c:82-143 on the full setup) to 1e-12; PCG with it takes the
    one-GPU iteration count."""
    X, _, _, _, _ = problem("1d")
    n, k = X.shape[0], 64
    z = np.concatenate([r[f"afn_{schur}_sz"] for r in gloo2])
    assert rel(z, single[f"afn_{schur}_z"]) < 1e-12
    m2 = [int(r[f"afn_{schur}_m2"]) for r in gloo2]
    assert sum(m2) == n - k  # every Schur point is held by exactly one rank
    for r, m in zip(gloo2, m2):
        assert int(r[f"afn_{schur}_k12"]) == k * m  # K12 memory per rank: k (n - k) / N, not k (n - k)
        assert m <= (n - k) // 2 + 200
    if schur == "fsai":
        # the G rows of the ranks together: the full pattern's n - k rows of up to lfil = 10 entries
        assert sum(int(r["afn_fsai_gnnz"]) for r in gloo2) <= 10 * (n - k)
    its = [int(r[f"afn_{schur}_sit"]) for r in gloo2]
    it1 = int(single[f"afn_{schur}_it"])
    assert len(set(its)) == 1 and its[0] > 0
    assert abs(its[0] - it1) <= max(3, it1 // 20), (its, it1)
    assert rel(np.concatenate([r[f"afn_{schur}_sx"] for r in gloo2]), single[f"afn_{schur}_x"]) < 1e-4


def test_row_sharded_afn_setup_failure_on_one_rank(gloo2):
    """A breakdown on one rank's rows only (fault-injected on rank 1): the sharded setup agrees the failure over
    the communicator, so BOTH ranks return NULL (and the worker went on to its next collectives)."""
    assert [int(r["afn_fault_raised"]) for r in gloo2] == [1, 1]


def test_row_sharded_nystrom_apply_and_pcg(gloo2, single):
    z = np.concatenate([r["nys_z"] for r in gloo2])
    assert rel(z, single["nys_z"]) < 1e-12
    its = [int(r["nys_it"]) for r in gloo2]
    assert len(set(its)) == 1 and its[0] > 0
    it1 = int(single["nys_it"])
    # the same run-to-run LDS-atomic order effect as in test_distributed_pcg_matches_single_gpu (58 vs 55 seen)
    assert abs(its[0] - it1) <= max(3, it1 // 20), (its, it1)
    assert rel(np.concatenate([r["nys_x"] for r in gloo2]), single["nys_x"]) < 1e-4


@pytest.mark.parametrize("kind", ["1d", "md"])
def test_rccl_communicator_one_rank(rccl1, single, kind):
    """RCCL itself (ncclCommInitRank + ncclAllReduce on the library stream) behind the same operators."""
    for part in ("rows", "components"):
        key = f"{kind}_{part}"
        assert rel(rccl1[0][key + "_y"], single[kind + "_y"]) < 1e-12
        assert rel(rccl1[0][key + "_g"], single[kind + "_g"]) < 1e-12
        assert int(rccl1[0][key + "_it"]) > 0


@pytest.mark.parametrize("kind", ["1d", "md"])
def test_callback_communicator_over_torch_nccl(nccl_cb1, single, kind):
    """The callback communicator on a torch "nccl" (RCCL) group: device buffers all-reduced in place."""
    for part in ("rows", "components"):
        key = f"{kind}_{part}"
        assert rel(nccl_cb1[0][key + "_y"], single[kind + "_y"]) < 1e-12
        assert rel(nccl_cb1[0][key + "_g"], single[kind + "_g"]) < 1e-12
        assert int(nccl_cb1[0][key + "_it"]) > 0
