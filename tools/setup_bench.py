"""Preconditioner setup timings on the GPU beside the reference's own CPU setups (oracle/_ref, OpenMP).

    python tools/setup_bench.py [--out gpurun_out/setup_bench.json]

* FSAI setup with gradients (fsai.c:302-673: KNN pattern + per-row solves), Gaussian kernel.
* Farthest point sampling (ordering.c:422-711, Par1), k points.
* AFN setup (afn.c:161-489 with rank k, FPS order, Schur-complement kernel FSAI).
The reference timings run on the same host (the GPU box's cores), on the same inputs where it finishes
in seconds, else on a smaller n (stated in the output).  Uniform random points, f = 1, mu = 0.01.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd  # noqa: E402
from preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd import _lib  # noqa: E402


def timed(fn, reps=1):
    best = None
    out = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        t = time.perf_counter() - t0
        best = t if best is None else min(best, t)
    return best, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/setup_bench.json")
    ap.add_argument("--no-ref", action="store_true")
    a = ap.parse_args()
    import torch
    assert torch.cuda.is_available()
    L = _lib.lib()
    import oracle as O
    use_ref = (not a.no_ref) and O.ref_available()
    res = {"host_threads": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count()))}
    rng = np.random.default_rng(5)

    # FSAI with gradients
    for n, d, lfil, l in [(100000, 3, 30, 0.2), (1000000, 3, 30, 0.05)]:
        X = np.asfortranarray(rng.random((n, d)))
        P = _lib.kernel_params(1.0, l, 0.01, n)
        h = L.Nfft4GPAmdPrecondFsaiCreate()
        L.Nfft4GPAmdPrecondFsaiSetLfil(h, lfil)
        t, _ = timed(lambda: L.Nfft4GPAmdPrecondFsaiSetupWithKernel(X.ctypes.data, n, n, d, None, P, 1, h), reps=2)
        L.Nfft4GPAmdPrecondFsaiFree(h)
        L.Nfft4GPKernelParamFree(P)
        res[f"fsai_grad_setup_gpu_s_n{n}_d{d}_lfil{lfil}"] = round(t, 4)
        print(f"FSAI+grad setup n={n} d={d} lfil={lfil}: GPU {t:.3f} s", flush=True)
    if use_ref:
        n, d, lfil = 20000, 3, 30
        X = np.asfortranarray(rng.random((n, d)))
        P = O.ref_gaussian_params(1.0, 0.2, 0.01, n)
        t_ref, _ = timed(lambda: O.RefFsai(X, P, lfil, grad=True))
        Pg = _lib.kernel_params(1.0, 0.2, 0.01, n)
        h = L.Nfft4GPAmdPrecondFsaiCreate()
        L.Nfft4GPAmdPrecondFsaiSetLfil(h, lfil)
        t, _ = timed(lambda: L.Nfft4GPAmdPrecondFsaiSetupWithKernel(X.ctypes.data, n, n, d, None, Pg, 1, h), reps=2)
        L.Nfft4GPAmdPrecondFsaiFree(h)
        res[f"fsai_grad_setup_ref_cpu_s_n{n}"] = round(t_ref, 4)
        res[f"fsai_grad_setup_gpu_s_n{n}"] = round(t, 4)
        print(f"FSAI+grad setup n={n}: reference CPU {t_ref:.3f} s, GPU {t:.4f} s", flush=True)

    # FPS
    for n, d, k in [(1000000, 32, 512), (1000000, 3, 2048)]:
        X = rng.random((n, d))
        Xd = torch.tensor(X.T.copy(), device="cuda")
        t, (p, _) = timed(lambda: amd.sort_fps(Xd, k), reps=2)
        res[f"fps_gpu_s_n{n}_d{d}_k{k}"] = round(t, 4)
        res[f"fps_gpu_bytes_per_s_n{n}_d{d}_k{k}"] = round((k - 1) * n * (8 * d + 12) / t / 1e9, 1)
        print(f"FPS n={n} d={d} k={k}: GPU {t:.3f} s ({res[f'fps_gpu_bytes_per_s_n{n}_d{d}_k{k}']} GB/s)", flush=True)
        del Xd
    if use_ref:
        n, d, k = 100000, 32, 512
        X = rng.random((n, d))
        t_ref, (pr, _) = timed(lambda: O.ref_sort_fps(X, k))
        t, (p, _) = timed(lambda: amd.sort_fps(X, k), reps=2)
        res[f"fps_ref_cpu_s_n{n}_d{d}_k{k}"] = round(t_ref, 4)
        res[f"fps_gpu_host_data_s_n{n}_d{d}_k{k}"] = round(t, 4)
        res["fps_same_order_as_reference"] = bool(np.array_equal(p, pr))
        print(f"FPS n={n} d={d} k={k}: reference CPU {t_ref:.3f} s, GPU {t:.4f} s, same order "
              f"{res['fps_same_order_as_reference']}", flush=True)

    # AFN setup
    for n, d, k, lfil, l in [(100000, 3, 512, 20, 0.1), (1000000, 3, 512, 20, 0.05)]:
        X = np.asfortranarray(rng.random((n, d)))
        t, pre = timed(lambda: amd.AfnPrecond.setup(X, k, 1.0, l, 0.01, perm_opt="fps", schur_lfil=lfil))
        res[f"afn_setup_gpu_s_n{n}_d{d}_k{k}_lfil{lfil}"] = round(t, 4)
        xd = torch.zeros(n, dtype=torch.float64, device="cuda")
        rd = torch.rand(n, dtype=torch.float64, device="cuda")
        pre.solve(xd, rd)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            pre.solve(xd, rd)
        torch.cuda.synchronize()
        ta = (time.perf_counter() - t0) / 20
        res[f"afn_apply_gpu_ms_n{n}_k{k}"] = round(ta * 1e3, 3)
        print(f"AFN setup n={n} d={d} k={k} lfil={lfil}: GPU {t:.3f} s; apply {ta * 1e3:.3f} ms", flush=True)
        pre.free()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
