#!/usr/bin/env python3
"""Headline benchmark: additive NFFT kernel matvecs/s (+ PCG wall time to 1e-6) on MI355X.

Workload (BASELINE.json configs[2], "headline single-GPU"): n = 1e6 points, d = 32 features, 32 1-D
additive windows {0},{1},...,{31}, Gaussian kernel f = 1, l = 1, mu = 0.01; points i.i.d. U[0,1)^d,
vector x ~ U(-0.5, 0.5) (TESTS/TEST1/foo.cpp:243-247), numpy PCG64 seed 906 (synthetic data).
One "step" = one Nfft4GPAdditiveNFFTMatSymv(y = K x) with x and y resident in HBM.

N = 1:  the matvec on one GPU.
N > 1:  one process per GPU: under torch.distributed.run (WORLD_SIZE set, which must equal --gpus) or, when
        no launcher set WORLD_SIZE, spawned by this script itself before anything touches the GPU (each child
        gets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT; the parent exits non-zero if
        any rank fails, or with RCCL if fewer than N devices are visible).  The library's own RCCL communicator
        does the all-reduces over xGMI, enqueued on the stream by dist.hip; the line reports the ranks RCCL
        itself counts (ncclCommCount) and each rank's kernel and all-reduce time.  The headline splits ROWS:
        each rank spreads its own n/N points for all 32 windows, the 32x64 oversampled grids (16 KB) are
        all-reduced, each rank interpolates its own rows.  The line also carries the split BASELINE
        configs[3] names, 4 COMPONENTS per GPU (y, 8 MB, all-reduced), timed the same way
        ("partition_components").  Total work is fixed -> "scaling": "strong".

Printed (rank 0): one JSON line with value = whole-job matvecs/s, the roofline of the dominant kernel
(measured live with hipEvents on the library stream), the CPU baseline (this repo's C/OpenMP
restatement of the reference NFFT path = oracle/, "kind": "port", on a bounded sample), and PCG
time to 1e-6 (unpreconditioned, N = 1).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_METRIC = "kernel matvecs/sec + PCG wall-time to 1e-6, n=1e6 d=32 additive, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)
F64_MFMA_PEAK_TFS = 78.6  # MI355X dense FP64 matrix peak (spec; gfx950 runs v_mfma_f64_16x16x4 at half of MI300X)


def make_problem(n, d, seed=906):
    rng = np.random.default_rng(seed)
    X = rng.random((n, d))
    x = rng.random(n) - 0.5
    return X, x


def algorithmic_bytes(info, n, nw, beta_zero=True):
    """Bytes each kernel must move with this layout:
    spread: 5 B per (point, window) [12-bit local index + 26-bit offset in the cell] + 8n (alpha)
            + nblocks*nw*64*8 (partial grids);
    interp: 5 B per (point, window) + 8n (x for the mu term) + 8n (y write) [+ 8n y read if beta != 0]."""
    pc = n * nw
    parts = info["nblocks"] * nw * 64 * 8
    spread = 5 * pc + 8 * n + parts
    interp = 5 * pc + 16 * n + (0 if beta_zero else 8 * n)
    return spread, interp


def host_info():
    """The CPU the baseline ran on: model name, logical CPUs this process may use, physical cores of the
    machine (sockets x cores per socket, /proc/cpuinfo), and the OpenMP binding variables in effect."""
    model, phys = None, set()
    try:
        cur = {}
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if ":" not in line:
                    if cur.get("physical id") is not None:
                        phys.add((cur.get("physical id"), cur.get("core id")))
                    cur = {}
                    continue
                k, v = (t.strip() for t in line.split(":", 1))
                cur[k] = v
                if k == "model name" and model is None:
                    model = v
    except OSError:
        pass
    return {"cpu_model": model, "physical_cores_machine": len(phys) or None,
            "cpus_allowed": len(os.sched_getaffinity(0)),
            "omp_env": {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OMP_PROC_BIND", "OMP_PLACES")}}


def _native_oracle():
    """A -march=native build of the oracle for this host (built into a scratch dir), or None."""
    try:
        out_dir = os.path.join(ROOT, "gpurun_out", "oracle_native")
        os.makedirs(out_dir, exist_ok=True)
        so = os.path.join(out_dir, "liboracle_native.so")
        subprocess.run(["gcc", "-O3", "-march=native", "-fPIC", "-fopenmp", "-std=gnu11", "-shared",
                        os.path.join(ROOT, "oracle", "nfft4gp_oracle.c"), "-o", so, "-lm"],
                       check=True, capture_output=True, timeout=120)
        return so
    except Exception:
        return None


def cpu_baseline_child(n, d, so, threads_list, max_seconds=12.0, min_samples=5, max_samples=15):
    """Child of cpu_baseline (its OpenMP binding fixed by the parent's environment before libgomp starts): one
    setup, then for each thread count the median of 5-15 timed full matvecs after one warm-up, bounded by
    max_seconds of timed work per count.  Prints one JSON line."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc_mod
    lib = orc_mod.oracle_lib(so) if so else orc_mod.oracle_lib()
    X, x = make_problem(n, d)
    o = orc_mod.OracleAdditiveNFFT(X, np.arange(d, dtype=np.int32), d, 1, lib=lib)
    t0 = time.time()
    o.setup(0, 1.0, 1.0, 0.01)
    out = {"setup_s": time.time() - t0, "runs": []}
    for th in threads_list:
        lib.orc_set_num_threads(th)
        o.matsymv(x)  # warm (and the team of this size started)
        times = []
        while len(times) < max_samples and (len(times) < min_samples or sum(times) < max_seconds):
            t0 = time.perf_counter()
            o.matsymv(x)
            times.append(time.perf_counter() - t0)
        out["runs"].append({"threads": int(lib.orc_num_threads()), "samples": len(times),
                            "median_s": float(np.median(times)), "min_s": float(min(times)),
                            "max_s": float(max(times))})
    print(json.dumps(out), flush=True)


def physical_cores_allowed():
    """Physical cores (distinct (physical id, core id) pairs of /proc/cpuinfo) among the CPUs this process's
    affinity mask grants."""
    allowed = os.sched_getaffinity(0)
    cores, cur = set(), {}
    try:
        with open("/proc/cpuinfo") as fh:
            for line in list(fh) + [""]:
                if ":" not in line:
                    if cur.get("processor") is not None and int(cur["processor"]) in allowed:
                        cores.add((cur.get("physical id"), cur.get("core id")))
                    cur = {}
                    continue
                k, v = (t.strip() for t in line.split(":", 1))
                cur[k] = v
    except OSError:
        return len(allowed)
    return len(cores) or len(allowed)


def cpu_quota():
    """CPUs the cgroup's CFS quota grants this process (cgroup v2 cpu.max, else v1 cpu.cfs_quota_us /
    cpu.cfs_period_us), or None when there is no quota."""
    paths = []
    try:
        with open("/proc/self/cgroup") as fh:
            for line in fh:
                parts = line.strip().split(":", 2)
                if len(parts) == 3 and (parts[1] == "" or "cpu" in parts[1].split(",")):
                    paths.append((parts[1], parts[2]))
    except OSError:
        pass
    for ctl, rel in paths:
        if ctl == "":  # v2
            for base in (os.path.join("/sys/fs/cgroup", rel.lstrip("/")), "/sys/fs/cgroup"):
                try:
                    quota, period = open(os.path.join(base, "cpu.max")).read().split()[:2]
                    if quota != "max":
                        return float(quota) / float(period)
                    break
                except (OSError, ValueError):
                    continue
        else:  # v1
            for base in (os.path.join("/sys/fs/cgroup/cpu", rel.lstrip("/")), "/sys/fs/cgroup/cpu"):
                try:
                    quota = int(open(os.path.join(base, "cpu.cfs_quota_us")).read())
                    period = int(open(os.path.join(base, "cpu.cfs_period_us")).read())
                    if quota > 0 and period > 0:
                        return quota / period
                    break
                except (OSError, ValueError):
                    continue
    return None


def cpu_baseline(n, d, threads=16, timeout=600):
    """Oracle (C + OpenMP restatement of nfft_interface.c + NFFT3 fastsum, oracle/nfft4gp_oracle.c, with
    NFFT3's PRE_PSI taps and a 1-D fast path) on this host's cores, in a child process whose OpenMP threads
    are bound one per physical core (OMP_PROC_BIND=close, OMP_PLACES=cores): at `threads` (16: the GPU box's
    CPU share, which its OMP_NUM_THREADS also names), at every physical core the affinity mask grants, and on
    one thread, each the median of 5-15 timed matvecs with min / max.  `value` is the faster of the two
    multi-thread runs (the strongest CPU figure this host gives), with both reported beside it."""
    so = _native_oracle()
    allcores = physical_cores_allowed()
    quota = cpu_quota()
    # never more threads than the CFS quota grants: above it the threads time-share the quota and the run is
    # slower than fewer threads (round 5's 128-thread leg on a 16-CPU share ran below one thread)
    cap = max(1, int(quota)) if quota else None
    share = min(threads, cap) if cap else threads
    usable = min(allcores, cap) if cap else allcores
    counts = [share] + ([usable] if usable != share else []) + [1]
    env = dict(os.environ, OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="close", OMP_PLACES="cores")
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", "--n", str(n), "--d", str(d),
           "--cpu-threads", ",".join(str(c) for c in counts)] + (["--cpu-oracle-so", so] if so else [])
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        raise RuntimeError(f"cpu baseline child failed ({r.returncode}): {r.stderr[-400:]}")
    res = json.loads(r.stdout.strip().splitlines()[-1])
    runs = res["runs"]
    single = runs[-1]
    multi = runs[:-1]
    best = min(multi, key=lambda x: x["median_s"])
    host = host_info()
    host["physical_cores_allowed"] = allcores
    host["cpu_quota_cpus"] = quota
    host["omp_env"] = {k: env.get(k) for k in ("OMP_NUM_THREADS", "OMP_PROC_BIND", "OMP_PLACES")}

    def rec(x):
        return {"value": 1.0 / x["median_s"], "cores": x["threads"], "samples": x["samples"],
                "median_s": x["median_s"], "min_s": x["min_s"], "max_s": x["max_s"]}

    return {
        "value": 1.0 / best["median_s"],
        "unit": "matvecs/s",
        "cores": best["threads"],
        "kind": "port",
        "samples": best["samples"],
        "median_s": best["median_s"],
        "min_s": best["min_s"],
        "max_s": best["max_s"],
        "box_share": rec(multi[0]),
        "all_usable_cores": rec(multi[1]) if len(multi) > 1 else rec(multi[0]),
        "one_thread": rec(single),
        "multi_thread_slower_than_one": any(m["median_s"] > single["median_s"] for m in multi),
        "host": host,
        "sample": f"median of 5-15 timed matvecs of the full workload (n={n}, {d} windows) after one warm-up per "
                  f"thread count, OpenMP threads bound one per physical core (close, cores) in a child process: "
                  f"{share} threads (the box's CPU share{', capped by the CFS quota of %.1f CPUs' % quota if quota else ''}), "
                  f"{usable} threads (the physical cores of the affinity mask, {allcores}, capped by the quota) and 1; "
                  f"value = the faster multi-thread median; setup (PRE_PSI taps, bhat) "
                  f"{res['setup_s']:.1f}s untimed; -march=native={so is not None}",
    }


def resolve_world(gpus, env=None):
    """How this process runs: ("single", 1), ("rank", WORLD_SIZE) under a launcher, or ("spawn", N) when --gpus N > 1
    and no launcher set WORLD_SIZE.  A launcher's WORLD_SIZE must equal --gpus when both are given."""
    env = os.environ if env is None else env
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        ws = int(ws)
        if gpus is not None and gpus != ws:
            raise SystemExit(f"bench: the launcher set WORLD_SIZE={ws} but --gpus {gpus}; they must agree")
        return ("rank" if ws > 1 else "single"), ws
    n = 1 if gpus is None else int(gpus)
    if n < 1:
        raise SystemExit(f"bench: --gpus {n}: need at least one GPU")
    return ("spawn" if n > 1 else "single"), n


def rank_envs(n, port, base=None):
    """The environment of each spawned rank (what torch.distributed.run would set on one node)."""
    base = dict(os.environ if base is None else base)
    return [dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)) for r in range(n)]


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def visible_devices():
    """GPUs this process may use; torch.cuda.device_count() does not initialise the GPU on this image."""
    import torch
    return torch.cuda.device_count()


def spawn_ranks(n, argv, backend=None, poll_s=0.2):
    """Start n ranks of this script (one process per GPU) and wait for them.  Nothing here touches the GPU: the
    children are new processes, not a fork of an initialised one.  Rank 0's stdout is this process's (it prints
    the line); the other ranks' stdout is discarded.  Returns the exit code: 0 only if every rank succeeded; when
    one fails the others are terminated (their own PIDs) so that none waits in a collective forever."""
    backend = backend or os.environ.get("NFFT4GP_BENCH_BACKEND", "nccl")
    if backend != "gloo" and "--launcher-selftest" not in argv:
        ndev = visible_devices()
        if ndev < n:
            print(f"bench: --gpus {n} with RCCL needs {n} visible GPUs, this box has {ndev}; not running "
                  f"(NFFT4GP_BENCH_BACKEND=gloo rehearses the ranks on fewer GPUs)", file=sys.stderr)
            return 2
    port = _free_port()
    procs = []
    for r, env in enumerate(rank_envs(n, port)):
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench: rank {procs.index(p)} exited with {code}; stopping the other ranks", file=sys.stderr)
                for q in live:
                    q.terminate()
        if live:
            time.sleep(poll_s)
    return rc


def launcher_selftest(fail_rank):
    """--launcher-selftest (CPU test of the plumbing): each rank writes what it received, one rank may fail."""
    rank = int(os.environ.get("RANK", "-1"))
    out = os.environ.get("NFFT4GP_BENCH_SELFTEST_DIR")
    rec = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                                          "MASTER_PORT")}
    rec["argv"] = sys.argv[1:]
    if out:
        with open(os.path.join(out, f"rank{rank}.json"), "w") as fh:
            json.dump(rec, fh)
    if rank == fail_rank:
        raise SystemExit(3)
    if rank == 0:
        print(json.dumps({"selftest": True, "world": int(rec["WORLD_SIZE"])}), flush=True)


def kernel_only(n, d, nys_rank=0, precision=64):
    """Child mode for the PMC passes: setup + one matvec + a few launches of each kernel (and, with
    nys_rank > 0, one rank-k Nystrom setup for its MFMA GEMM k_gemm_f64)."""
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    X, x_host = make_problem(n, d)
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    if precision != 64:
        op.set_precision(precision)
    assert op.setup(amd.GAUSSIAN, f=1.0, l=1.0, mu=0.01) == 0
    xd = torch.tensor(x_host, device="cuda")
    yd = torch.zeros(n, dtype=torch.float64, device="cuda")
    op.matsymv(xd, 1.0, 0.0, yd)
    for k in op.KERNELS:
        op.kernel_bench(k, xd, yd, reps=5)
    if nys_rank > 0:
        assert op.setup(amd.GAUSSIAN, f=1.0, l=0.1, mu=0.01) == 0
        perm = np.random.default_rng(908).permutation(n).astype(np.int32)
        amd.NystromPrecond.from_additive(op, perm, nys_rank, k11="landmarks").free()
    torch.cuda.synchronize()


def pmc_traffic(n, d, timeout=600, precision=64):
    """HBM bytes per launch of k_spread / k_interp from rocprofv3 PMC counters, one counter per pass
    (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass), on a child process running --kernel-only.
    FETCH_SIZE is doubled (gfx950 tallies 128-B reads at 64 B, MI355X_MICROARCH.md 'HBM');
    both counters are in KiB.  Returns {kernel: {"fetch": B, "write": B, "traffic": B}} or None."""
    import csv
    import shutil
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None
    out = {}
    base = os.path.join(ROOT, "gpurun_out", "bench_pmc")
    env = dict(os.environ, TMPDIR="/tmp")
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d_out = os.path.join(base, counter.lower())
        shutil.rmtree(d_out, ignore_errors=True)
        cmd = [exe, "--pmc", counter, "--output-format", "csv", "-d", d_out, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__), "--kernel-only", "--n", str(n), "--d", str(d),
               "--kernel-only-precision", str(precision)]
        r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=timeout)
        if r.returncode != 0:
            return None
        path = os.path.join(d_out, "pmc_counter_collection.csv")
        sums = {}
        with open(path) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                name = row["Kernel_Name"]
                key = "spread" if "k_spread" in name else "interp" if "k_interp" in name else \
                      "grid" if "k_grid" in name else None
                if key is None:
                    continue
                s = sums.setdefault(key, [0.0, 0])
                s[0] += float(row["Counter_Value"])
                s[1] += 1
        for key, (tot, cnt) in sums.items():
            kib = tot / cnt
            rec = out.setdefault(key, {})
            rec["fetch" if counter == "FETCH_SIZE" else "write"] = \
                kib * 1024 * (2 if counter == "FETCH_SIZE" else 1)
    for rec in out.values():
        rec["traffic"] = rec.get("fetch", 0.0) + rec.get("write", 0.0)
    return out


def run_pcg_single(op, torch, n, rng_seed=906, tol=1e-6, maxits=3000, l_pcg=0.1, rows=None, dist=None,
                   prefix="pcg"):
    """PCG to 1e-6 on the same points.  At l = 1 the NFFT-approximated kernel of this data is
    indefinite (bhat_k < 0 for a Gaussian truncated at r = 1/2; DESIGN.md 'SPD'), which is why the
    reference solves with FGMRES; CG needs an SPD operator, so it runs at l = 0.1 (all bhat_k > 0).
    With a distributed operator (N > 1) the same Nfft4GPSolverPcg runs on this rank's rows (rows =
    (rb, re)); the time is the max over ranks."""
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    assert op.setup(amd.GAUSSIAN, f=1.0, l=l_pcg, mu=0.01) == 0
    rb, re = rows if rows is not None else (0, n)
    rng = np.random.default_rng(rng_seed + 1)
    b = torch.tensor((rng.random(n) - 0.5)[rb:re], device="cuda")
    x = torch.zeros(re - rb, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.time()
    _, relres, hist, iters = amd.pcg(op, b, x, maxits=maxits, tol=tol)
    torch.cuda.synchronize()
    t = time.time() - t0
    if dist is not None:
        tt = torch.tensor([t], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    out = {"_time_s": t, "_iters": iters, "_rel_res": relres, "_converged": iters > 0, "_tol": tol, "_l": l_pcg,
           "_ms_per_iter": 1e3 * t / max(iters if iters > 0 else len(hist) - 1, 1)}
    out = {prefix + k: v for k, v in out.items()}
    if prefix == "pcg":
        out["pcg_precond"] = "none"
    return out


def run_pcg_nystrom(op, torch, n, k, rng_seed=906, tol=1e-6, maxits=3000, l_pcg=0.1):
    """PCG to 1e-6 with a rank-k Nystrom preconditioner set up on the GPU (nys.c:518-660 restated,
    K11 = K(perm[:k], perm[:k]) -- the reference's own K11 is built from the wrong points)."""
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    assert op.setup(amd.GAUSSIAN, f=1.0, l=l_pcg, mu=0.01) == 0
    perm = np.random.default_rng(rng_seed + 2).permutation(n).astype(np.int32)
    # the first setup in a process also pays rocSOLVER's initialisation; an optimizer loop re-runs the
    # setup every loss evaluation (gp_loss.c:163-166), so the second (steady-state) setup is reported
    torch.cuda.synchronize()
    t0 = time.time()
    pre = amd.NystromPrecond.from_additive(op, perm, k, k11="landmarks")
    torch.cuda.synchronize()
    t_setup_first = time.time() - t0
    # the steady-state setup: the median of three (each rebuilds the factors from scratch)
    setups = []
    for _ in range(3):
        pre.free()
        torch.cuda.synchronize()
        t0 = time.time()
        pre = amd.NystromPrecond.from_additive(op, perm, k, k11="landmarks")
        torch.cuda.synchronize()
        setups.append(time.time() - t0)
    t_setup = float(np.median(setups))
    ms = pre.setup_times()
    flops = 2.0 * n * k * k  # each of the three n x k x k products
    mfma = {"kernel": "k_gemm_f64 (v_mfma_f64_16x16x4)", "peak": F64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
            "flops_per_product": flops, "panel_ms": ms["panel"]}
    for key in ("gemm1", "gram", "gemm2"):
        tf = flops / (ms[key] * 1e-3) / 1e12 if ms[key] > 0 else None
        mfma[key] = {"ms": ms[key], "achieved": tf, "frac": tf / F64_MFMA_PEAK_TFS if tf else None}
    b = torch.tensor(np.random.default_rng(rng_seed + 1).random(n) - 0.5, device="cuda")
    x = torch.zeros(n, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    t0 = time.time()
    _, relres, hist, iters = amd.pcg(op, b, x, maxits=maxits, tol=tol, precond=pre)
    torch.cuda.synchronize()
    t = time.time() - t0
    # the same solve with the apply reading an fp32 copy of U (fp64 accumulation; PCG still stops on its
    # fp64 true residual): half the bytes of the two HBM-bound passes
    pre.set_storage(32)
    x32 = torch.zeros(n, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    t1 = time.time()
    _, relres32, _, iters32 = amd.pcg(op, b, x32, maxits=maxits, tol=tol, precond=pre)
    torch.cuda.synchronize()
    t32 = time.time() - t1
    pre.free()
    return {"pcg_nys_f32u_time_s": t32, "pcg_nys_f32u_iters": iters32, "pcg_nys_f32u_rel_res": relres32,
            "pcg_nys_rank": k, "pcg_nys_setup_s": t_setup, "pcg_nys_time_s": t, "pcg_nys_iters": iters,
            "pcg_nys_rel_res": relres, "pcg_nys_total_s": t_setup + t, "pcg_nys_setup_first_s": t_setup_first,
            "pcg_nys_setup_samples_s": setups, "nys_setup_mfma": mfma}


def run_fgmres(op, torch, n, rng_seed=906, tol=1e-6, kdim=1000, maxits=1000, l=1.0, rows=None, dist=None, ortho=0):
    """FGMRES (the reference's solver for this system, gp_loss.c:199-213; fgmres.c:3-252) to 1e-6 at the
    metric's own l = 1, where the NFFT-approximated kernel is indefinite and CG cannot run.  The spectrum
    has ~1000 outlying Fourier modes around mu = 0.01, so a restarted FGMRES stagnates (restart 50: 2.7e-2
    after 3000 iterations; tools/fgmres_probe.py) and it runs unrestarted (kdim = maxits = 1000; converges
    in ~330).  ortho 0: the reference's modified Gram-Schmidt; 1: block classical Gram-Schmidt with the DGKS
    second pass; 2: delayed CGS2, two basis sweeps per step (Nfft4GPAmdSetFgmresOrtho).  With a distributed operator every rank runs it on its rows (time: max over
    ranks)."""
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    assert op.setup(amd.GAUSSIAN, f=1.0, l=l, mu=0.01) == 0
    amd.lib().Nfft4GPAmdSetFgmresOrtho(ortho)
    amd.lib().Nfft4GPAmdFgmresSecondPasses()  # reset the DGKS counter
    rb, re = rows if rows is not None else (0, n)
    b = torch.tensor((np.random.default_rng(rng_seed + 1).random(n) - 0.5)[rb:re], device="cuda")
    x = torch.zeros(re - rb, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.time()
    _, relres, hist, iters = amd.fgmres(op, b, x, kdim=kdim, maxits=maxits, tol=tol)
    torch.cuda.synchronize()
    t = time.time() - t0
    amd.lib().Nfft4GPAmdSetFgmresOrtho(0)
    if dist is not None:
        tt = torch.tensor([t], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    p = ["fgmres_", "fgmres_cgs2_", "fgmres_dcgs2_"][ortho]
    extra = {p + "second_passes": int(amd.lib().Nfft4GPAmdFgmresSecondPasses())} if ortho == 1 else {}
    return {**extra, p + "time_s": t, p + "iters": iters, p + "rel_res": relres, p + "converged": relres <= tol,
            p + "tol": tol, p + "l": l, p + "kdim": kdim, p + "ms_per_iter": 1e3 * t / max(iters, 1),
            p + "ortho": ["modified Gram-Schmidt (fgmres.c)",
                          "block classical Gram-Schmidt, second pass by the DGKS test",
                          "delayed CGS2 (second pass lagged one step, two basis sweeps per step)"][ortho]}


def run_pcg_afn(op, X, torch, n, k, lfil=20, rng_seed=906, tol=1e-6, maxits=3000, l_pcg=0.1, schur="fsai",
                order="random"):
    """PCG to 1e-6 with the AFN preconditioner (BASELINE configs[1-2]: "AFN rank=512") of the same dense
    additive kernel, set up on the GPU the way the reference's Nfft4GPPrecondAFNSetup does it
    (Nfft4GPAmdPrecondAFNSetup, afn.c:161-489): rank estimation with max_k = k, then the AFN when the
    estimate reaches max_k, or the rank-k' Nystrom the reference switches to when it does not
    (afn.c:294-304; reported as ..._kind "nystrom" with the estimated rank)."""
    import ctypes
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    assert op.setup(amd.GAUSSIAN, f=1.0, l=l_pcg, mu=0.01) == 0
    ctypes.CDLL(None).srand(807)  # the rank estimation and random order draw libc rand() as the reference's
    torch.cuda.synchronize()
    t0 = time.time()
    pre = amd.PrecondAFN(X, k, perm_opt=order, schur=schur, schur_lfil=lfil, op=op)
    torch.cuda.synchronize()
    t_setup = time.time() - t0
    b = torch.tensor(np.random.default_rng(rng_seed + 1).random(n) - 0.5, device="cuda")
    x = torch.zeros(n, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    t0 = time.time()
    _, relres, hist, iters = amd.pcg(op, b, x, maxits=maxits, tol=tol, precond=pre)
    torch.cuda.synchronize()
    t = time.time() - t0
    r = torch.rand(n, dtype=torch.float64, device="cuda")
    pre.solve(x, r)
    torch.cuda.synchronize()
    t1 = time.time()
    for _ in range(10):
        pre.solve(x, r)
    torch.cuda.synchronize()
    t_apply = (time.time() - t1) / 10
    # the same solve with the apply's K12 (or the Nystrom branch's U) read as an fp32 copy, fp64 accumulation
    pre.set_storage(32)
    x32 = torch.zeros(n, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    t1 = time.time()
    _, relres32, _, iters32 = amd.pcg(op, b, x32, maxits=maxits, tol=tol, precond=pre)
    torch.cuda.synchronize()
    t32 = time.time() - t1
    pre.solve(x, r)
    torch.cuda.synchronize()
    t1 = time.time()
    for _ in range(10):
        pre.solve(x, r)
    torch.cuda.synchronize()
    t_apply32 = (time.time() - t1) / 10
    # the same solve with K12^T y1 and K12 y2 as matvecs of the additive operator itself (Nfft4GPAmdAfnSetOperator:
    # the NFFT operator's approximation of the dense kernel instead of the stored K12)
    op_leg = {}
    if pre.kind == "afn":
        pre.set_storage(64)
        pre.set_operator(op)
        xo = torch.zeros(n, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        t1 = time.time()
        _, relres_o, _, iters_o = amd.pcg(op, b, xo, maxits=maxits, tol=tol, precond=pre)
        torch.cuda.synchronize()
        t_o = time.time() - t1
        pre.solve(x, r)
        torch.cuda.synchronize()
        t1 = time.time()
        for _ in range(10):
            pre.solve(x, r)
        torch.cuda.synchronize()
        t_apply_o = (time.time() - t1) / 10
        pre.set_operator(None)
        op_leg = {"op_time_s": t_o, "op_iters": iters_o, "op_rel_res": relres_o, "op_apply_ms": 1e3 * t_apply_o}
    kind, rank = pre.kind, pre.k
    pre.free()
    key = "pcg_afn" if schur == "fsai" else "pcg_afn_" + schur
    if order != "random":
        key += "_" + order
    out = {key + "_max_k": k, key + "_kind": kind, key + "_rank": rank, key + "_order": order,
           key + "_schur": schur, key + "_schur_lfil": lfil if schur == "fsai" else None,
           key + "_setup_s": t_setup, key + "_time_s": t, key + "_iters": iters, key + "_rel_res": relres,
           key + "_total_s": t_setup + t, key + "_apply_ms": 1e3 * t_apply, key + "_f32_time_s": t32,
           key + "_f32_iters": iters32, key + "_f32_rel_res": relres32, key + "_f32_apply_ms": 1e3 * t_apply32}
    out.update({key + "_" + kk: v for kk, v in op_leg.items()})
    return out


def run_config_e(torch, steps, warmup, traffic=True, n=10_000_000, d=64, precisions=(64, 32), tag="configs[4]",
                 with_loss=True):
    """BASELINE configs[4]'s operator on one GPU, under the same clock as the headline: n = 1e7 points, 64 1-D
    windows (Gaussian f = 1, l = 1, mu = 0.01), the additive matvec with x, y in HBM, out of the 256 MB
    Infinity Cache (the layout is 2.8-3.5 GB per pass).  Two legs: the fp64 default records and the 32-bit
    records configs[4] grants (fp32 coordinates, fp64 accumulation; Nfft4GPAmdSetPrecision).  Each leg: pre-warm,
    W warmup, K timed matvecs between synchronisations, then the same K with dispatch-attached hipEvents for the
    per-kernel durations, and a roofline for k_spread and k_interp against SURVEY 8(d)'s configs[4] bytes:
    fp32 coordinates, n (4d + 4) for the spread pass (coordinates + v) and n (4d + 8) for the interpolation pass
    (coordinates + y written); the PMC HBM bytes per launch beside them."""
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    t0 = time.time()
    X, x_host = make_problem(n, d)
    gen_s = time.time() - t0
    win = np.arange(d, dtype=np.int32)
    xd = torch.tensor(x_host, device="cuda")
    yd = torch.zeros(n, dtype=torch.float64, device="cuda")
    y_loss = R_loss = None
    if with_loss:  # the loss leg's labels and its fixed Rademacher probes (probe-major = column-major n x nvecs)
        rng = np.random.default_rng(909)
        y_loss = rng.random(n) - 0.5
        R_loss = torch.tensor(np.where(rng.random((10, n)) < 0.5, -1.0, 1.0), device="cuda")
    survey = {"spread": n * (4 * d + 4), "interp": n * (4 * d + 8)}
    out = {"workload": f"BASELINE {tag} operator on 1 GPU: additive NFFT matvec, n={n}, d={d}, {d} x 1-D windows, "
                       f"Gaussian f=1 l=1 mu=0.01 (synthetic: numpy PCG64 seed 906)",
           "n": n, "d": d, "steps": steps, "warmup": warmup, "data_gen_s": gen_s,
           "survey_bytes_per_matvec": n * (8 * d + 12),
           "survey_bytes_def": "SURVEY 8(d) configs[4]'s form: n (4*2d + 4 + 8), fp32 coordinates and v, fp64 y"}
    if tag != "configs[4]":  # SURVEY 8(d)'s fp64 form for the fp64 configs: 8 n (d + 1) per pass
        survey = {"spread": 8 * n * (d + 1), "interp": 8 * n * (d + 1)}
        out["survey_bytes_per_matvec"] = 8 * n * (2 * d + 2)
        out["survey_bytes_def"] = "SURVEY 8(d): 8 n (2d + 2), fp64 coordinates and vectors"
    for bits in precisions:
        t0 = time.time()
        op = amd.NFFTAdditiveKernel(X, win, d, 1)
        if bits == 32:
            op.set_precision(32)
        if op.setup(amd.GAUSSIAN, f=1.0, l=1.0, mu=0.01) != 0:
            raise SystemExit("config E setup failed")
        torch.cuda.synchronize()
        setup_s = time.time() - t0
        t_end = time.perf_counter() + 0.5
        while time.perf_counter() < t_end:
            for _ in range(20):
                op.matsymv(xd, 1.0, 0.0, yd)
            torch.cuda.synchronize()
        for _ in range(warmup):
            op.matsymv(xd, 1.0, 0.0, yd)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            op.matsymv(xd, 1.0, 0.0, yd)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        op.timing(True)
        torch.cuda.synchronize()
        for _ in range(steps):
            op.matsymv(xd, 1.0, 0.0, yd)
        torch.cuda.synchronize()
        avg = {k: ms / max(c, 1) for k, (ms, c) in op.timing_query().items()}
        op.timing(False)
        info = op.layout_info()
        loss_rec = None
        if with_loss:
            loss_rec = config_e_loss(op, torch, X, y_loss, R_loss, d)
        op.free()
        pmc = None
        if traffic:
            try:
                pmc = pmc_traffic(n, d, precision=bits)
            except Exception:
                pmc = None
        rl = {}
        for k in ("spread", "interp"):
            a = survey[k] / (avg[k] * 1e-3) / 1e9
            tr = pmc.get(k, {}).get("traffic") if pmc else None
            rl["k_" + k] = {"bound": "hbm", "achieved": a, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": a / HBM_PEAK_GBS, "traffic": tr, "algorithmic_bytes_per_launch": survey[k],
                            "avg_launch_ms": avg[k],
                            "achieved_pmc": tr / (avg[k] * 1e-3) / 1e9 if tr else None,
                            "frac_pmc": tr / (avg[k] * 1e-3) / 1e9 / HBM_PEAK_GBS if tr else None}
        dom = "k_spread" if avg["spread"] >= avg["interp"] else "k_interp"
        out[f"f{bits}"] = {
            "value": steps / el, "unit": "matvecs/s", "ms_per_step": 1e3 * el / steps,
            "frac_of_survey_bytes": out["survey_bytes_per_matvec"] / (el / steps) / 1e9 / HBM_PEAK_GBS,
            "records": "fp64 default, 5 B per (point, window)" if bits == 64 else
                       "32-bit records (fp32 coordinates, fp64 accumulation), 4 B per (point, window)",
            "setup_s": setup_s, "kernels_ms": avg, "layout": info,
            "roofline": dict(rl[dom], kernel=dom), "roofline_per_kernel": rl,
            "traffic_unit": "bytes per launch (2 x FETCH_SIZE + WRITE_SIZE)"}
        if loss_rec is not None:
            out[f"f{bits}"]["loss"] = loss_rec
    return out


def config_b_pcg(torch, n=100_000, d=8, k=256):
    """BASELINE configs[1]'s solve: PCG to 1e-6 at n = 1e5, 8 1-D windows, l = 0.1, without a preconditioner, with
    the rank-256 Nystrom and with the rank-256 AFN (Schur FSAI and I/mu; each also with its K12 products through
    the operator), the same legs as config C's."""
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    X, _ = make_problem(n, d)
    op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
    out = {}
    out.update(run_pcg_single(op, torch, n))
    out.update(run_pcg_nystrom(op, torch, n, k))
    out.update(run_pcg_afn(op, X, torch, n, k, schur="fsai"))
    out.update(run_pcg_afn(op, X, torch, n, k, schur="noise"))
    op.free()
    return {kk: v for kk, v in out.items() if not kk.startswith("nys_setup_mfma")}


def config_e_loss(op, torch, X, y, R, d, maxits=50, nvecs=10, l=0.1):
    """BASELINE configs[4]'s step on one GPU: one Nfft4GPGpLoss (gp_loss.c:96-307: FGMRES for K^-1 y with the
    reference's MGS, nvecs Rademacher probes x maxits Lanczos steps, the gradient matvecs) on the leg's handle
    at (f, l, mu) = (1, 0.1, 0.01), identity transform (l = 0.1: the NFFT operator is SPD there)."""
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    win = np.arange(d, dtype=np.int32)
    torch.cuda.synchronize()
    t0 = time.time()
    with _StdoutToStderr():
        loss, grad = amd.gp_loss(X, win, d, 1, y, (1.0, l, 0.01), maxits=maxits, nvecs=nvecs, rademacher=R,
                                 tol=1e-6, transform=3, op=op)
        torch.cuda.synchronize()
    t = time.time() - t0
    return {"time_s": t, "value": loss, "grad": [float(g) for g in grad], "maxits": maxits, "nvecs": nvecs, "l": l,
            "fgmres_ortho": "modified Gram-Schmidt (the reference's)"}


class _StdoutToStderr:
    """The reference's loss prints progress with printf (gp_loss.c 'Transform ...'); the bench's stdout must
    carry only the JSON line, so C-level stdout goes to stderr inside this block."""

    def __enter__(self):
        import ctypes
        self.libc = ctypes.CDLL(None)
        sys.stdout.flush()
        self.libc.fflush(None)
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        self.libc.fflush(None)
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def run_loss(op, torch, n, d, X, rng_seed=906, maxits=50, nvecs=10, rows=None, dist=None, l=0.1, ortho=0):
    """One log-marginal-likelihood + gradient evaluation (Nfft4GPGpLoss, gp_loss.c:96-307: FGMRES for K^-1 y,
    stochastic Lanczos quadrature with nvecs Rademacher probes of maxits steps, the gradient matvecs) on the
    bench's operator at (f, l, mu) = (1, 0.1, 0.01), identity transform -- the loop BASELINE configs[4] runs
    at n = 1e7 on 8 GPUs, here at the bench's size.  l = 0.1 as for PCG: at l = 1 the NFFT operator is
    indefinite and the quadrature's Lanczos solve (lanczos.c, an LDL^T recursion of T) breaks
    down, so the gradient comes out NaN there, as the reference's would.  With a distributed operator every
    rank runs it on its rows (krylov.hip sums every inner product over the ranks); time: max over ranks.
    ortho 2: the loss's FGMRES solve with delayed CGS2 instead of the reference's MGS (loss_dcgs2_*)."""
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    rb, re = rows if rows is not None else (0, n)
    amd.lib().Nfft4GPAmdSetFgmresOrtho(ortho)
    rng = np.random.default_rng(rng_seed + 3)
    y = rng.random(n) - 0.5
    R = np.where(rng.random((n, nvecs)) < 0.5, -1.0, 1.0)
    win = np.arange(d, dtype=np.int32)
    Rl = torch.tensor(np.asfortranarray(R[rb:re]).T.copy(), device="cuda")  # probe-major = column-major n x nvecs
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.time()
    with _StdoutToStderr():
        loss, grad = amd.gp_loss(X, win, d, 1, y[rb:re], (1.0, l, 0.01), maxits=maxits, nvecs=nvecs,
                                 rademacher=Rl, tol=1e-6, transform=3, op=op)
        torch.cuda.synchronize()
    t = time.time() - t0
    amd.lib().Nfft4GPAmdSetFgmresOrtho(0)
    if dist is not None:
        tt = torch.tensor([t], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    if ortho == 2:
        return {"loss_dcgs2_time_s": t, "loss_dcgs2_value": loss, "loss_dcgs2_grad": [float(g) for g in grad]}
    return {"loss_time_s": t, "loss_value": loss, "loss_grad": [float(g) for g in grad], "loss_maxits": maxits,
            "loss_nvecs": nvecs, "loss_l": l}


def peer_enable_verified(op, xd, dist):
    """N > 1, rows: switch the operator to the peer-memory exchange (Nfft4GPAmdDistPeerEnable) if every rank can,
    and keep it only if its matvec equals the communicator all-reduce's (relative difference <= 1e-12, max over
    the ranks).  Every step that can fail on one rank only is followed by an all-reduced failure flag, so all
    ranks take the same branch.  Returns the record for the line."""
    import torch

    def agree(ok):
        t = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64, device="cuda")
        dist.all_reduce(t)
        return float(t.item()) == 0.0

    y_ref = op.matsymv(xd).clone()
    if not op.enable_peer():
        return {"enabled": False, "reason": "Nfft4GPAmdDistPeerEnable refused (a rank could not export or open)"}
    ok, rel, err = True, None, None
    try:
        y_p = op.matsymv(xd)
        op.check()
        rel = float(torch.linalg.norm(y_p - y_ref) / torch.linalg.norm(y_ref))
    except RuntimeError as e:
        ok, err = False, str(e)
    t = torch.tensor([rel if rel is not None else float("inf")], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    rel = float(t.item())
    if not agree(ok) or not rel <= 1e-12:
        # the exchange opened on every rank but its matvec timed out or differs from the all-reduce's: that is a
        # defect, not a configuration the bench may quietly route around
        raise SystemExit(f"bench: the peer-memory exchange failed its check on rank {int(os.environ.get('RANK', 0))}: "
                         f"{'timed out (' + err + ')' if err else 'matvec differs from the all-reduce by %.3g' % rel}; "
                         f"rerun with --no-peer to measure the all-reduce path")
    return {"enabled": True, "verified": True, "max_rel_diff_vs_allreduce": rel,
            "how": "rank-order sum of every rank's IPC-shared grid slots inside the grid kernel (dist.hip), no "
                   "all-reduce; 16 KB of epoch-stamped words read per rank"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one process each); without a launcher N > 1 ranks are spawned here (default 1)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=32)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcg", action="store_true")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC passes")
    ap.add_argument("--nys-rank", type=int, default=512, help="rank of the Nystrom-preconditioned PCG (0: off)")
    ap.add_argument("--afn-rank", type=int, default=512, help="rank of the AFN-preconditioned PCG (0: off)")
    ap.add_argument("--afn-schur", default="both", choices=["fsai", "noise", "both"],
                    help="AFN Schur-complement solve: kernel FSAI (schur_opt 3), I/mu (0) or both")
    ap.add_argument("--afn-order", default="both", choices=["random", "fps", "both"],
                    help="AFN landmark order: random (perm_opt 0) or farthest points (1)")
    ap.add_argument("--partition", default="rows", choices=["rows", "components"],
                    help="N > 1: the headline split (the other one is timed too)")
    ap.add_argument("--cpu-threads", type=int, default=16, help="OpenMP threads of the CPU baseline")
    ap.add_argument("--no-peer", action="store_true", help="N > 1, rows: skip the peer-memory exchange leg")
    ap.add_argument("--kernel-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-baseline-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-oracle-so", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--kernel-only-nys", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--kernel-only-precision", type=int, default=64, help=argparse.SUPPRESS)
    ap.add_argument("--precision", type=int, default=64, choices=[32, 64],
                    help="N = 1 headline leg: the fp64 records (default) or the 32-bit records (A/B at other sizes)")
    ap.add_argument("--no-config-e", action="store_true",
                    help="N = 1: skip the BASELINE configs[4]-size matvec leg (n = 1e7, 64 windows)")
    ap.add_argument("--launcher-selftest", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--launcher-selftest-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    if "--cpu-baseline-child" in sys.argv:  # the child's --cpu-threads is a list "16,1"
        i = sys.argv.index("--cpu-threads")
        threads_list = [int(t) for t in sys.argv[i + 1].split(",")]
        del sys.argv[i:i + 2]
        args = ap.parse_args()
        cpu_baseline_child(args.n, args.d, args.cpu_oracle_so, threads_list)
        return
    args = ap.parse_args()
    if args.kernel_only:
        kernel_only(args.n, args.d, args.kernel_only_nys, args.kernel_only_precision)
        return
    mode, nranks = resolve_world(args.gpus)
    if mode == "spawn":
        raise SystemExit(spawn_ranks(nranks, sys.argv[1:]))
    if args.launcher_selftest:
        launcher_selftest(args.launcher_selftest_fail_rank)
        return

    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; NFFT4GP_BENCH_BACKEND=gloo rehearses the N > 1 path with several ranks on
    # one GPU (RCCL refuses duplicate devices); the driver's multi-GPU runs use the default, nccl (RCCL)
    if world > 1 and os.environ.get("NFFT4GP_BENCH_BACKEND", "nccl") != "gloo" and torch.cuda.device_count() < world:
        raise SystemExit(f"bench: {world} ranks with RCCL need {world} visible GPUs, this box has "
                         f"{torch.cuda.device_count()}")
    dev = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    # one dedicated stream for torch and the library: launches on the legacy null stream carry its implicit
    # synchronisation and cost ~8 us per matvec (tools/graph_probe.py: 93 -> 85 us at config C)
    torch.cuda.set_stream(torch.cuda.Stream())
    if world > 1:
        import torch.distributed as dist
        with _StdoutToStderr():  # gloo announces its peers on stdout; the line must be stdout's only content
            dist.init_process_group(os.environ.get("NFFT4GP_BENCH_BACKEND", "nccl"))
    L = amd.lib()
    L.Nfft4GPAmdSetStream(torch.cuda.current_stream().cuda_stream)

    n, d = args.n, args.d
    X, x_host = make_problem(n, d)
    win = np.arange(d, dtype=np.int32)
    comm = None
    if world == 1:
        op = amd.NFFTAdditiveKernel(X, win, d, 1)
        if args.precision == 32:
            op.set_precision(32)
        rb, re = 0, n
    else:
        from preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd.dist import (
            Communicator, DistributedAdditiveKernel)
        # RCCL; the gloo rehearsal of several ranks on one GPU (RCCL refuses that) uses the group's own
        # all-reduce through a staging buffer instead
        gloo = os.environ.get("NFFT4GP_BENCH_BACKEND", "nccl") == "gloo"
        comm_kind = "rccl"
        with _StdoutToStderr():  # RCCL / gloo diagnostics go to stderr
            if gloo:
                comm, comm_kind = Communicator.callback(), "gloo"
            else:
                try:
                    comm = Communicator.rccl()
                except RuntimeError as e:  # the library's own RCCL communicator failed on every rank alike
                    print(f"bench: {e}; using torch's RCCL through Communicator.callback() instead", file=sys.stderr)
                    comm, comm_kind = Communicator.callback(), "callback"
        op = DistributedAdditiveKernel(X, win, d, 1, comm, partition=args.partition)
        rb, re = op.row_begin, op.row_end
    t0 = time.time()
    rc = op.setup(amd.GAUSSIAN, f=1.0, l=1.0, mu=0.01)
    setup_s = time.time() - t0
    if rc != 0:
        raise SystemExit("setup failed")
    xd = torch.tensor(x_host[rb:re], device="cuda")
    yd = torch.zeros(re - rb, dtype=torch.float64, device="cuda")

    def step():
        # N = 1: the whole matvec.  N > 1, rows: local spread -> all-reduce of the 32x64 grids -> local
        # interpolation; components: local windows -> all-reduce of y
        op.matsymv(xd, 1.0, 0.0, yd)

    def prewarm(seconds=0.5):
        """Untimed matvecs for `seconds` before the W warmup steps: the GPU leaves its idle clock state only
        after a few hundred back-to-back matvecs (measured: 92.3 us per matvec after 20 warmup steps, 85.6 us
        after 500, with the same kernel durations -- the gaps between the three launches shrink), and a
        running GP loop sits in the busy state.  The timed region is unchanged: exactly K steps."""
        torch.cuda.synchronize()
        t_end = time.perf_counter() + seconds
        while True:
            for _ in range(50):
                step()
            torch.cuda.synchronize()
            more = time.perf_counter() < t_end
            if world > 1:  # rank 0's clock decides, so every rank runs the same steps (collectives match)
                flag = torch.tensor([1.0 if more else 0.0], dtype=torch.float64, device="cuda")
                dist.broadcast(flag, src=0)
                more = bool(flag.item())
            if not more:
                break

    # The PCG legs (the metric's second half) run first, after a pre-warm (the GPU's idle clock state costs
    # the first few hundred matvecs ~15 %, tools/warm_probe.py: 100 us per matvec cold, 85 us warm, back to
    # 100 us after 2 s idle).  Then the kernel is set up again at the matvec workload's l = 1 and the
    # pre-warm, the W warmup and the K timed steps follow.
    pcg = {}
    pcie_rate = None
    prewarm()
    if world == 1:
        # host-pointer calls (the reference's calling convention): x and y staged over PCIe each call
        xh = np.ascontiguousarray(x_host)
        yh = np.zeros(n)
        op.matsymv(xh, 1.0, 0.0, yh)
        reps_h = 20
        t0 = time.perf_counter()
        for _ in range(reps_h):
            op.matsymv(xh, 1.0, 0.0, yh)
        pcie_rate = reps_h / (time.perf_counter() - t0)
    if world == 1 and not args.no_pcg:
        pcg.update(run_loss(op, torch, n, d, X))
        pcg.update(run_loss(op, torch, n, d, X, ortho=2))
        pcg.update(run_fgmres(op, torch, n))
        pcg.update(run_fgmres(op, torch, n, ortho=1))
        pcg.update(run_fgmres(op, torch, n, ortho=2))
        pcg.update(run_pcg_single(op, torch, n))
        # the preconditioned legs are the metric's "PCG time with AFN rank=512": an exception here ends the
        # bench (no silent *_error key)
        if args.nys_rank > 0:
            pcg.update(run_pcg_nystrom(op, torch, n, args.nys_rank))
        if args.afn_rank > 0:
            for schur in (["noise", "fsai"] if args.afn_schur == "both" else [args.afn_schur]):
                for order in (["random", "fps"] if args.afn_order == "both" else [args.afn_order]):
                    pcg.update(run_pcg_afn(op, X, torch, n, args.afn_rank, schur=schur, order=order))
        if op.setup(amd.GAUSSIAN, f=1.0, l=1.0, mu=0.01) != 0:
            raise SystemExit("setup failed")

    prewarm()
    for _ in range(args.warmup):
        step()

    def gather_ranks(rec):
        """{key: value} of this rank -> {key: [value of rank 0, 1, ...]} on every rank (one all-reduce of a
        zero-padded world x keys table, which gloo and RCCL both take)."""
        keys = sorted(rec)
        tab = torch.zeros(world, len(keys), dtype=torch.float64, device="cuda")
        tab[rank] = torch.tensor([float(rec[k]) for k in keys], dtype=torch.float64)
        dist.all_reduce(tab)
        tab = tab.cpu().numpy()
        return {k: [float(v) for v in tab[:, i]] for i, k in enumerate(keys)}

    def rank_times(per, el_inst):
        """The per-rank instrumented timing of one partition, in microseconds per matvec."""
        return {"kernels_before_exchange_us": [1e3 * v for v in per["local_before_ms"]],
                "allreduce_us": [1e3 * v for v in per["allreduce_ms"]],
                "kernels_after_exchange_us": [1e3 * v for v in per["local_after_ms"]],
                "matvecs_timed": [int(v) for v in per["matvecs"]],
                "ms_per_step_instrumented": 1e3 * el_inst / args.steps,
                "source": "hipEvents on the library stream around each rank's kernels and its enqueued all-reduce "
                          "(components: each chunk's all-reduce on the comm stream), over a repeat of the timed steps"}

    def timed(instrumented):
        """K steps bracketed by barrier + synchronize; with `instrumented` every spread / grid / interp
        dispatch of the loop carries start / stop hipEvents (Nfft4GPAmdTimingEnable), so the per-kernel
        durations are measured over this same timed region."""
        if instrumented:
            op.timing(True)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        per = None
        if instrumented:
            if world == 1:
                per = {k: ms / max(c, 1) for k, (ms, c) in op.timing_query().items()}
            else:
                per = gather_ranks(op.timing_query())
            op.timing(False)
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64, device="cuda")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        return el, per

    # N > 1, rows: the grids go through the peer-memory exchange when every rank can and its matvec equals the
    # all-reduce's (the all-reduce is timed below as well)
    peer = None
    if world > 1 and args.partition == "rows" and not args.no_peer:
        peer = peer_enable_verified(op, xd, dist)
        if peer.get("verified"):
            prewarm()
            for _ in range(args.warmup):
                step()
    # the headline timed region is uninstrumented; it is repeated at once with dispatch-attached events on
    # every kernel (about 13 us per matvec of event overhead, reported as ms_per_step_instrumented) for the
    # per-kernel durations of the roofline
    elapsed, _ = timed(False)
    elapsed_inst, kern_avg = timed(True)
    if peer is not None and peer.get("verified"):
        op.check()  # a peer wait that gave up in the timed steps fails the bench (raises), loudly
    per_rank = rank_times(kern_avg, elapsed_inst) if world > 1 else None
    rows_allreduce = None
    if peer is not None and peer.get("verified"):
        # the same steps over the communicator's all-reduce, for comparison
        op.disable_peer()
        prewarm()
        for _ in range(args.warmup):
            step()
        el_a, _ = timed(False)
        el_ai, per_a = timed(True)
        rows_allreduce = {"value": args.steps / el_a, "ms_per_step": 1e3 * el_a / args.steps,
                          "per_rank": rank_times(per_a, el_ai)}
        # the solver legs below run over the exchange again: their grids and their small all-reduces (dots,
        # norms, Hessenberg columns: PeerComm, dist.hip) go through the peer buffers
        peer["solvers"] = bool(peer_enable_verified(op, xd, dist).get("verified"))
    alt = None
    if world > 1:
        # the other split, timed the same way (W warmup + K steps between barriers, max over ranks)
        other = "components" if args.partition == "rows" else "rows"
        op2 = DistributedAdditiveKernel(X, win, d, 1, comm, partition=other)
        if op2.setup(amd.GAUSSIAN, f=1.0, l=1.0, mu=0.01) != 0:
            raise SystemExit("setup failed")
        x2 = torch.tensor(x_host[op2.row_begin:op2.row_end], device="cuda")
        y2 = torch.zeros(op2.n, dtype=torch.float64, device="cuda")
        op_main, xd_main, yd_main = op, xd, yd
        op, xd, yd = op2, x2, y2
        prewarm()
        for _ in range(args.warmup):
            step()
        el2, _ = timed(False)
        el2_inst, per2 = timed(True)
        alt = {"partition": other, "value": args.steps / el2, "ms_per_step": 1e3 * el2 / args.steps,
               "all_reduce_bytes_per_matvec": 8 * (op2.n if other == "components" else d * 64),
               "per_rank": rank_times(per2, el2_inst)}
        if not args.no_pcg:
            alt.update(run_pcg_single(op2, torch, n, rows=(op2.row_begin, op2.row_end), dist=dist))
            alt.update(run_fgmres(op2, torch, n, rows=(op2.row_begin, op2.row_end), dist=dist, ortho=1))
        op2.free()
        op, xd, yd = op_main, xd_main, yd_main
    headline = n == 1_000_000 and d == 32
    cfg_tag = "BASELINE configs[2]" if headline else "reduced size, not a BASELINE config" \
        if (n, d) != (100_000, 8) else "BASELINE configs[1] sizes"
    result = {
        # BASELINE.json's metric at its headline config; a descriptive name at other sizes
        "metric": BASELINE_METRIC if headline else f"kernel matvecs/sec (additive NFFT matvec, n={n}, d={d})",
        "value": args.steps / elapsed,
        "unit": "matvecs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "ms_per_step_instrumented": 1e3 * elapsed_inst / args.steps if elapsed_inst else None,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64" if args.precision == 64 else "f32 records, f64 accumulation",
        "data": "synthetic: X ~ U[0,1)^d, x ~ U(-0.5,0.5), numpy PCG64 seed 906",
        "config": {"workload": f"additive NFFT matvec, n={n}, d={d}, {d} x 1-D windows, Gaussian f=1 l=1 "
                               f"mu=0.01 ({cfg_tag})" + (f"; {world} GPUs, {args.partition} sharded" if world > 1 else ""),
                   "n": n, "d": d, "nwindows": d, "setup_s": setup_s,
                   "parallelism": f"{args.partition}{world}" if world > 1 else "single"},
    }
    if world == 1:
        result.update(pcg)
        # per-kernel durations: dispatch-attached hipEvents over the instrumented repeat of the timed region
        # (the same begin / end timestamps rocprofv3's kernel trace reports; profiles/ holds that trace of
        # this command)
        info = op.layout_info()
        b_spread, b_interp = algorithmic_bytes(info, n, d)
        avg = kern_avg
        dom = "spread" if avg["spread"] >= avg["interp"] else "interp"
        # achieved = SURVEY.md 8(d)'s algorithmic bytes: one matvec moves 8n(2d+2) (fp64 coordinates and
        # vectors), of which the spread pass reads coords + v = 8n(d+1) and the interpolation pass reads
        # coords and writes y = 8n(d+1).  This layout stores the same information in 5 B per
        # (point, window), so it moves fewer bytes than that; the rate on the bytes it
        # actually moves is reported beside it (achieved_layout / frac_layout, and frac_pmc on the PMC
        # HBM bytes).
        survey_bytes = 8 * n * (d + 1)
        bytes_dom = b_spread if dom == "spread" else b_interp
        achieved = survey_bytes / (avg[dom] * 1e-3) / 1e9
        achieved_layout = bytes_dom / (avg[dom] * 1e-3) / 1e9
        traffic = None
        if not args.no_traffic:
            try:
                pmc = pmc_traffic(n, d)
            except Exception as e:  # report, do not fail the GPU measurement
                pmc = None
                result["pmc_error"] = repr(e)
            if pmc:
                result["pmc_bytes_per_launch"] = pmc
                traffic = pmc.get(dom, {}).get("traffic")
        result["roofline"] = {"bound": "hbm", "kernel": f"k_{dom}", "achieved": achieved, "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                              "traffic_unit": "bytes per launch (2 x FETCH_SIZE + WRITE_SIZE)",
                              "algorithmic_bytes_per_launch": survey_bytes,
                              "algorithmic_bytes_def": "SURVEY 8(d): 8n(d+1) per pass (fp64 coords + vector)",
                              "layout_bytes_per_launch": bytes_dom,
                              "achieved_layout": achieved_layout, "frac_layout": achieved_layout / HBM_PEAK_GBS,
                              "achieved_pmc": (traffic / (avg[dom] * 1e-3) / 1e9) if traffic else None,
                              "frac_pmc": (traffic / (avg[dom] * 1e-3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
                              "avg_launch_ms": avg[dom],
                              "avg_launch_source": f"dispatch-attached hipEvents over a repeat of the {args.steps} timed steps"}
        result["kernels_ms"] = avg
        result["kernels_ms_sum"] = sum(avg.values())
        result["layout"] = info
        # survey-defined whole-matvec bytes (fp64 coords: 8n(2d+2)) for reference
        result["matvec_bytes_survey_def"] = 8 * n * (2 * d + 2)
        result["pcie_inclusive_matvecs_per_s"] = pcie_rate
        if not args.no_config_e:
            result["config_e"] = run_config_e(torch, args.steps, args.warmup, traffic=not args.no_traffic)
            # BASELINE configs[1]'s operator (n = 1e5, 8 windows, fp64): cache-resident and launch-bound
            result["config_b"] = run_config_e(torch, max(args.steps, 200), args.warmup, traffic=False, n=100_000, d=8,
                                              precisions=(64,), tag="configs[1]", with_loss=False)
            if not args.no_pcg:
                result["config_b"].update(config_b_pcg(torch))
        if not args.no_cpu_baseline:
            try:
                result["cpu_baseline"] = cpu_baseline(n, d, threads=args.cpu_threads)
            except Exception as e:  # report, do not fail the GPU measurement
                result["cpu_baseline"] = {"value": None, "error": repr(e)}
    if world > 1:
        result["config"]["all_reduce_bytes_per_matvec"] = 8 * (op.n if args.partition == "components" else d * 64)
        result["rccl_ranks"] = comm.ranks() if comm_kind == "rccl" else None
        result["comm_ranks"] = comm.ranks()
        result["config"]["devices_visible"] = torch.cuda.device_count()
        result["per_rank"] = per_rank
        result["config"]["communicator"] = ("gloo rehearsal (host all-reduce)" if gloo else
                                            "RCCL (library-owned ncclComm, all-reduce enqueued by dist.hip)"
                                            if comm_kind == "rccl" else
                                            "RCCL through torch.distributed (callback fallback, synchronising)")
        if not args.no_pcg:
            result.update(run_pcg_single(op, torch, n, rows=(rb, re), dist=dist))
            result["pcg_impl"] = f"Nfft4GPSolverPcg on Nfft4GPAmdDistMatSymv ({args.partition}), device-controlled"
            result.update(run_fgmres(op, torch, n, rows=(rb, re), dist=dist))
            result.update(run_fgmres(op, torch, n, rows=(rb, re), dist=dist, ortho=1))
            result.update(run_fgmres(op, torch, n, rows=(rb, re), dist=dist, ortho=2))
            result.update(run_loss(op, torch, n, d, X, rows=(rb, re), dist=dist))
        result["partition_" + alt["partition"]] = alt
        if peer is not None:
            result["grid_exchange"] = "peer memory" if peer.get("verified") else "all-reduce"
            result["peer_exchange"] = peer
            if rows_allreduce is not None:
                result["rows_allreduce"] = rows_allreduce
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        op.free()
        comm.free()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
