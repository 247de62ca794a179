"""Sweep layout knobs (block size B, windows per spread group CG) and kernel variants for the config-C
matvec.  Each setting runs in a fresh subprocess (env vars are read at handle creation).
usage: python tools/sweep_layout.py "B,CG,SV,IV[,GPW]" ...   ("-" keeps the library default)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, sys, time, numpy as np, torch
sys.path.insert(0, %r)
import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
n, d = 1000000, 32
rng = np.random.default_rng(906); X = rng.random((n, d)); x = rng.random(n) - 0.5
op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
assert op.setup(amd.GAUSSIAN, 1.0, 1.0, 0.01) == 0
xd = torch.tensor(x, device="cuda"); yd = torch.zeros(n, dtype=torch.float64, device="cuda")
for _ in range(10): op.matsymv(xd, 1.0, 0.0, yd)
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(200): op.matsymv(xd, 1.0, 0.0, yd)
torch.cuda.synchronize(); el = time.perf_counter() - t
kb = {k: round(op.kernel_bench(k, xd, yd, reps=100), 4) for k in op.KERNELS}
print(json.dumps({"ms": round(el * 5, 4), **kb}))
''' % ROOT
configs = sys.argv[1:] or ["4096,4,0,0"]
for cfg in configs:
    parts = cfg.split(",")
    B, CG, SV, IV = parts[:4]
    GPW = parts[4] if len(parts) > 4 else "-"
    env = dict(os.environ, NFFT4GP_AMD_BLOCK=B, NFFT4GP_AMD_CG=CG)
    if GPW != "-":
        env["NFFT4GP_AMD_GPW"] = GPW
    if SV != "-":
        env["NFFT4GP_AMD_SPREAD_VARIANT"] = SV
    if IV != "-":
        env["NFFT4GP_AMD_INTERP_VARIANT"] = IV
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-300:]
    print(f"B={B} CG={CG} SV={SV} IV={IV} GPW={GPW} {line}", flush=True)
