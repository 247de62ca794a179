"""Probe: matvec time of consecutive timed loops (clock ramp / instrumentation overhead)."""
import os, sys, time, json
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
torch.cuda.set_device(0)
amd.lib().Nfft4GPAmdSetStream(torch.cuda.current_stream().cuda_stream)
n, d = 1_000_000, 32
rng = np.random.default_rng(906)
X = rng.random((n, d)); x = rng.random(n) - 0.5
op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
assert op.setup(amd.GAUSSIAN, 1.0, 1.0, 0.01) == 0
xd = torch.tensor(x, device="cuda"); yd = torch.zeros(n, dtype=torch.float64, device="cuda")
out = []
def loop(k, inst=False):
    if inst: op.timing(True)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(k): op.matsymv(xd, 1.0, 0.0, yd)
    torch.cuda.synchronize(); t = (time.perf_counter() - t0) / k * 1e6
    per = None
    if inst:
        per = {kk: round(ms / max(c, 1) * 1e3, 2) for kk, (ms, c) in op.timing_query().items()}; op.timing(False)
    out.append((k, inst, round(t, 2), per))
for _ in range(5): op.matsymv(xd, 1.0, 0.0, yd)
for k in (20, 20, 20, 200, 20, 200, 2000, 20, 200):
    loop(k)
loop(200, True); loop(200); loop(20, True); loop(20)
time.sleep(2.0); loop(20); loop(20); loop(200)
for o in out: print(o)
