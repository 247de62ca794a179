"""Per-workgroup timeline of k_spread (diagnostic variant 4, s_memrealtime stamps at 100 MHz)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

os.environ["NFFT4GP_AMD_SPREAD_VARIANT"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd  # noqa: E402

n, d = 1000000, 32
ranks = int(sys.argv[1]) if len(sys.argv) > 1 else 1  # > 1: the row shard [0, n / ranks) (tools/shard_probe.py)
rng = np.random.default_rng(906)
X = rng.random((n, d))
x = rng.random(n) - 0.5
nl = n // ranks
op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1, shard=(0, nl) if ranks > 1 else None)
assert op.setup(amd.GAUSSIAN, 1.0, 1.0, 0.01) == 0
xd = torch.tensor(x[:nl], device="cuda")
yd = torch.zeros(nl, dtype=torch.float64, device="cuda")
grid = torch.zeros(max(1, amd.lib().Nfft4GPAmdShardGridSize(op.h)), dtype=torch.float64, device="cuda")
for _ in range(5):
    if ranks > 1:
        amd.lib().Nfft4GPAmdShardSpread(op.h, xd.data_ptr(), grid.data_ptr())
    else:
        op.matsymv(xd, 1.0, 0.0, yd)
torch.cuda.synchronize()
info = op.layout_info()
ngroups, nblocks = info["ngroups"], info["nblocks"]
nwg = ((nblocks + 7) // 8) * 8 * ngroups
L = amd.lib()
f = L.Nfft4GPAmdDebugStamps
f.argtypes = [C.c_void_p, C.c_int]
out = np.zeros(nwg * 4, dtype=np.uint64)
f(out.ctypes.data, nwg)
s = out.reshape(nwg, 4).astype(np.float64) * 10.0 / 1000.0  # -> microseconds
valid = s[:, 0] > 0
s = s[valid]
t0 = s[:, 0].min()
s -= t0
pro = s[:, 1] - s[:, 0]
loop = s[:, 2] - s[:, 1]
fold = s[:, 3] - s[:, 2]
print(f"WGs {len(s)}  kernel span {s[:,3].max():.1f} us")
for nm, v in [("prologue", pro), ("loop", loop), ("fold", fold), ("total", s[:, 3] - s[:, 0])]:
    print(f"{nm:9s} mean {v.mean():6.2f}  p10 {np.percentile(v,10):6.2f}  p50 {np.median(v):6.2f}  p90 {np.percentile(v,90):6.2f} us")
starts = np.sort(s[:, 0])
print("start times percentiles (us):", [round(float(np.percentile(starts, p)), 1) for p in (0, 10, 25, 50, 75, 90, 100)])
# concurrency histogram over time
tt = np.linspace(0, s[:, 3].max(), 30)
conc = [int(np.sum((s[:, 0] <= t) & (s[:, 3] > t))) for t in tt]
print("resident WGs over time:", conc)
