"""Matvec rate with the three launches of each matvec captured in a HIP graph (torch.cuda.CUDAGraph over
the library stream) against plain back-to-back launches, config C."""
import sys, time, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd

n, d = 1_000_000, 32
rng = np.random.default_rng(906)
X = rng.random((n, d)); x = rng.random(n) - 0.5
op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
assert op.setup(amd.GAUSSIAN, f=1.0, l=1.0, mu=0.01) == 0
xd = torch.tensor(x, device="cuda"); yd = torch.zeros(n, dtype=torch.float64, device="cuda")
L = amd.lib()
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    L.Nfft4GPAmdSetStream(s.cuda_stream)
    for _ in range(50):
        op.matsymv(xd, 1.0, 0.0, yd)
    torch.cuda.synchronize()
    y_ref = yd.clone()
    K = 200
    for rep in range(3):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        for _ in range(K):
            op.matsymv(xd, 1.0, 0.0, yd)
        torch.cuda.synchronize(); t_plain = (time.perf_counter() - t0) / K
        print(f"plain: {t_plain*1e6:.1f} us/matvec", flush=True)
    g = torch.cuda.CUDAGraph()
    steps = 20
    with torch.cuda.graph(g, stream=s):
        L.Nfft4GPAmdSetStream(torch.cuda.current_stream().cuda_stream)
        for _ in range(steps):
            op.matsymv(xd, 1.0, 0.0, yd)
    L.Nfft4GPAmdSetStream(s.cuda_stream)
    for rep in range(3):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        for _ in range(K // steps):
            g.replay()
        torch.cuda.synchronize(); t_graph = (time.perf_counter() - t0) / K
        print(f"graph: {t_graph*1e6:.1f} us/matvec", flush=True)
    print("max diff graph vs plain", float((yd - y_ref).abs().max() / y_ref.abs().max()))
