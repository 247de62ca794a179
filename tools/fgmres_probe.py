import sys, time, numpy as np, torch
sys.path.insert(0, "/root/repo")
import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
torch.cuda.set_device(0)
s = torch.cuda.Stream(); torch.cuda.set_stream(s); amd.lib().Nfft4GPAmdSetStream(s.cuda_stream)
n, d = 1_000_000, 32
rng = np.random.default_rng(906); X = rng.random((n, d)); x = rng.random(n) - 0.5
op = amd.NFFTAdditiveKernel(X, np.arange(d, dtype=np.int32), d, 1)
assert op.setup(amd.GAUSSIAN, f=1.0, l=1.0, mu=0.01) == 0
b = torch.tensor(np.random.default_rng(907).random(n) - 0.5, device="cuda")
for kdim in [int(a) for a in sys.argv[1:]]:
    xs = torch.zeros_like(b); torch.cuda.synchronize(); t0 = time.time()
    _, rr, hist, it = amd.fgmres(op, b, xs, kdim=kdim, maxits=kdim, tol=1e-6)
    torch.cuda.synchronize()
    h = hist[:it+1]
    print(kdim, "iters", it, "rel", rr, "time", round(time.time()-t0, 3), "hist@", [float("%.2e" % h[i]) for i in range(0, len(h), max(1, len(h)//10))], flush=True)
# block CGS2 orthogonalisation (Nfft4GPAmdSetFgmresOrtho(1)) at the largest restart dimension given
amd.lib().Nfft4GPAmdSetFgmresOrtho(1)
kdim = int(sys.argv[-1])
xs = torch.zeros_like(b); torch.cuda.synchronize(); t0 = time.time()
_, rr, hist, it = amd.fgmres(op, b, xs, kdim=kdim, maxits=kdim, tol=1e-6)
torch.cuda.synchronize()
print("cgs2", kdim, "iters", it, "rel", rr, "time", round(time.time()-t0, 3), flush=True)
