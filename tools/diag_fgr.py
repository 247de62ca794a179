import sys, numpy as np
sys.path.insert(0, '/root/repo/tests'); sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/oracle')
import torch
from test_gpu_krylov import HostDenseOp, load
import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
z = load("pcg_synth"); k = load("krylov_synth")
op = HostDenseOp(np.asarray(z["X"]), float(k["f"]), float(k["l"]), float(k["mu"]))
b = torch.tensor(np.asarray(z["b"]), device="cuda")
for kd, mi, key in ((10, 60, "fgr"), (100, 400, "fg")):
    x = torch.zeros(op.n, dtype=torch.float64, device="cuda")
    x, rr, hist, it = amd.fgmres(op, b, x, kdim=kd, maxits=mi, tol=1e-8)
    h = np.asarray(k[key + "_hist"])
    m = min(it, int(k[key + "_iters"]))
    d = np.abs(hist[:m+1] - h[:m+1]) / h[:m+1]
    print(key, it, int(k[key+"_iters"]), " ".join(f"{v:.1e}" for v in d))
    xr = np.asarray(k[key + "_x"]); xc = x.cpu().numpy()
    print("x rel", np.linalg.norm(xc - xr) / np.linalg.norm(xr))
    # true residual of each
    K = op.K; bb = np.asarray(z["b"])
    print("true res ours", np.linalg.norm(bb - K @ xc) / np.linalg.norm(bb), "ref", np.linalg.norm(bb - K @ xr) / np.linalg.norm(bb))
