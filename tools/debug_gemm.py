import ctypes as C, sys, numpy as np, torch
sys.path.insert(0, '.')
import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
L = amd.lib()
f = L.Nfft4GPAmdDebugGemm
f.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_longlong, C.c_void_p, C.c_longlong, C.c_void_p, C.c_longlong]
rng = np.random.default_rng(0)
for (tA, M, N, K) in [(0, 64, 64, 16), (0, 100, 70, 33), (1, 64, 64, 16), (1, 70, 50, 300)]:
    if tA:
        A = rng.standard_normal((K, M))
        ref = A.T @ (Bm := rng.standard_normal((K, N)))
    else:
        A = rng.standard_normal((M, K))
        ref = A @ (Bm := rng.standard_normal((K, N)))
    Ad = torch.tensor(np.asfortranarray(A).ravel(order='F'), device='cuda')
    Bd = torch.tensor(np.asfortranarray(Bm).ravel(order='F'), device='cuda')
    Cd = torch.zeros(M * N, dtype=torch.float64, device='cuda')
    lda = A.shape[0]
    rc = f(tA, M, N, K, Ad.data_ptr(), lda, Bd.data_ptr(), K, Cd.data_ptr(), M)
    Cm = Cd.cpu().numpy().reshape(N, M).T
    print(tA, M, N, K, rc, np.abs(Cm - ref).max())
    if np.abs(Cm - ref).max() > 1e-10:
        print(np.round(Cm[:6, :6] - ref[:6, :6], 3))
