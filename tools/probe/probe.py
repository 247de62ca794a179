import ctypes as C, sys, time, numpy as np
order = sys.argv[1]
if order == "torch_first":
    import torch; torch.cuda.init(); x = torch.ones(4, device="cuda")
L = C.CDLL(__file__.replace("probe.py", "librocsolver_probe.so"))
if order == "lib_first":
    pass
rng = np.random.default_rng(0)
for n in [64, 512]:
    B = rng.standard_normal((n, n)); A = np.asfortranarray(B @ B.T)
    w = np.zeros(n); V = np.zeros((n, n), order="F")
    t = time.time()
    rc = L.probe_syevd(A.ctypes.data_as(C.c_void_p), n, w.ctypes.data_as(C.c_void_p), V.ctypes.data_as(C.c_void_p))
    t = time.time() - t
    rc2 = L.probe_syevd(A.ctypes.data_as(C.c_void_p), n, w.ctypes.data_as(C.c_void_p), V.ctypes.data_as(C.c_void_p)); t2=time.time()
    print(order, n, "rc", rc, rc2, "err", np.abs(w - np.linalg.eigvalsh(A)).max() / np.abs(w).max(), "t", t)
if order == "lib_first":
    import torch; print("torch after:", torch.cuda.is_available())
