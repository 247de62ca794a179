"""k_gemm_f64 in isolation (Nfft4GPAmdDebugGemm): C = A B with A n x k (random, dense), B k x k (dense, or upper
triangular like the setup's first product), five back-to-back launches each, hipEvent-timed.
    python tools/gemm_probe2.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    import ctypes as C
    L = amd.lib()
    L.Nfft4GPAmdDebugGemm.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_longlong, C.c_void_p,
                                      C.c_longlong, C.c_void_p, C.c_longlong]
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    L.Nfft4GPAmdSetStream(s.cuda_stream)
    n, k = 1_000_000, 512
    g = torch.Generator(device="cuda").manual_seed(3)
    A = torch.rand(k, n, dtype=torch.float64, device="cuda", generator=g) - 0.5  # column-major n x k
    C = torch.empty(k, n, dtype=torch.float64, device="cuda")
    out = {}
    for name in ("dense", "triangular", "dense_again"):
        B = torch.rand(k, k, dtype=torch.float64, device="cuda", generator=g) - 0.5
        if name == "triangular":
            B = torch.triu(B)
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert L.Nfft4GPAmdDebugGemm(0, n, k, k, A.data_ptr(), n, B.data_ptr(), k, C.data_ptr(), n) == 0
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        out[name] = ts
    flops = 2.0 * n * k * k
    print(json.dumps({k2: {"ms": v, "frac_best": flops / (min(v) * 1e-3) / 1e12 / 78.6} for k2, v in out.items()}))


if __name__ == "__main__":
    main()
