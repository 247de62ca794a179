"""Times the Lanczos re-orthogonalisation's classical pass (Ctx::block_gs: h = V^T w in one launch, w -= Z h with
||w||^2 in another) at config E's n on device buffers, for several basis sizes m, and prints the rate against the
pass's algorithmic bytes: dots (m + 1) 8n (the m columns and w), update (m + 2) 8n (w read and written, m columns).

    python tools/reorth_probe.py [--n 10000000] [--m 2,8,26,50] [--reps 10] [--alias 1]
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--m", default="2,8,26,50")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--alias", type=int, default=1, help="Z = V (Lanczos without a preconditioner)")
    a = ap.parse_args()
    import torch
    from preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd import _lib
    L = _lib.lib()
    f = L.Nfft4GPAmdDebugBlockGs
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_longlong, C.c_int, C.c_int, C.c_int,
                  C.POINTER(C.c_float), C.POINTER(C.c_double)]
    L.Nfft4GPAmdSetStream(C.c_void_p(torch.cuda.current_stream().cuda_stream))
    ms_list = [int(s) for s in a.m.split(",")]
    mmax = max(ms_list)
    g = torch.Generator(device="cuda").manual_seed(5)
    V = torch.randn(mmax, a.n, device="cuda", dtype=torch.float64, generator=g)
    V /= V.norm(dim=1, keepdim=True)
    Z = V if a.alias else torch.randn(mmax, a.n, device="cuda", dtype=torch.float64, generator=g)
    out = []
    for m in ms_list:
        w = torch.randn(a.n, device="cuda", dtype=torch.float64, generator=g)
        t = C.c_float(0)
        h = (C.c_double * (m + 2))()
        torch.cuda.synchronize()
        rc = f(w.data_ptr(), V.data_ptr(), Z.data_ptr(), a.n, m, 0, a.reps, C.byref(t), h)
        assert rc == 0, rc
        byts = (2 * m + 3) * 8 * a.n
        rec = {"m": m, "us_per_pass": round(t.value * 1e3, 1), "GB_s": round(byts / (t.value * 1e-3) / 1e9, 1)}
        out.append(rec)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"n": a.n, "alias": a.alias, "passes": out}))


if __name__ == "__main__":
    main()
