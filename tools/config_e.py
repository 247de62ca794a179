"""BASELINE configs[4] on one GPU: n = 1e7, d = 64 additive (64 1-D windows), the additive NFFT matvec
and gradient matvec rates, and one log-marginal-likelihood + gradient evaluation (Nfft4GPGpLoss:
FGMRES for K^{-1} y, Lanczos quadrature with nvecs Rademacher probes for log det and the trace terms).

    python tools/config_e.py [--n 10000000] [--d 64] [--nvecs 10] [--maxits 50]

Prints one JSON line.  Synthetic data: X ~ U[0,1)^d, y ~ U(-0.5, 0.5) (numpy PCG64 seed 906).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--nvecs", type=int, default=10)
    ap.add_argument("--maxits", type=int, default=50)
    ap.add_argument("--reps", type=int, default=20)
    # l = 0.1: the NFFT-approximated Gaussian is SPD on U[0,1) data (at l >= 0.3 some bhat_k < 0, the
    # Lanczos Cholesky of T fails and the reference's gradient is NaN; DESIGN.md 'SPD')
    ap.add_argument("--l", type=float, default=0.1)
    ap.add_argument("--precision", type=int, default=64, choices=[32, 64],
                    help="Nfft4GPAmdSetPrecision: 64 (default records) or 32 (BASELINE configs[4]'s fp32 matvec)")
    args = ap.parse_args()
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    torch.cuda.set_device(0)
    L = amd.lib()
    L.Nfft4GPAmdSetStream(torch.cuda.current_stream().cuda_stream)
    n, d = args.n, args.d
    rng = np.random.default_rng(906)
    t0 = time.time()
    X = np.asfortranarray(rng.random((n, d)))
    y = rng.random(n) - 0.5
    t_gen = time.time() - t0
    win = np.arange(d, dtype=np.int32)
    out = {"workload": f"BASELINE configs[4] on 1 GPU: n={n}, d={d} ({d} x 1-D windows), Gaussian f=1 "
                       f"l={args.l} mu=0.01", "data_gen_s": t_gen}
    t0 = time.time()
    op = amd.NFFTAdditiveKernel(X, win, d, 1)
    if args.precision == 32:
        op.set_precision(32)
    out["precision"] = args.precision
    out["create_s"] = time.time() - t0
    t0 = time.time()
    assert op.setup(amd.GAUSSIAN, f=1.0, l=args.l, mu=0.01) == 0
    torch.cuda.synchronize()
    out["setup_s"] = time.time() - t0
    out["layout"] = op.layout_info()
    # bytes a matvec's kernels move: the layout in both passes, alpha, x and y, the partial grids written and read;
    # against SURVEY 8(d)'s figure for configs[4] (fp32 coordinates in both passes, 2 x 4 n d, plus the fp64 vector
    # read and y written, 16 n)
    lay = out["layout"]
    moved = 2 * lay["layout_bytes"] + 24 * n + 2 * 8 * lay["nblocks"] * d * 64
    out["bytes_moved_per_matvec"] = moved
    out["bytes_survey_fp32_per_matvec"] = 8 * n * d + 16 * n
    out["bytes_ratio"] = moved / out["bytes_survey_fp32_per_matvec"]
    xd = torch.tensor(y, device="cuda")
    yd = torch.zeros(n, dtype=torch.float64, device="cuda")
    gd = torch.zeros(3 * n, dtype=torch.float64, device="cuda")
    for _ in range(3):
        op.matsymv(xd, 1.0, 0.0, yd)
        op.gradmatsymv(xd, 1.0, 0.0, gd)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        op.matsymv(xd, 1.0, 0.0, yd)
    torch.cuda.synchronize()
    out["matvecs_per_s"] = args.reps / (time.perf_counter() - t0)
    t0 = time.perf_counter()
    for _ in range(args.reps):
        op.gradmatsymv(xd, 1.0, 0.0, gd)
    torch.cuda.synchronize()
    out["grad_matvecs_per_s"] = args.reps / (time.perf_counter() - t0)
    out["kernels_ms"] = {k: op.kernel_bench(k, xd, yd, reps=10) for k in op.KERNELS}
    # loss + gradient (gp_loss.c:96-307 through the C ABI; host label/data as the reference's driver), on
    # the same handle as an optimizer step would (its layout is already built)
    R = np.asfortranarray(np.where(np.random.default_rng(7).random((n, args.nvecs)) < 0.5, -1.0, 1.0))
    Rd = torch.tensor(R.ravel(order="F"), device="cuda")
    torch.cuda.synchronize()
    t0 = time.time()
    loss, grad = amd.gp_loss(X, win, d, 1, y, (1.0, args.l, 0.01), maxits=args.maxits, nvecs=args.nvecs,
                             rademacher=Rd, transform=3, op=op)
    torch.cuda.synchronize()
    out["loss_s"] = time.time() - t0
    out["loss"] = loss
    out["grad"] = [float(g) for g in grad]
    # the same loss with the loss's FGMRES solve orthogonalised by delayed CGS2 (Nfft4GPAmdSetFgmresOrtho(2))
    # instead of the reference's MGS; the Lanczos quadrature is unchanged
    L.Nfft4GPAmdSetFgmresOrtho(2)
    torch.cuda.synchronize()
    t0 = time.time()
    loss2, grad2 = amd.gp_loss(X, win, d, 1, y, (1.0, args.l, 0.01), maxits=args.maxits, nvecs=args.nvecs,
                               rademacher=Rd, transform=3, op=op)
    torch.cuda.synchronize()
    out["loss_dcgs2_s"] = time.time() - t0
    L.Nfft4GPAmdSetFgmresOrtho(0)
    out["loss_dcgs2_rel_diff"] = abs(loss2 - loss) / abs(loss)
    out["grad_dcgs2_rel_diff"] = float(np.max(np.abs(np.asarray(grad2) - np.asarray(grad)) / np.abs(np.asarray(grad))))
    out["nvecs"] = args.nvecs
    out["maxits"] = args.maxits
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
