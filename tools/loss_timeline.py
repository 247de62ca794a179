"""Where a GP loss + gradient's wall time goes on the device: run one Nfft4GPGpLoss at config E (or --n / --d)
between two marker kernels, then (with --trace, on the rocprofv3 kernel-trace CSV of that run) report the kernels'
busy time, the idle time between them and the largest idle gaps with the kernels around them.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lt -o lt -- python tools/loss_timeline.py
    python tools/loss_timeline.py --trace gpurun_out/lt/..._kernel_trace.csv
"""
import argparse
import csv
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(a):
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    rng = np.random.default_rng(906)
    X = np.asfortranarray(rng.random((a.n, a.d)))
    y = rng.random(a.n) - 0.5
    win = np.arange(a.d, dtype=np.int32)
    op = amd.NFFTAdditiveKernel(X, win, a.d, 1)
    if a.precision == 32:
        op.set_precision(32)
    assert op.setup(amd.GAUSSIAN, f=1.0, l=a.l, mu=0.01) == 0
    R = torch.tensor(np.where(np.random.default_rng(7).random((10, a.n)) < 0.5, -1.0, 1.0), device="cuda")
    for rep in range(2):  # the first loss warms the solver scratch; the second is the one traced
        mark = torch.full((17,), float(rep), dtype=torch.float64, device="cuda")  # marker kernel
        torch.cuda.synchronize()
        t0 = time.time()
        loss, grad = amd.gp_loss(X, win, a.d, 1, y, (1.0, a.l, 0.01), maxits=50, nvecs=10, rademacher=R,
                                 transform=3, op=op)
        torch.cuda.synchronize()
        t = time.time() - t0
        mark = torch.full((19,), float(rep), dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
    print(json.dumps({"n": a.n, "d": a.d, "loss_s": t, "loss": loss}), flush=True)


def analyse(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    fills = [i for i, k in enumerate(ks) if "FillFunctor" in k[2]]
    # the last two marker fills bracket the traced loss
    a, b = fills[-2], fills[-1]
    win = ks[a + 1:b]
    t0, t1 = win[0][0], max(e for _, e, _ in win)
    busy, gaps, end = 0, [], t0
    for i, (s, e, name) in enumerate(win):
        if s > end:
            gaps.append((s - end, win[i - 1][2] if i else "", name))
        busy += max(0, e - max(s, end))
        end = max(end, e)
    gaps.sort(reverse=True)
    by = {}
    for s, e, name in win:
        key = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][-60:]
        by[key] = by.get(key, 0) + (e - s)
    out = {"span_ms": (t1 - t0) / 1e6, "busy_ms": busy / 1e6, "idle_ms": (t1 - t0 - busy) / 1e6,
           "kernels": len(win), "gaps_over_20us": sum(1 for g in gaps if g[0] > 20000),
           "idle_in_gaps_over_20us_ms": sum(g[0] for g in gaps if g[0] > 20000) / 1e6,
           "top_gaps": [{"us": g[0] / 1e3, "after": g[1][:70], "before": g[2][:70]} for g in gaps[:12]],
           "busy_by_kernel_ms": {k: v / 1e6 for k, v in sorted(by.items(), key=lambda x: -x[1])[:15]}}
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--l", type=float, default=0.1)
    ap.add_argument("--precision", type=int, default=64)
    ap.add_argument("--trace", default=None)
    a = ap.parse_args()
    if a.trace:
        analyse(a.trace)
    else:
        run(a)


if __name__ == "__main__":
    main()
