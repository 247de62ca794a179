"""Host side of one distributed matvec step (rows partition, RCCL): wall time per step of
DistributedAdditiveKernel.matsymv against the same steps captured in a HIP graph (torch.cuda.CUDAGraph on
the library stream), on however many ranks torchrun starts (1 on a one-GPU box: the all-reduce is local).
    torchrun --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 tools/dist_step_probe.py --points 125000
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=125000)
    ap.add_argument("--d", type=int, default=32)
    ap.add_argument("--reps", type=int, default=400)
    ap.add_argument("--graph", type=int, default=1)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    from preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd.dist import (
        Communicator, DistributedAdditiveKernel)
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    dist.init_process_group("nccl")
    L = amd.lib()
    L.Nfft4GPAmdSetStream(s.cuda_stream)
    X = np.asfortranarray(np.random.default_rng(906).random((args.points, args.d)))
    comm = Communicator.rccl()
    op = DistributedAdditiveKernel(X, np.arange(args.d, dtype=np.int32), args.d, 1, comm, partition="rows")
    assert op.setup(amd.GAUSSIAN, f=1.0, l=1.0, mu=0.01) == 0
    x = torch.tensor(np.random.default_rng(1).random(op.row_end - op.row_begin) - 0.5, device="cuda")
    y = torch.zeros_like(x)
    for _ in range(200):
        op.matsymv(x, 1.0, 0.0, y)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        op.matsymv(x, 1.0, 0.0, y)
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / args.reps * 1e6
    out = {"rank": rank, "n_rows": op.row_end - op.row_begin, "eager_us_per_step": eager}
    y_ref = y.clone()
    if args.graph:
        try:
            g = torch.cuda.CUDAGraph()
            steps = 20
            with torch.cuda.graph(g, stream=s):
                L.Nfft4GPAmdSetStream(torch.cuda.current_stream().cuda_stream)
                for _ in range(steps):
                    op.matsymv(x, 1.0, 0.0, y)
            L.Nfft4GPAmdSetStream(s.cuda_stream)
            g.replay()
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.reps // steps):
                g.replay()
            torch.cuda.synchronize()
            out["graph_us_per_step"] = (time.perf_counter() - t0) / (args.reps // steps * steps) * 1e6
            out["graph_max_rel_diff"] = float((y - y_ref).abs().max() / y_ref.abs().max())
        except Exception as e:  # capture refused: report it
            out["graph_error"] = repr(e)[:300]
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
