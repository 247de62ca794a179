"""Per-rank matvec time of an N-GPU run on one GPU, without the all-reduce:

* rows (default): Nfft4GPAmdShardSpread -> Nfft4GPAmdShardFinish for rows [0, n_global / N) of config C;
* components: rank 0 of the component split (BASELINE configs[3]: 4 of config C's 32 windows per GPU at
  N = 8) -- Nfft4GPAdditiveNFFTMatSymv on a handle of windows [0, nw / N) for all n points
  (Nfft4GPAmdAdditiveComponentShard, the mu x term on this rank).

* rows --peer: the same shard as a distributed operator over the peer-memory exchange (Nfft4GPAmdDistPeerEnable)
  on a one-process communicator with NFFT4GP_AMD_PEER_FAKE_WORLD = N: the exchange kernels wait for N flags and
  sum N slots (all this rank's own -- local reads where N GPUs would read N - 1 slots over xGMI), so the time
  includes the exchange's kernels but not the peers' link latency (timing only; y is not the operator's).

    python tools/shard_probe.py [--ranks 8] [--partition components] [--peer]
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
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=32)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2000)
    ap.add_argument("--partition", default="rows", choices=["rows", "components"])
    ap.add_argument("--peer", action="store_true")
    args = ap.parse_args()
    import torch
    import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd
    torch.cuda.set_device(0)
    L = amd.lib()
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    L.Nfft4GPAmdSetStream(s.cuda_stream)
    n, d = args.n, args.d
    X = np.asfortranarray(np.random.default_rng(906).random((n, d)))
    win = np.arange(d, dtype=np.int32)
    if args.partition == "rows":
        re = n // args.ranks
        op = amd.NFFTAdditiveKernel(X, win, d, 1, shard=(0, re))
        assert op.setup(amd.GAUSSIAN, f=1.0, l=1.0, mu=0.01) == 0
        h = op.h
        g = L.Nfft4GPAmdShardGridSize(h)
        grid = torch.zeros(g, dtype=torch.float64, device="cuda")
        if args.peer:
            import ctypes as C
            import torch.distributed as dist
            from preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd.dist import Communicator
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            dist.init_process_group("gloo", rank=0, world_size=1)
            comm = Communicator.callback()
            L.Nfft4GPAmdDistCreate.restype = C.c_void_p
            L.Nfft4GPAmdDistCreate.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
            dop = L.Nfft4GPAmdDistCreate(h, 0, comm.h)
            os.environ["NFFT4GP_AMD_PEER_FAKE_WORLD"] = str(args.ranks)
            assert L.Nfft4GPAmdDistPeerEnable(C.c_void_p(dop)) == 0
    else:
        re = n
        nwl = d // args.ranks
        op = amd.NFFTAdditiveKernel(X, win[:nwl], nwl, 1)
        assert L.Nfft4GPAmdAdditiveComponentShard(op.h, d, 1) == 0
        assert op.setup(amd.GAUSSIAN, f=1.0, l=1.0, mu=0.01) == 0
        h = op.h
    x = torch.tensor(np.random.default_rng(1).random(re) - 0.5, device="cuda")
    y = torch.zeros(re, dtype=torch.float64, device="cuda")

    def step():
        if args.peer:
            assert L.Nfft4GPAmdDistMatSymv(dop, re, 1.0, x.data_ptr(), 0.0, y.data_ptr()) == 0
        elif args.partition == "rows":
            assert L.Nfft4GPAmdShardSpread(h, x.data_ptr(), grid.data_ptr()) == 0
            assert L.Nfft4GPAmdShardFinish(h, grid.data_ptr(), 0, 1.0, x.data_ptr(), 0.0, y.data_ptr()) == 0
        else:
            op.matsymv(x, 1.0, 0.0, y)

    t_end = time.perf_counter() + 0.5
    while time.perf_counter() < t_end:
        for _ in range(50):
            step()
        torch.cuda.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        step()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / args.reps * 1e6
    print(json.dumps({"partition": args.partition + ("+peer" if args.peer else ""), "ranks": args.ranks, "rows": re,
                      "windows": d if args.partition == "rows" else d // args.ranks, "us_per_shard_matvec": us,
                      "y_norm": float(y.norm())}))


if __name__ == "__main__":
    main()
