#!/bin/bash
# the N > 1 bench line rehearsed with 2 gloo ranks on one GPU: torchrun, then self-launched
set -o pipefail
mkdir -p gpurun_out
NFFT4GP_BENCH_BACKEND=gloo timeout -k 10 540 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || { echo GLOO2_FAIL; tail -30 gpurun_out/bench_gloo2.err; exit 1; }
head -c 300 gpurun_out/bench_gloo2.json
NFFT4GP_BENCH_BACKEND=gloo timeout -k 10 540 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-pcg > gpurun_out/bench_gloo2_self.json 2> gpurun_out/bench_gloo2_self.err || { echo GLOO2_SELF_FAIL; tail -30 gpurun_out/bench_gloo2_self.err; exit 1; }
head -c 300 gpurun_out/bench_gloo2_self.json
