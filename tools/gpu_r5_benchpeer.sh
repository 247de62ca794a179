#!/bin/bash
# the N > 1 bench line rehearsed with 2 gloo ranks on one GPU (self-launched), including the peer-exchange leg
set -o pipefail
mkdir -p gpurun_out
NFFT4GP_BENCH_BACKEND=gloo timeout -k 10 540 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-pcg > gpurun_out/bench_gloo2_peer.json 2> gpurun_out/bench_gloo2_peer.err
