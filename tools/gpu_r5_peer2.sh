#!/bin/bash
# peer exchange: tests + N = 8 shard probe with and without it (one GPU)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_peer.py > gpurun_out/peer_tests.log 2>&1 &&
timeout -k 10 120 python -u tools/shard_probe.py --ranks 8 > gpurun_out/shard8_rows.log 2>&1 &&
timeout -k 10 120 python -u tools/shard_probe.py --ranks 8 --peer > gpurun_out/shard8_peer.log 2>&1 &&
timeout -k 10 120 python -u tools/shard_probe.py --ranks 8 > gpurun_out/shard8_rows_b.log 2>&1 &&
timeout -k 10 120 python -u tools/shard_probe.py --ranks 8 --peer > gpurun_out/shard8_peer_b.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_peer8 -o run -- python3 tools/shard_probe.py --ranks 8 --peer --reps 500 > gpurun_out/shard8_peer_prof.log 2>&1
