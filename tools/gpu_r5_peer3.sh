#!/bin/bash
# peer exchange with the partial-grid sum folded into the grid kernel: tests + N = 8 probes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_peer.py > gpurun_out/peer_tests.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_knn.py tests/test_gpu_dist.py > gpurun_out/knn_dist_tests.log 2>&1 &&
for k in 1 2; do
timeout -k 10 120 python -u tools/shard_probe.py --ranks 8 > gpurun_out/shard8_rows_$k.log 2>&1 &&
timeout -k 10 120 python -u tools/shard_probe.py --ranks 8 --peer > gpurun_out/shard8_peer_$k.log 2>&1 || exit 1
done
