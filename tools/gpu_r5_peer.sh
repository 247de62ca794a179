#!/bin/bash
# peer exchange tests (two processes on one GPU) + the distributed suite, then the tiled KNN timings
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_peer.py > gpurun_out/peer_tests.log 2>&1 &&
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_knn.py tests/test_gpu_md.py > gpurun_out/dist_tests.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_knn4a -o run -- python3 tools/knn_probe.py --variants 4 > gpurun_out/knn_probe_a.log 2>&1 &&
NFFT4GP_AMD_KNN_TILE_PROBE=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_knn4b -o run -- python3 tools/knn_probe.py --variants 4 > gpurun_out/knn_probe_b.log 2>&1 &&
timeout -k 10 120 python -u tools/shard_probe.py --ranks 8 > gpurun_out/shard8_rows.log 2>&1 &&
timeout -k 10 120 python -u tools/shard_probe.py --ranks 8 --peer > gpurun_out/shard8_peer.log 2>&1
