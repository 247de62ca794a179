#!/bin/bash
# peer exchange (epoch-stamped words): tests + N = 8 probes; tiled KNN: staged vs direct loads (parity + time)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_peer.py > gpurun_out/peer_tests.log 2>&1 &&
timeout -k 10 120 python -u tools/shard_probe.py --ranks 8 > gpurun_out/shard8_rows.log 2>&1 &&
timeout -k 10 120 python -u tools/shard_probe.py --ranks 8 --peer > gpurun_out/shard8_peer.log 2>&1 &&
timeout -k 10 120 python -u tools/shard_probe.py --ranks 8 > gpurun_out/shard8_rows_b.log 2>&1 &&
timeout -k 10 120 python -u tools/shard_probe.py --ranks 8 --peer > gpurun_out/shard8_peer_b.log 2>&1 &&
NFFT4GP_AMD_KNN_TILE_DIRECT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_knn.py > gpurun_out/knn_direct_tests.log 2>&1 &&
for m in 0 1 0 1; do
  NFFT4GP_AMD_KNN_TILE_DIRECT=$m timeout -k 10 120 python -u tools/knn_probe.py --variants 4,4 > gpurun_out/knn_d$m.log 2>&1 || exit 1
  tail -1 gpurun_out/knn_d$m.log | sed "s/^/direct=$m /" >> gpurun_out/knn_ab.txt
  NFFT4GP_AMD_KNN_TILE_PROBE=1 NFFT4GP_AMD_KNN_TILE_DIRECT=$m timeout -k 10 120 python -u tools/knn_probe.py --variants 4,4 > gpurun_out/knn_d$m.log 2>&1 || exit 1
  tail -1 gpurun_out/knn_d$m.log | sed "s/^/scan-only direct=$m /" >> gpurun_out/knn_ab.txt
done
