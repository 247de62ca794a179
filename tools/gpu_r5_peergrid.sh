#!/bin/bash
# peer exchange, unsplit shards: fused grid launch against reduce_parts + peer_sum + k_grid (A/B)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_peer.py -x -v --timeout 120 --timeout-method thread > gpurun_out/peergrid_tests.log 2>&1 || exit 1
for r in 2 4; do
  timeout -k 10 120 python tools/shard_probe.py --ranks $r --reps 3000 >> gpurun_out/peergrid_ab.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/shard_probe.py --ranks $r --reps 3000 --peer >> gpurun_out/peergrid_ab.txt 2>&1 || exit 1

done
tail -3 gpurun_out/peergrid_tests.log
