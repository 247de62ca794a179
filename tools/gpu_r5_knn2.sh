#!/bin/bash
# tiled KNN screen: parity tests + kernel time at n = 1e6, d = 32
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_knn.py -s > gpurun_out/knn_tests.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_knn4p -o run -- python3 tools/knn_probe.py --variants 4,1 > gpurun_out/knn_probe.log 2>&1
