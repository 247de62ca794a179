#!/bin/bash
# KNN screens: parity tests, n = 1e6 d = 32 timings, config-C AFN setup with the tiled screen (profiled)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_knn.py -s > gpurun_out/knn_tests.log 2>&1 &&
timeout -k 10 120 python -u tools/knn_probe.py --variants 4,3,1 > gpurun_out/knn_probe.log 2>&1 &&
NFFT4GP_AMD_KNN=4 timeout -k 10 120 python -u tools/afn_config_c_probe.py > gpurun_out/afn_c_v4.log 2>&1 &&
NFFT4GP_AMD_KNN=4 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_knn4 -o run -- python3 tools/afn_config_c_probe.py > gpurun_out/afn_c_v4_prof.log 2>&1
