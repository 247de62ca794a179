#!/bin/bash
# k_interp with the next tile's loads issued before the current tile's work (A) against HEAD (B); parity tests on A
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_nfft.py tests/test_gpu_configs.py tests/test_gpu_golden.py tests/test_gpu_determinism.py tests/test_gpu_precision.py > gpurun_out/interp_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/interp_tests.log; exit 1; }
tail -1 gpurun_out/interp_tests.log
bash tools/ab_lib.sh > gpurun_out/interp_ab.txt 2>&1
cat gpurun_out/interp_ab.txt
