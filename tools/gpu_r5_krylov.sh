#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_krylov.py -x -v --timeout 300 --timeout-method thread > gpurun_out/krylov_tests.log 2>&1 || { tail -40 gpurun_out/krylov_tests.log; exit 1; }
tail -3 gpurun_out/krylov_tests.log
