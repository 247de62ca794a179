#!/bin/bash
# Lanczos step with one host read: the Krylov / loss parity tests, then the config-C loss timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_krylov.py tests/test_gpu_dist_krylov.py tests/test_gpu_multi.py -x -v --timeout 300 --timeout-method thread > gpurun_out/lanczos_tests.log 2>&1 || { tail -30 gpurun_out/lanczos_tests.log; exit 1; }
tail -3 gpurun_out/lanczos_tests.log
timeout -k 10 300 python tools/loss_probe.py --reps 3 > gpurun_out/lanczos_loss.txt 2>&1 || { tail -20 gpurun_out/lanczos_loss.txt; exit 1; }
grep '^{' gpurun_out/lanczos_loss.txt | cut -c1-120
