#!/bin/bash
# Lanczos: the Krylov / loss parity tests, then the config-C loss timing with the one-launch local pass (default)
# and with block_gs's three launches (NFFT4GP_AMD_LANCZOS_LOCAL=0)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_krylov.py tests/test_gpu_dist_krylov.py tests/test_gpu_multi.py tests/test_gpu_determinism.py -x -v --timeout 300 --timeout-method thread > gpurun_out/lanczos_tests.log 2>&1 || { tail -30 gpurun_out/lanczos_tests.log; exit 1; }
tail -3 gpurun_out/lanczos_tests.log
timeout -k 10 300 python tools/loss_probe.py --reps 3 > gpurun_out/lanczos_loss.txt 2>&1 || { tail -20 gpurun_out/lanczos_loss.txt; exit 1; }
NFFT4GP_AMD_LANCZOS_LOCAL=0 timeout -k 10 300 python tools/loss_probe.py --reps 3 > gpurun_out/lanczos_loss_off.txt 2>&1 || { tail -20 gpurun_out/lanczos_loss_off.txt; exit 1; }
grep '^{' gpurun_out/lanczos_loss.txt | cut -c1-150
grep '^{' gpurun_out/lanczos_loss_off.txt | cut -c1-150
