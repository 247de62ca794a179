#!/bin/bash
# k_block_reduce folded into k_block_dots: Krylov tests, then loss and FGMRES CGS2 timing with and without
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_krylov.py tests/test_gpu_dist_krylov.py tests/test_gpu_multi.py tests/test_gpu_determinism.py -x -v --timeout 300 --timeout-method thread > gpurun_out/bdfold_tests.log 2>&1 || { tail -30 gpurun_out/bdfold_tests.log; exit 1; }
tail -3 gpurun_out/bdfold_tests.log
timeout -k 10 300 python tools/loss_probe.py --reps 3 > gpurun_out/bdfold_loss_on.txt 2>&1 || { tail -20 gpurun_out/bdfold_loss_on.txt; exit 1; }
NFFT4GP_AMD_BD_FOLD=0 timeout -k 10 300 python tools/loss_probe.py --reps 3 > gpurun_out/bdfold_loss_off.txt 2>&1 || { tail -20 gpurun_out/bdfold_loss_off.txt; exit 1; }
grep '^{' gpurun_out/bdfold_loss_on.txt | cut -c1-110
grep '^{' gpurun_out/bdfold_loss_off.txt | cut -c1-110
