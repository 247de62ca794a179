#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_krylov.py tests/test_gpu_dist_krylov.py tests/test_gpu_peer.py -x -v --timeout 300 --timeout-method thread > gpurun_out/bdfold2_tests.log 2>&1 || { tail -30 gpurun_out/bdfold2_tests.log; exit 1; }
tail -3 gpurun_out/bdfold2_tests.log
timeout -k 10 400 python tools/fgmres_ortho_ab.py --reps 2 > gpurun_out/bdfold2_ab.txt 2>&1 || { tail -20 gpurun_out/bdfold2_ab.txt; exit 1; }
grep '^{' gpurun_out/bdfold2_ab.txt
