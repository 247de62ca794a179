#!/bin/bash
# fused PCG direction update: determinism + solver tests, then the A/B timing and a kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_solvers.py -x -v --timeout 200 --timeout-method thread > gpurun_out/fusep_tests.log 2>&1 || { tail -30 gpurun_out/fusep_tests.log; exit 1; }
tail -4 gpurun_out/fusep_tests.log
timeout -k 10 300 python tools/pcg_fusep_ab.py --reps 3 > gpurun_out/fusep_ab.txt 2>&1 || { tail -20 gpurun_out/fusep_ab.txt; exit 1; }
grep '^{' gpurun_out/fusep_ab.txt
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_fusep -o run -- python3 $GRAFT_REPO_ROOT/tools/pcg_fusep_ab.py --reps 1 > $GRAFT_REPO_ROOT/gpurun_out/fusep_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/fusep_prof.log; exit 1; }
cp $(find $GRAFT_REPO_ROOT/gpurun_out/prof_fusep -name "*kernel_stats.csv" | head -1) $GRAFT_REPO_ROOT/gpurun_out/fusep_kernel_stats.csv && head -8 $GRAFT_REPO_ROOT/gpurun_out/fusep_kernel_stats.csv
