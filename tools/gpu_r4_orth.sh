# FGMRES block CGS2 (ortho 1) and delayed CGS2 (ortho 2): probe, Krylov tests, kernel trace
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_krylov.py tests/test_gpu_dist_krylov.py > gpurun_out/r4/pt_krylov.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r4/pt_krylov.log; exit 1; }
tail -2 gpurun_out/r4/pt_krylov.log
timeout -k 10 200 python tools/fgmres_cgs2_probe.py 2 2>/dev/null || { echo PROBE_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r4/prof_orth3 -o run -- python3 $GRAFT_REPO_ROOT/tools/fgmres_cgs2_probe.py 1 > $GRAFT_REPO_ROOT/gpurun_out/r4/prof_orth3.log 2>&1 || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r4/prof_orth3.log; exit 1; }
