# Round 5: the GPU suite on the in-tree build (optional), then the spread's moment table, window groups and the
# deterministic mode on the in-tree build (tools/ab_env.sh, two alternating reps).
#   bash tools/gpu_r5_ab.sh [tests] ["SETTINGS"]
set -o pipefail
mkdir -p gpurun_out
if [ "$1" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/r5_pytest.log; exit 1; }
  tail -2 gpurun_out/r5_pytest.log
fi
SETS="${2:-NFFT4GP_AMD_DET=1 NFFT4GP_AMD_DET=0 NFFT4GP_AMD_SPREAD_VARIANT=2,NFFT4GP_AMD_DET=0 NFFT4GP_AMD_CG=4,NFFT4GP_AMD_DET=0 NFFT4GP_AMD_CG=4}"
bash tools/ab_env.sh "$SETS" --steps 500 2>&1 | tee gpurun_out/r5_ab_env.txt
