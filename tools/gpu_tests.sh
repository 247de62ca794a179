# GPU tests in one pytest process, stopping at the first failure: the whole suite, or the given
# test files / pytest arguments
set -o pipefail
mkdir -p gpurun_out
if [ $# -eq 0 ]; then set -- tests; fi
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -5; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
