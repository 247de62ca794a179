# usage: bash tools/gpu_quick.sh "<pytest -k expr or empty>" [bench args...]
set -o pipefail
mkdir -p gpurun_out
K="$1"; shift
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_quick.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_quick.log; exit 1; }
  tail -3 gpurun_out/pytest_quick.log
fi
if [ "$1" != "nobench" ]; then
  timeout -k 10 400 python bench.py --no-cpu-baseline --no-traffic "$@" > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_quick.err; exit 1; }
  cat gpurun_out/bench_quick.json; tail -12 gpurun_out/bench_quick.err
fi
