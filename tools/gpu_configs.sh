set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_configs.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_configs.log; exit 1; }
grep -E "rel err|config|PASS|FAIL|passed|failed" gpurun_out/pytest_configs.log | tail -60
timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic --no-pcg > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_quick.err; exit 1; }
cat gpurun_out/bench_quick.json
