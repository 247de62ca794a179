set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_afn_flow.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_afn_flow.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_afn_flow.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed|rank|Nystrom" gpurun_out/pytest_afn_flow.log | tail -20
timeout -k 10 300 python bench.py --n 100000 --d 8 --nys-rank 256 --afn-rank 256 --no-cpu-baseline --no-traffic --steps 100 > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || { echo BENCHB_FAIL; tail -30 gpurun_out/bench_b.err; exit 1; }
cat gpurun_out/bench_b.json
timeout -k 10 400 python bench.py --no-cpu-baseline --no-traffic > gpurun_out/bench_c.json 2> gpurun_out/bench_c.err || { echo BENCHC_FAIL; tail -30 gpurun_out/bench_c.err; exit 1; }
cat gpurun_out/bench_c.json
