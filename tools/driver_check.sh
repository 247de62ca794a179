# The driver's round-end commands, in its order: the GPU suite, smoke(), and the default-size bench line.
# Logs under gpurun_out/driver_*; copy them into profiles/rNN_* at the final commit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/driver_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/driver_pytest.log; exit 1; }
tail -3 gpurun_out/driver_pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/driver_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/driver_smoke.log; exit 1; }
tail -2 gpurun_out/driver_smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driver_bench.json 2> gpurun_out/driver_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/driver_bench.err; exit 1; }
cat gpurun_out/driver_bench.json
