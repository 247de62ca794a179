# Round evidence: full GPU test suite, the driver's bench command (with PMC traffic and the CPU baseline),
# a rocprofv3 kernel trace of the bench (CSV + tools/prof_summary.py over its timed loops), the SQ / LDS /
# MFMA counter passes (tools/pmc_sq.py) and the setup benchmark.  Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-traffic > gpurun_out/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_bench.log; exit 1; }
python tools/prof_summary.py $(find gpurun_out/prof -name "*kernel_trace.csv" | head -1) --steps 200 --out gpurun_out/prof_summary.json
timeout -k 10 600 python tools/pmc_sq.py --out gpurun_out/pmc_sq.csv > gpurun_out/pmc_sq.log 2>&1 || { echo PMC_SQ_FAIL; tail -20 gpurun_out/pmc_sq.log; exit 1; }
tail -2 gpurun_out/pmc_sq.log
timeout -k 10 400 python -u tools/setup_bench.py --out gpurun_out/setup_bench.json > gpurun_out/setup_bench.log 2>&1 || { echo SETUP_BENCH_FAIL; tail -20 gpurun_out/setup_bench.log; exit 1; }
grep -v "^Using\|KNN time\|amdgpu.ids" gpurun_out/setup_bench.log | tail -12
