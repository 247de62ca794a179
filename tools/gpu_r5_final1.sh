# round-5 final evidence, part 1: the driver's three commands, then a rocprofv3 kernel trace of the bench
set -o pipefail
bash tools/driver_check.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-traffic --no-pcg > gpurun_out/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_bench.log; exit 1; }
python tools/prof_summary.py $(find gpurun_out/prof -name "*kernel_trace.csv" | head -1) --steps 200 --out gpurun_out/prof_summary.json
cp $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1) gpurun_out/prof_kernel_stats.csv
rm -rf gpurun_out/prof
cat gpurun_out/prof_summary.json | head -c 1500
