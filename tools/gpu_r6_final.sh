# round-6 evidence: the driver's three commands (tools/driver_check.sh), then a rocprofv3 kernel trace of the
# headline bench (config C only: --no-config-e, so the trace's last loops are the headline's) with
# tools/prof_summary.py over its timed loops, and the SQ / LDS counter passes (tools/pmc_sq.py)
set -o pipefail
bash tools/driver_check.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof gpurun_out/oracle_native
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-traffic --no-pcg --no-config-e > gpurun_out/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_bench.log; exit 1; }
python tools/prof_summary.py $(find gpurun_out/prof -name "*kernel_trace.csv" | head -1) --steps 200 --out gpurun_out/prof_summary.json
cp $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1) gpurun_out/prof_kernel_stats.csv
rm -rf gpurun_out/prof
head -c 1200 gpurun_out/prof_summary.json; echo
timeout -k 10 600 python tools/pmc_sq.py --out gpurun_out/pmc_sq.csv > gpurun_out/pmc_sq.log 2>&1 || { echo PMC_SQ_FAIL; tail -20 gpurun_out/pmc_sq.log; exit 1; }
tail -2 gpurun_out/pmc_sq.log
