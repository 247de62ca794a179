# Round evidence at the current head: the driver's three commands (tools/driver_check.sh), then a rocprofv3
# kernel trace of the bench (tools/prof_summary.py over its timed loops) and the SQ / LDS counter passes
# (tools/pmc_sq.py).  Outputs under gpurun_out/; copy the ones to keep into profiles/rNN_*.
set -o pipefail
bash tools/driver_check.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-traffic > gpurun_out/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_bench.log; exit 1; }
python tools/prof_summary.py $(find gpurun_out/prof -name "*kernel_trace.csv" | head -1) --steps 200 --out gpurun_out/prof_summary.json
cp $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1) gpurun_out/prof_kernel_stats.csv
rm -rf gpurun_out/prof  # the full trace is > 64 MiB: gpurun would not copy gpurun_out/ back
timeout -k 10 600 python tools/pmc_sq.py --out gpurun_out/pmc_sq.csv > gpurun_out/pmc_sq.log 2>&1 || { echo PMC_SQ_FAIL; tail -20 gpurun_out/pmc_sq.log; exit 1; }
tail -2 gpurun_out/pmc_sq.log
rm -rf gpurun_out/pmc_sq  # per-pass counter dumps; the summary is pmc_sq.csv
# the N > 1 path rehearsed with 2 gloo ranks on the one GPU (host all-reduce through the callback communicator)
NFFT4GP_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || { echo GLOO2_FAIL; tail -30 gpurun_out/bench_gloo2.err; exit 1; }
cat gpurun_out/bench_gloo2.json
du -sh gpurun_out/* | sort -h | tail -5
