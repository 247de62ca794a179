# kernel trace of the N = 8 row-shard probe (per-rank kernels without the all-reduce)
set -o pipefail
mkdir -p gpurun_out/r4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4/prof_shard -o run -- python3 $GRAFT_REPO_ROOT/tools/shard_probe.py --ranks 8 > $GRAFT_REPO_ROOT/gpurun_out/r4/prof_shard.log 2>&1 || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r4/prof_shard.log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/gpurun_out/r4/prof_shard -name '*kernel_stats.csv' | head -1); cp $f $GRAFT_REPO_ROOT/gpurun_out/r4/shard_kernel_stats.csv
rm -rf $GRAFT_REPO_ROOT/gpurun_out/r4/prof_shard
