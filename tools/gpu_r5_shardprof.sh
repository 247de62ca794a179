#!/bin/bash
# kernel durations of the N = 8 row shard over the peer exchange (fake world) and without any exchange
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for mode in peer plain; do
  flag=""; [ $mode = peer ] && flag="--peer"
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_shard_$mode
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_shard_$mode -o run -- python3 $GRAFT_REPO_ROOT/tools/shard_probe.py --ranks 8 --reps 3000 $flag > $GRAFT_REPO_ROOT/gpurun_out/shardprof_$mode.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/shardprof_$mode.log; exit 1; }
  cp $(find $GRAFT_REPO_ROOT/gpurun_out/prof_shard_$mode -name "*kernel_stats.csv" | head -1) $GRAFT_REPO_ROOT/gpurun_out/shard8_${mode}_kernel_stats.csv
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_shard_$mode
  head -6 $GRAFT_REPO_ROOT/gpurun_out/shard8_${mode}_kernel_stats.csv | cut -c1-200
done
