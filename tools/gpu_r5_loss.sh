#!/bin/bash
# config-C loss: wall vs kernel time
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_loss
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_loss -o run -- python3 $GRAFT_REPO_ROOT/tools/loss_probe.py --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/loss_probe.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/loss_probe.log; exit 1; }
cp $(find $GRAFT_REPO_ROOT/gpurun_out/prof_loss -name "*kernel_stats.csv" | head -1) $GRAFT_REPO_ROOT/gpurun_out/loss_kernel_stats.csv
cp $(find $GRAFT_REPO_ROOT/gpurun_out/prof_loss -name "*kernel_trace.csv" | head -1) $GRAFT_REPO_ROOT/gpurun_out/loss_kernel_trace.csv
rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_loss
grep '^{' $GRAFT_REPO_ROOT/gpurun_out/loss_probe.log | cut -c1-200
