set -o pipefail
mkdir -p gpurun_out/r4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4/prof_md -o run -- python3 $GRAFT_REPO_ROOT/tools/md_probe.py > $GRAFT_REPO_ROOT/gpurun_out/r4/prof_md.log 2>&1 || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r4/prof_md.log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/gpurun_out/r4/prof_md -name '*kernel_stats.csv' | head -1); cp $f $GRAFT_REPO_ROOT/gpurun_out/r4/md_kernel_stats.csv
rm -rf $GRAFT_REPO_ROOT/gpurun_out/r4/prof_md
head -14 $GRAFT_REPO_ROOT/gpurun_out/r4/md_kernel_stats.csv | cut -c1-160
