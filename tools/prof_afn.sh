# kernel trace of the config-C AFN setup (rank 512, Schur FSAI lfil 20)
set -o pipefail
mkdir -p gpurun_out/r4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4/prof_afn -o run -- python3 $GRAFT_REPO_ROOT/tools/afn_config_c_probe.py > $GRAFT_REPO_ROOT/gpurun_out/r4/prof_afn.log 2>&1 || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r4/prof_afn.log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/gpurun_out/r4/prof_afn -name '*kernel_stats.csv' | head -1); cp $f $GRAFT_REPO_ROOT/gpurun_out/r4/afn_kernel_stats.csv
rm -rf $GRAFT_REPO_ROOT/gpurun_out/r4/prof_afn
