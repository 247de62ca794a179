# FGMRES block-CGS2 kernels: old (BGS_VARIANT 0) vs 16-byte dots / 4-column update (1), then a kernel trace of 1
set -o pipefail
mkdir -p gpurun_out/r4
for v in 0 1 0 1; do
  echo "variant $v"
  NFFT4GP_AMD_BGS_VARIANT=$v timeout -k 10 200 python tools/fgmres_cgs2_probe.py 2 2>/dev/null || { echo PROBE_FAIL; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4/prof_orth -o run -- python3 $GRAFT_REPO_ROOT/tools/fgmres_cgs2_probe.py 1 > $GRAFT_REPO_ROOT/gpurun_out/r4/prof_orth.log 2>&1 || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r4/prof_orth.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/r4/prof_orth -name '*kernel_stats.csv' | head -1 | xargs head -12
