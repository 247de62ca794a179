# md spread: line-owned variant (NFFT4GP_AMD_MD_SPREAD=2) -- md tests on it, then tools/md_probe.py A/B and
# work-item sizes
set -o pipefail
mkdir -p gpurun_out/r4
NFFT4GP_AMD_MD_SPREAD=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_md.py tests/test_gpu_golden.py > gpurun_out/r4/pt_mdlines.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r4/pt_mdlines.log; exit 1; }
tail -2 gpurun_out/r4/pt_mdlines.log
for v in 1 2; do
  echo "md_spread=$v"
  NFFT4GP_AMD_MD_SPREAD=$v timeout -k 10 300 python tools/md_probe.py 2>/dev/null || { echo MD_PROBE_FAIL; exit 1; }
done
for c in 200000 1000000; do
  echo "md_spread=2 chunk_taps=$c"
  NFFT4GP_AMD_MD_SPREAD=2 NFFT4GP_AMD_MD_CHUNK=$c timeout -k 10 300 python tools/md_probe.py 2>/dev/null || { echo MD_PROBE_FAIL; exit 1; }
done
