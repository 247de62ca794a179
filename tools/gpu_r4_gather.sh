# spread variant 2 (alpha gathered from global memory): parity, row-shard per-rank time, config C A/B
set -o pipefail
mkdir -p gpurun_out/r4
NFFT4GP_AMD_SPREAD_VARIANT=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nfft.py tests/test_gpu_golden.py tests/test_gpu_dist.py > gpurun_out/r4/pt_gather.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r4/pt_gather.log; exit 1; }
tail -2 gpurun_out/r4/pt_gather.log
for rep in 1 2; do
  for v in 0 2; do
    for r in 8 4; do
      o=$(NFFT4GP_AMD_SPREAD_VARIANT=$v timeout -k 10 120 python tools/shard_probe.py --ranks $r 2>/dev/null) || { echo PROBE_FAIL; exit 1; }
      echo "variant=$v ranks=$r rep=$rep $o"
    done
  done
done
bash tools/ab_env.sh "NFFT4GP_AMD_SPREAD_VARIANT=0 NFFT4GP_AMD_SPREAD_VARIANT=2" --steps 300
