# round-4 batch: distributed Krylov (DCGS2) and shard tests, the shard atomic-tail A/B, spread variants'
# parity and A/B at C and E
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_dist_krylov.py tests/test_gpu_dist.py tests/test_gpu_configs.py > gpurun_out/r4/pt_batch.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r4/pt_batch.log; exit 1; }
tail -2 gpurun_out/r4/pt_batch.log
NFFT4GP_AMD_SHARD_TAIL=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_configs.py > gpurun_out/r4/pt_tail.log 2>&1 || { echo PYTEST_TAIL_FAIL; tail -30 gpurun_out/r4/pt_tail.log; exit 1; }
tail -2 gpurun_out/r4/pt_tail.log
NFFT4GP_AMD_SPREAD_VARIANT=3 NFFT4GP_AMD_BLOCK=2032 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nfft.py tests/test_gpu_golden.py > gpurun_out/r4/pt_v3.log 2>&1 || { echo PYTEST_V3_FAIL; tail -30 gpurun_out/r4/pt_v3.log; exit 1; }
tail -2 gpurun_out/r4/pt_v3.log
for rep in 1 2; do
  for t in 0 1; do
    r=$(NFFT4GP_AMD_SHARD_TAIL=$t timeout -k 10 120 python tools/shard_probe.py --ranks 8 2>/dev/null) || { echo PROBE_FAIL; exit 1; }
    echo " rep=$rep $r"
  done
done
bash tools/ab_env.sh "NFFT4GP_AMD_SPREAD_VARIANT=0 NFFT4GP_AMD_SPREAD_VARIANT=2 NFFT4GP_AMD_BLOCK=2032 NFFT4GP_AMD_BLOCK=2032,NFFT4GP_AMD_SPREAD_VARIANT=3 NFFT4GP_AMD_SPREAD_VARIANT=3 NFFT4GP_AMD_CG=4,NFFT4GP_AMD_BLOCK=3840" --steps 300 || exit 1
bash tools/ab_env.sh "NFFT4GP_AMD_SPREAD_VARIANT=0 NFFT4GP_AMD_SPREAD_VARIANT=2 NFFT4GP_AMD_BLOCK=2032 NFFT4GP_AMD_BLOCK=2032,NFFT4GP_AMD_SPREAD_VARIANT=3" --n 10000000 --d 64 --steps 30 --warmup 5
