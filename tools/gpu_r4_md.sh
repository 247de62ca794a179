set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests/test_gpu_md.py tests/test_gpu_dist.py -m gpu -q -s --timeout 600 --timeout-method thread > gpurun_out/r4/pt_md.log 2>&1 || { echo PYTEST_FAIL; grep -E "^FAILED|tiled 3-D|Error" gpurun_out/r4/pt_md.log | head -30; exit 1; }
grep -E "tiled 3-D|passed|failed" gpurun_out/r4/pt_md.log | tail -3
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_krylov.py tests/test_gpu_slq_pairs.py tests/test_gpu_dist_krylov.py -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/r4/pt_b3.log 2>&1 || { echo PYTEST_FAIL2; grep -E "^FAILED|Error" gpurun_out/r4/pt_b3.log | head -30; exit 1; }
tail -1 gpurun_out/r4/pt_b3.log
