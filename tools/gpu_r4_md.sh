# multi-feature windows: parity / reproducibility tests and matvec times
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_gpu_md.py tests/test_gpu_dist.py tests/test_gpu_golden.py -m gpu -q -s --timeout 600 --timeout-method thread > gpurun_out/r4/pt_md.log 2>&1 || { echo PYTEST_FAIL; grep -E "^FAILED|tiled 3-D|Error" gpurun_out/r4/pt_md.log | head -30; exit 1; }
grep -E "tiled 3-D|passed|failed" gpurun_out/r4/pt_md.log | tail -3
timeout -k 10 300 python tools/md_probe.py > gpurun_out/r4/md_probe.txt 2>&1 || { echo MDPROBE_FAIL; tail -5 gpurun_out/r4/md_probe.txt; exit 1; }
tail -6 gpurun_out/r4/md_probe.txt
