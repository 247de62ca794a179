# Round 5: the 32-bit precision mode -- its GPU tests, the layout tests, then config E at 64 and 32 bits.
set -o pipefail
mkdir -p gpurun_out/prec
timeout -k 10 600 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_layout.py -x -v --timeout 300 --timeout-method thread > gpurun_out/prec/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/prec/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/prec/pytest.log | tail -1; grep "32-bit" gpurun_out/prec/pytest.log
for p in 64 32; do
  timeout -k 10 600 python tools/config_e.py --reps 20 --precision $p > gpurun_out/prec/config_e_$p.json 2>/dev/null || { echo CONFIG_E_FAIL; exit 1; }
  tail -1 gpurun_out/prec/config_e_$p.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('E', $p, round(d['matvecs_per_s'],1), round(1e3/d['matvecs_per_s'],3), 'ms', {k:round(x*1e3,1) for k,x in d['kernels_ms'].items()}, 'loss', round(d['loss_s'],3), round(d['loss_dcgs2_s'],3), d['loss'], 'bytes ratio', round(d['bytes_ratio'],3))"
done
