set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_krylov.py tests/test_gpu_slq_pairs.py tests/test_gpu_md.py tests/test_gpu_dist.py tests/test_gpu_dist_krylov.py -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/r4/pt_b2.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r4/pt_b2.log; exit 1; }
tail -2 gpurun_out/r4/pt_b2.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 600 --timeout-method thread -k "config_e" > gpurun_out/r4/pt_e.log 2>&1 || { echo PYTEST_E_FAIL; tail -40 gpurun_out/r4/pt_e.log; exit 1; }
tail -2 gpurun_out/r4/pt_e.log
S="0:1:0 1:1:0 2:1:0 1:2:0 2:2:0 1:4:0 2:11:0 1:1:2032 2:1:2032 0:1:2032"
timeout -k 10 300 python tools/spread2_ab.py --n 1000000 --d 32 --settings "$S" > gpurun_out/r4/s2_c.jsonl 2> gpurun_out/r4/s2_c.err || { echo AB_C_FAIL; tail -20 gpurun_out/r4/s2_c.err; exit 1; }
cat gpurun_out/r4/s2_c.jsonl
timeout -k 10 500 python tools/spread2_ab.py --n 10000000 --d 64 --nv 4 --reps 5 --settings "$S" > gpurun_out/r4/s2_e.jsonl 2> gpurun_out/r4/s2_e.err || { echo AB_E_FAIL; tail -20 gpurun_out/r4/s2_e.err; exit 1; }
cat gpurun_out/r4/s2_e.jsonl
