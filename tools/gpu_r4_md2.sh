set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests/test_gpu_md.py tests/test_gpu_dist.py -m gpu -q -s --timeout 600 --timeout-method thread > gpurun_out/r4/pt_md.log 2>&1 || { echo PYTEST_FAIL; grep -E "^FAILED|tiled 3-D|Error" gpurun_out/r4/pt_md.log | head -30; exit 1; }
grep -E "tiled 3-D|passed|failed" gpurun_out/r4/pt_md.log | tail -3
timeout -k 10 300 python tools/md_probe.py > gpurun_out/r4/md_probe.txt 2>&1 || { echo MDPROBE_FAIL; tail -5 gpurun_out/r4/md_probe.txt; exit 1; }
tail -8 gpurun_out/r4/md_probe.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_krylov.py tests/test_gpu_slq_pairs.py tests/test_gpu_dist_krylov.py -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/r4/pt_b3.log 2>&1 || { echo PYTEST_FAIL2; grep -E "^FAILED|Error" gpurun_out/r4/pt_b3.log | head -30; exit 1; }
tail -1 gpurun_out/r4/pt_b3.log
S="0:1:0 1:1:0 2:1:0 1:2:0 2:2:0 1:4:0 2:11:0 1:1:2032 2:1:2032 0:1:2032"
timeout -k 10 300 python tools/spread2_ab.py --n 1000000 --d 32 --settings "$S" > gpurun_out/r4/s2_c.jsonl 2> gpurun_out/r4/s2_c.err || { echo AB_C_FAIL; tail -20 gpurun_out/r4/s2_c.err; exit 1; }
cat gpurun_out/r4/s2_c.jsonl
timeout -k 10 500 python tools/spread2_ab.py --n 10000000 --d 64 --nv 4 --reps 5 --settings "$S" > gpurun_out/r4/s2_e.jsonl 2> gpurun_out/r4/s2_e.err || { echo AB_E_FAIL; tail -20 gpurun_out/r4/s2_e.err; exit 1; }
cat gpurun_out/r4/s2_e.jsonl
bash tools/ab_env.sh "NFFT4GP_AMD_SPREAD_VARIANT=0 NFFT4GP_AMD_SPREAD_VARIANT=2,NFFT4GP_AMD_SPREAD2_GPW=1 NFFT4GP_AMD_SPREAD_VARIANT=2,NFFT4GP_AMD_SPREAD2_GPW=2 NFFT4GP_AMD_SPREAD_VARIANT=2,NFFT4GP_AMD_SPREAD2_GPW=4" --steps 300
