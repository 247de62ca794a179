# round 4 A/B and probes (after the full suite passed once)
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_krylov.py -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/r4/pt_dk.log 2>&1 || { echo PYTEST_FAIL; grep -E "^FAILED|Error" gpurun_out/r4/pt_dk.log | head; exit 1; }
tail -1 gpurun_out/r4/pt_dk.log
S="0:1:0 1:1:0 2:1:0 1:2:0 2:2:0 1:4:0 1:1:2032 2:1:2032"
timeout -k 10 300 python tools/spread2_ab.py --n 1000000 --d 32 --settings "$S" > gpurun_out/r4/s2_c.jsonl 2> gpurun_out/r4/s2_c.err || { echo AB_C_FAIL; tail -20 gpurun_out/r4/s2_c.err; exit 1; }
cat gpurun_out/r4/s2_c.jsonl
timeout -k 10 500 python tools/spread2_ab.py --n 10000000 --d 64 --nv 4 --reps 5 --settings "$S" > gpurun_out/r4/s2_e.jsonl 2> gpurun_out/r4/s2_e.err || { echo AB_E_FAIL; tail -20 gpurun_out/r4/s2_e.err; exit 1; }
cat gpurun_out/r4/s2_e.jsonl
bash tools/ab_env.sh "NFFT4GP_AMD_SPREAD_VARIANT=0 NFFT4GP_AMD_SPREAD_VARIANT=2,NFFT4GP_AMD_SPREAD2_GPW=1 NFFT4GP_AMD_SPREAD_VARIANT=2,NFFT4GP_AMD_SPREAD2_GPW=2 NFFT4GP_AMD_SPREAD_VARIANT=2,NFFT4GP_AMD_SPREAD2_GPW=4" --steps 300 || exit 1
timeout -k 10 300 python tools/md_probe.py > gpurun_out/r4/md_probe.txt 2>&1 || { echo MDPROBE_FAIL; tail -5 gpurun_out/r4/md_probe.txt; exit 1; }
tail -8 gpurun_out/r4/md_probe.txt
timeout -k 10 600 python tools/config_e.py --reps 5 > gpurun_out/r4/config_e.json 2> gpurun_out/r4/config_e.err || { echo CONFIG_E_FAIL; tail -20 gpurun_out/r4/config_e.err; exit 1; }
cat gpurun_out/r4/config_e.json
timeout -k 10 600 python bench.py --steps 200 --warmup 20 --afn-rank 0 --no-traffic --no-cpu-baseline > gpurun_out/r4/b_nys.json 2> gpurun_out/r4/b_nys.err || { echo BENCH_FAIL; tail -20 gpurun_out/r4/b_nys.err; exit 1; }
python -c "
import json; r=json.load(open('gpurun_out/r4/b_nys.json')); print(r['value'], r['kernels_ms']); print({k:v for k,v in r.items() if k.startswith(('pcg','fgmres','loss','nys'))})"
