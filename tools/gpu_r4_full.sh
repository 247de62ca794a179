# full GPU suite (all failures listed), then round 4's probes: md matvec times, config E loss, the bench with
# the Nystrom leg (MFMA rates)
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -s --timeout 600 --timeout-method thread > gpurun_out/r4/pt_full.log 2>&1
rc=$?
grep -E "tiled 3-D|^FAILED|^ERROR|passed|failed" gpurun_out/r4/pt_full.log | tail -25
[ $rc -eq 0 ] || { echo PYTEST_RC $rc; exit 1; }
timeout -k 10 300 python tools/md_probe.py > gpurun_out/r4/md_probe.txt 2>&1 || { echo MDPROBE_FAIL; tail -5 gpurun_out/r4/md_probe.txt; exit 1; }
tail -8 gpurun_out/r4/md_probe.txt
timeout -k 10 600 python tools/config_e.py --reps 5 > gpurun_out/r4/config_e.json 2> gpurun_out/r4/config_e.err || { echo CONFIG_E_FAIL; tail -20 gpurun_out/r4/config_e.err; exit 1; }
cat gpurun_out/r4/config_e.json
timeout -k 10 600 python bench.py --steps 200 --warmup 20 --afn-rank 0 --no-traffic --no-cpu-baseline > gpurun_out/r4/b_nys.json 2> gpurun_out/r4/b_nys.err || { echo BENCH_FAIL; tail -20 gpurun_out/r4/b_nys.err; exit 1; }
python -c "
import json; r=json.load(open('gpurun_out/r4/b_nys.json')); print(r['value'], r['kernels_ms']); print({k:v for k,v in r.items() if k.startswith(('pcg','fgmres','loss','nys'))})"
