# full GPU suite (all failures listed), then the A/B and probes of round 4
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -s --timeout 600 --timeout-method thread > gpurun_out/r4/pt_full.log 2>&1
rc=$?
grep -E "tiled 3-D|reference FGMRES|^FAILED|^ERROR|passed|failed" gpurun_out/r4/pt_full.log | tail -25
[ $rc -eq 0 ] || { echo PYTEST_RC $rc; exit 1; }
S="0:1:0 1:1:0 2:1:0 1:2:0 2:2:0 1:4:0 1:1:2032 2:1:2032"
timeout -k 10 300 python tools/spread2_ab.py --n 1000000 --d 32 --settings "$S" > gpurun_out/r4/s2_c.jsonl 2> gpurun_out/r4/s2_c.err || { echo AB_C_FAIL; tail -20 gpurun_out/r4/s2_c.err; exit 1; }
cat gpurun_out/r4/s2_c.jsonl
timeout -k 10 500 python tools/spread2_ab.py --n 10000000 --d 64 --nv 4 --reps 5 --settings "$S" > gpurun_out/r4/s2_e.jsonl 2> gpurun_out/r4/s2_e.err || { echo AB_E_FAIL; tail -20 gpurun_out/r4/s2_e.err; exit 1; }
cat gpurun_out/r4/s2_e.jsonl
bash tools/ab_env.sh "NFFT4GP_AMD_SPREAD_VARIANT=0 NFFT4GP_AMD_SPREAD_VARIANT=2,NFFT4GP_AMD_SPREAD2_GPW=1 NFFT4GP_AMD_SPREAD_VARIANT=2,NFFT4GP_AMD_SPREAD2_GPW=2 NFFT4GP_AMD_SPREAD_VARIANT=2,NFFT4GP_AMD_SPREAD2_GPW=4" --steps 300 || exit 1
timeout -k 10 300 python tools/md_probe.py > gpurun_out/r4/md_probe.txt 2>&1 || { echo MDPROBE_FAIL; tail -5 gpurun_out/r4/md_probe.txt; exit 1; }
tail -8 gpurun_out/r4/md_probe.txt
