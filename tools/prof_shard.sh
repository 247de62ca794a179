set -o pipefail
mkdir -p gpurun_out/prof_sh
export TMPDIR=/tmp
NFFT4GP_AMD_FUSED_FINISH=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sh -o sh -- python3 tools/shard_probe.py --ranks 8 --reps 500 > gpurun_out/sh.log 2>&1 || { echo FAIL; tail -20 gpurun_out/sh.log; exit 1; }
f=$(find gpurun_out/prof_sh -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:8]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.2f} us  {r["Name"][:70]}')
PY
