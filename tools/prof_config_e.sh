# config E (n = 1e7, 64 windows) loss + gradient under a rocprofv3 kernel trace
set -o pipefail
mkdir -p gpurun_out/prof_e
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_e -o e -- python3 tools/config_e.py --reps 5 "$@" > gpurun_out/config_e.json 2> gpurun_out/config_e.err || { echo CONFIG_E_FAIL; tail -30 gpurun_out/config_e.err; exit 1; }
tail -1 gpurun_out/config_e.json
f=$(find gpurun_out/prof_e -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/config_e_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/config_e_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.2f} us  {r["Name"][:90]}')
PY
