# kernel times of the two-vector matvec against the single-vector kernels (rocprofv3 kernel trace)
set -o pipefail
mkdir -p gpurun_out/prof_m
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_m -o m -- python3 tools/multi_probe.py "$@" > gpurun_out/multi.json 2> gpurun_out/multi.err || { echo FAIL; tail -30 gpurun_out/multi.err; exit 1; }
tail -1 gpurun_out/multi.json
f=$(find gpurun_out/prof_m -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.2f} us  {r["Name"][:80]}')
PY
