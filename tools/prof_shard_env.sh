# Per-kernel times of a row shard (tools/shard_probe.py) under each of the given environment settings:
#   RANKS=8 bash tools/prof_shard_env.sh "NFFT4GP_AMD_SHARD_SPLIT=1 NFFT4GP_AMD_SHARD_SPLIT=4"
set -o pipefail
export TMPDIR=/tmp
for kv in $1; do
  rm -rf gpurun_out/prof_she
  env $kv timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_she -o sh -- python3 tools/shard_probe.py --ranks ${RANKS:-8} --reps 500 > gpurun_out/she.log 2>&1 || { echo FAIL; tail -20 gpurun_out/she.log; exit 1; }
  f=$(find gpurun_out/prof_she -name "*kernel_stats.csv" | head -1)
  echo "$kv $(grep us_per gpurun_out/she.log)"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:5]:
    print(f'   {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.2f} us  {r["Name"][:60]}')
PY
done
