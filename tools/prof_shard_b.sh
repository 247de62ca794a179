# Per-kernel times of the 8-way row shard of config C at several block sizes (rocprofv3 kernel trace).
set -o pipefail
export TMPDIR=/tmp
for b in ${BLOCKS:-2032 1016 508}; do
  rm -rf gpurun_out/prof_shb
  NFFT4GP_AMD_BLOCK=$b timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_shb -o sh -- python3 tools/shard_probe.py --ranks ${RANKS:-8} --reps 500 > gpurun_out/shb.log 2>&1 || { echo FAIL; tail -20 gpurun_out/shb.log; exit 1; }
  f=$(find gpurun_out/prof_shb -name "*kernel_stats.csv" | head -1)
  echo "B=$b $(grep us_per gpurun_out/shb.log)"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:4]:
    print(f'   {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.2f} us  {r["Name"][:60]}')
PY
done
