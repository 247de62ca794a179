# A/B on BASELINE configs[4]'s operator only (n = 1e7, 64 windows), 32-bit and fp64 records, two reps
set -o pipefail
mkdir -p gpurun_out
SETS="$1"; shift
for rep in 1 2; do
  for cfg in "--n 10000000 --d 64 --steps 100 --precision 32" "--n 10000000 --d 64 --steps 100"; do
    i=0
    for kv in $SETS; do
      i=$((i+1))
      env $(echo "$kv" | tr ',' ' ') timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic --no-pcg --no-config-e $cfg "$@" > gpurun_out/abe_$i.json 2> gpurun_out/abe_$i.err || { echo BENCH_FAIL $kv $cfg; tail -20 gpurun_out/abe_$i.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/abe_$i.json'));print('$kv [$cfg] rep $rep', round(d['ms_per_step']*1e3,1), {k:round(x*1e3,2) for k,x in d['kernels_ms'].items()})"
    done
  done
done
