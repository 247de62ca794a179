# A/B of environment settings on the bench workload (the library reads its knobs at handle creation), the
# settings alternated on one box, two reps:
#   bash tools/ab_env.sh "NFFT4GP_AMD_SPREAD_VARIANT=0 NFFT4GP_AMD_BLOCK=2032,NFFT4GP_AMD_CG=2" [bench args]
# one setting per word, several variables of one setting joined by commas.  AB_CONFIGS runs every setting on
# several workloads, bench argument sets separated by ';', e.g. config E in both record precisions and config C:
#   AB_CONFIGS="--n 10000000 --d 64 --steps 100 --precision 32;--n 10000000 --d 64 --steps 100;--steps 500"
set -o pipefail
mkdir -p gpurun_out
SETS="$1"; shift
IFS=';' read -r -a CFGS <<< "${AB_CONFIGS:-}"
if [ ${#CFGS[@]} -eq 0 ]; then CFGS=(""); fi
for rep in 1 2; do
  for cfg in "${CFGS[@]}"; do
    i=0
    for kv in $SETS; do
      i=$((i+1))
      env $(echo "$kv" | tr ',' ' ') timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic --no-pcg --no-config-e $cfg "$@" > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || { echo BENCH_FAIL $kv $cfg; tail -20 gpurun_out/ab_$i.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/ab_$i.json'));print('$kv [$cfg] rep $rep', round(d['ms_per_step']*1e3,1), {k:round(x*1e3,2) for k,x in d['kernels_ms'].items()})"
    done
  done
done
