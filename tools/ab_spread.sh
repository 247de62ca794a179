# A/B of spread kernel variants / block sizes on the bench workload:
#   bash tools/ab_spread.sh "0:4064 0:2032" [extra bench args]   (variant:block)
set -o pipefail
mkdir -p gpurun_out
VARS="$1"; shift
for rep in 1 2; do
  for vb in $VARS; do
    v=${vb%%:*}; b=${vb##*:}
    NFFT4GP_AMD_SPREAD_VARIANT=$v NFFT4GP_AMD_BLOCK=$b timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic --no-pcg "$@" > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo BENCH_FAIL $vb; tail -20 gpurun_out/ab_$v.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('variant $vb rep $rep', round(d['ms_per_step']*1e3,1), {k:round(x*1e3,2) for k,x in d['kernels_ms'].items()})"
  done
done
