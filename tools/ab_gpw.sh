set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for g in 1 2 3 11; do
    NFFT4GP_AMD_GPW=$g timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic --no-pcg > gpurun_out/abw.json 2>/dev/null || { echo FAIL $g; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abw.json'));print('gpw $g rep $rep', round(d['ms_per_step']*1e3,1), {k:round(x*1e3,2) for k,x in d['kernels_ms'].items()})"
  done
done
