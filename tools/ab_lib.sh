# A/B of two builds of the library on one box: the in-tree build (A) against gpurun_ab/libnfft4gp_amd.so (B),
# alternating, on the bench's matvec kernels and the 8/4-way shard probe.
#   bash tools/ab_lib.sh
set -o pipefail
mkdir -p gpurun_out
LIB=preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd/libnfft4gp_amd.so
cp $LIB gpurun_out/lib_a.so || exit 1
for rep in 1 2; do
  for v in a b; do
    if [ $v = a ]; then cp gpurun_out/lib_a.so $LIB; else cp gpurun_ab/libnfft4gp_amd.so $LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic --no-pcg --no-config-e --steps 500 > gpurun_out/ab_$v.json 2>/dev/null || { echo BENCH_FAIL $v; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('lib $v rep $rep', round(d['ms_per_step']*1e3,2), {k:round(x*1e3,2) for k,x in d['kernels_ms'].items()})"
    for N in 8 4; do echo -n "lib $v N=$N "; timeout -k 10 300 python tools/shard_probe.py --ranks $N 2>/dev/null | tail -1 || exit 1; done
  done
done
cp gpurun_out/lib_a.so $LIB
rm -f gpurun_out/lib_a.so
