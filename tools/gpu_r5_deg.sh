# Round 5: degree-7 taps (in-tree) against the degree-9 build in gpurun_ab/: the GPU suite, then tools/ab_lib.sh,
# then config E on both builds.
set -o pipefail
mkdir -p gpurun_out/deg
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/deg/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/deg/pytest.log; exit 1; }
tail -1 gpurun_out/deg/pytest.log
bash tools/ab_lib.sh 2>&1 | tee gpurun_out/deg/ab.txt || exit 1
LIB=preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd/libnfft4gp_amd.so
cp $LIB gpurun_out/deg/lib_a.so
timeout -k 10 600 python tools/config_e.py --reps 20 > gpurun_out/deg/config_e_a.json 2>/dev/null || { echo CONFIG_E_FAIL; exit 1; }
cp gpurun_ab/libnfft4gp_amd.so $LIB
timeout -k 10 600 python tools/config_e.py --reps 20 > gpurun_out/deg/config_e_b.json 2>/dev/null || { cp gpurun_out/deg/lib_a.so $LIB; echo CONFIG_E_FAIL; exit 1; }
cp gpurun_out/deg/lib_a.so $LIB
rm -f gpurun_out/deg/lib_a.so
for v in a b; do python -c "import json;d=json.load(open('gpurun_out/deg/config_e_$v.json'));print('E $v', round(d['matvecs_per_s'],1), {k:round(x*1e3,1) for k,x in d['kernels_ms'].items()}, 'loss', round(d['loss_s'],3), round(d['loss_dcgs2_s'],3), d['loss'])"; done
