# round 6: the wide MGS sweep (k_mgs_wide) -- bitwise tests, then config E's loss with it and without it
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_tests.sh tests/test_gpu_determinism.py tests/test_gpu_krylov.py || exit 1
for w in 1 0; do
  NFFT4GP_AMD_MGS_WIDE=$w timeout -k 10 300 python tools/config_e.py > gpurun_out/cfge_wide$w.json 2> gpurun_out/cfge_wide$w.err || { echo CFGE_FAIL $w; tail -20 gpurun_out/cfge_wide$w.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/cfge_wide$w.json').read().strip().splitlines()[-1]);print('MGS_WIDE=$w', 'loss_s', round(d['loss_s'],3), 'dcgs2', round(d['loss_dcgs2_s'],3), 'loss', d['loss'], 'mv/s', round(d['matvecs_per_s'],1), d['kernels_ms'])"
done
