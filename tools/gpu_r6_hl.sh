# round 6: k_interp_hl (the window group's H rows staged in LDS) -- bitwise check against k_interp in deterministic
# mode at C and E (both precisions), then the A/B timing
set -o pipefail
mkdir -p gpurun_out
for cfg in "--n 1000000 --d 32" "--n 10000000 --d 64 --precision 32" "--n 10000000 --d 64"; do
  NFFT4GP_AMD_INTERP_HL=0 timeout -k 10 120 python tools/interp_check.py $cfg --out gpurun_out/y_a.npy > /dev/null 2>gpurun_out/hl_a.err || { echo CHECK_A_FAIL; tail gpurun_out/hl_a.err; exit 1; }
  NFFT4GP_AMD_INTERP_HL=1 timeout -k 10 120 python tools/interp_check.py $cfg --out gpurun_out/y_b.npy > /dev/null 2>gpurun_out/hl_b.err || { echo CHECK_B_FAIL; tail gpurun_out/hl_b.err; exit 1; }
  python -c "import numpy as np;a=np.load('gpurun_out/y_a.npy');b=np.load('gpurun_out/y_b.npy');print('[$cfg] bitwise', np.array_equal(a,b), 'max rel', float(np.abs(a-b).max()/np.abs(a).max()))"
done
rm -f gpurun_out/y_a.npy gpurun_out/y_b.npy
bash tools/ab_e.sh "NFFT4GP_AMD_INTERP_HL=0 NFFT4GP_AMD_INTERP_HL=1"
