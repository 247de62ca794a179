# round 6: k_interp_hl with more staging slots on 1024-thread workgroups -- bitwise check, then A/B at config E
set -o pipefail
mkdir -p gpurun_out
for cfg in "--n 10000000 --d 64 --precision 32" "--n 10000000 --d 64"; do
  NFFT4GP_AMD_INTERP_HL=0 timeout -k 10 120 python tools/interp_check.py $cfg --out gpurun_out/y_a.npy > /dev/null 2>gpurun_out/hl_a.err || { echo CHECK_A_FAIL; tail gpurun_out/hl_a.err; exit 1; }
  NFFT4GP_AMD_INTERP_THREADS=1024 NFFT4GP_AMD_HL_SLOTS=6 timeout -k 10 120 python tools/interp_check.py $cfg --out gpurun_out/y_b.npy > /dev/null 2>gpurun_out/hl_b.err || { echo CHECK_B_FAIL; tail gpurun_out/hl_b.err; exit 1; }
  python -c "import numpy as np;a=np.load('gpurun_out/y_a.npy');b=np.load('gpurun_out/y_b.npy');print('[$cfg] bitwise', np.array_equal(a,b))"
done
rm -f gpurun_out/y_a.npy gpurun_out/y_b.npy
bash tools/ab_e2.sh "NFFT4GP_AMD_HL_SLOTS=2 NFFT4GP_AMD_INTERP_THREADS=1024,NFFT4GP_AMD_HL_SLOTS=2 NFFT4GP_AMD_INTERP_THREADS=1024,NFFT4GP_AMD_HL_SLOTS=4 NFFT4GP_AMD_INTERP_THREADS=1024,NFFT4GP_AMD_HL_SLOTS=6"
