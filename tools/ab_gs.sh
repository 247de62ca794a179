# FGMRES (MGS) at config C, k_gs_step variants: 0 = 256 threads x 4, 1 = 1024 x 4, 2 = 1024 x 8, 3 = 512 x 4
set -o pipefail
export TMPDIR=/tmp
for t in 0 1 2 3; do
  rm -rf gpurun_out/prof_gs$t
  NFFT4GP_AMD_GS_VARIANT=$t timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gs$t -o g -- python3 tools/fgmres_probe.py 1000 > gpurun_out/gs$t.log 2>&1 || { echo FAIL $t; tail -5 gpurun_out/gs$t.log; exit 1; }
  echo "variant $t: $(grep -m1 iters gpurun_out/gs$t.log)"
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_gs$t/g_kernel_stats.csv')):
    if 'gs_step' in r['Name']: print('  ', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')
"
done
