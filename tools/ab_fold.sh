# A/B of the spread fold (variant 1: two chains; variant 8: one chain) at config C and config E, one box
set -o pipefail
bash tools/ab_spread.sh "1:4064 8:4064" --steps 500 || exit 1
for rep in 1 2; do for v in 1 8; do
NFFT4GP_AMD_SPREAD_VARIANT=$v timeout -k 10 300 python3 tools/config_e.py --reps 5 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('config E variant $v', round(d['matvecs_per_s'],1), d['kernels_ms'])" || exit 1
done; done
