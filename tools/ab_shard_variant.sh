# spread variants on the row-shard probe (N = 8 / 4) and the bench matvec, one box.  Variants 9 (256 threads)
# and 10 (1024 threads) were removed after the round-3 measurement; re-add them to re-run this.
set -o pipefail
for rep in 1 2; do for v in 1 9 10; do
  for N in 8 4; do echo -n "variant $v N=$N "; NFFT4GP_AMD_SPREAD_VARIANT=$v timeout -k 10 300 python tools/shard_probe.py --ranks $N 2>/dev/null | tail -1 || exit 1; done
done; done
bash tools/ab_spread.sh "1:4064 9:4064 10:4064" --steps 300 || exit 1
