# Per-rank row-shard matvec time (tools/shard_probe.py, N = 8) over layout knobs: window groups per spread
# workgroup (NFFT4GP_AMD_CG) and block size (NFFT4GP_AMD_BLOCK).  Two reps each, one box.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for cg in 1 2 3; do
    for b in 1016 2032; do
      r=$(NFFT4GP_AMD_CG=$cg NFFT4GP_AMD_BLOCK=$b timeout -k 10 120 python tools/shard_probe.py --ranks ${RANKS:-8} 2>/dev/null) || { echo PROBE_FAIL cg=$cg b=$b; exit 1; }
      echo "cg=$cg B=$b rep=$rep $r"
    done
  done
done
