# md tiled spread/interp work-item size (NFFT4GP_AMD_MD_CHUNK = taps per item) on tools/md_probe.py's configurations
set -o pipefail
for c in ${CHUNKS:-2000000 500000 200000}; do
  echo "chunk_taps=$c"
  NFFT4GP_AMD_MD_CHUNK=$c timeout -k 10 300 python tools/md_probe.py 2>/dev/null || { echo MD_PROBE_FAIL; exit 1; }
done
