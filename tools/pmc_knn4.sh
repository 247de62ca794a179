#!/bin/bash
# PMC passes over the tiled KNN screen (tools/knn_probe.py --variants 4) at n = 1e6, d = 32; one pass per group
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_INSTS_SMEM" ; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_knn4_$i
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_knn4_$i -o p -- python3 tools/knn_probe.py --variants 4 > gpurun_out/pmc_knn4_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_knn4_$i.log; exit 1; }
  f=$(find gpurun_out/pmc_knn4_$i -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "knn_tile" in r["Kernel_Name"]:
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
for c, v in sorted(acc.items()):
    print(f"k_knn_tile {c:28s} {v:.4g}")
PY
done
