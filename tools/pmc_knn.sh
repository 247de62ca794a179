# PMC passes over the KNN screen kernels (tools/knn_probe.py, variant 1) at n = 1e6, d = 32; one pass per
# counter group (rocprofv3 does not split counters over passes).
set -o pipefail
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC" \
           "TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_knn$i
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_knn$i -o p -- python3 tools/knn_probe.py --variants 1 > gpurun_out/pmc_knn$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_knn$i.log; continue; }
  f=$(find gpurun_out/pmc_knn$i -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "knn_screen" in r["Kernel_Name"]:
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        acc[(k, r["Counter_Name"])] += float(r["Counter_Value"])
for (k, c), v in sorted(acc.items()):
    print(f"{k:32s} {c:28s} {v:.4g}")
PY
done
