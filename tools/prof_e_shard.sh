# config E loss profile, then the 8-way shard kernels; the kernel traces are dropped after the summaries
set -o pipefail
bash tools/prof_config_e.sh > gpurun_out/prof_e.txt 2>&1 || { echo PROF_E_FAIL; tail -20 gpurun_out/prof_e.txt; exit 1; }
cat gpurun_out/prof_e.txt
rm -rf gpurun_out/prof_e
bash tools/prof_shard.sh > gpurun_out/prof_sh.txt 2>&1 || { echo PROF_SH_FAIL; tail -20 gpurun_out/prof_sh.txt; exit 1; }
cat gpurun_out/prof_sh.txt
cp $(find gpurun_out/prof_sh -name "*kernel_stats.csv" | head -1) gpurun_out/shard8_kernel_stats.csv
rm -rf gpurun_out/prof_sh
