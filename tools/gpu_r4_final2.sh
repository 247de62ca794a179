# round-4 final evidence, part 2: config B bench line, per-rank shard probes (rows, components), config E tool
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 600 python bench.py --n 100000 --d 8 --nys-rank 256 --afn-rank 256 --steps 200 --warmup 20 --no-traffic > gpurun_out/final/config_b.json 2> gpurun_out/final/config_b.err || { echo CONFIG_B_FAIL; tail -20 gpurun_out/final/config_b.err; exit 1; }
timeout -k 10 120 python tools/shard_probe.py --ranks 8 > gpurun_out/final/shard_rows8.json 2>/dev/null || { echo SHARD_FAIL; exit 1; }
timeout -k 10 120 python tools/shard_probe.py --ranks 8 --partition components > gpurun_out/final/shard_components8.json 2>/dev/null || { echo SHARD_FAIL; exit 1; }
cat gpurun_out/final/shard_rows8.json gpurun_out/final/shard_components8.json
timeout -k 10 600 python tools/config_e.py > gpurun_out/final/config_e.json 2> gpurun_out/final/config_e.err || { echo CONFIG_E_FAIL; tail -20 gpurun_out/final/config_e.err; exit 1; }
cat gpurun_out/final/config_e.json
