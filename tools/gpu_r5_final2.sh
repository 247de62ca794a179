# round-5 final evidence, part 2: config B line, per-rank shard probes (rows, rows + peer exchange, components),
# config E in both precisions, the KNN screens and the config-C AFN setup
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 600 python bench.py --n 100000 --d 8 --nys-rank 256 --afn-rank 256 --steps 200 --warmup 20 --no-traffic > gpurun_out/final/config_b.json 2> gpurun_out/final/config_b.err || { echo CONFIG_B_FAIL; tail -20 gpurun_out/final/config_b.err; exit 1; }
timeout -k 10 120 python tools/shard_probe.py --ranks 8 > gpurun_out/final/shard_rows8.json 2>/dev/null || { echo SHARD_FAIL; exit 1; }
timeout -k 10 120 python tools/shard_probe.py --ranks 8 --peer > gpurun_out/final/shard_rows8_peer.json 2>/dev/null || { echo SHARD_FAIL; exit 1; }
timeout -k 10 120 python tools/shard_probe.py --ranks 8 --partition components > gpurun_out/final/shard_components8.json 2>/dev/null || { echo SHARD_FAIL; exit 1; }
cat gpurun_out/final/shard_rows8.json gpurun_out/final/shard_rows8_peer.json gpurun_out/final/shard_components8.json
timeout -k 10 600 python tools/config_e.py > gpurun_out/final/config_e.json 2> gpurun_out/final/config_e.err || { echo CONFIG_E_FAIL; tail -20 gpurun_out/final/config_e.err; exit 1; }
timeout -k 10 600 python tools/config_e.py --precision 32 > gpurun_out/final/config_e_32.json 2> gpurun_out/final/config_e_32.err || { echo CONFIG_E32_FAIL; tail -20 gpurun_out/final/config_e_32.err; exit 1; }
tail -1 gpurun_out/final/config_e.json; tail -1 gpurun_out/final/config_e_32.json
timeout -k 10 200 python -u tools/knn_probe.py --variants 4,3,1 > gpurun_out/final/knn_probe.json 2>/dev/null || { echo KNN_FAIL; exit 1; }
timeout -k 10 120 python -u tools/afn_config_c_probe.py > gpurun_out/final/afn_c.log 2>&1 || { echo AFN_FAIL; exit 1; }
tail -1 gpurun_out/final/knn_probe.json; tail -1 gpurun_out/final/afn_c.log
