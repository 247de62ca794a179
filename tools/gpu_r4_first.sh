set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_dist.py -m gpu -x -v --timeout 600 --timeout-method thread -k "component_shards or config_b_pcg or config_c_pcg or rccl or callback" > gpurun_out/r4/pt1.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r4/pt1.log; exit 1; }
grep -E "PASS|FAIL|config" gpurun_out/r4/pt1.log | tail -20
timeout -k 10 120 python tools/shard_probe.py --ranks 8 --partition components --reps 1000 > gpurun_out/r4/shard_comp8.json 2>&1 || { echo PROBE_FAIL; tail gpurun_out/r4/shard_comp8.json; exit 1; }
timeout -k 10 120 python tools/shard_probe.py --ranks 8 --reps 1000 > gpurun_out/r4/shard_rows8.json 2>&1 || { echo PROBE_FAIL; exit 1; }
cat gpurun_out/r4/shard_comp8.json gpurun_out/r4/shard_rows8.json
timeout -k 10 400 python bench.py --steps 200 --warmup 20 --no-pcg --no-traffic > gpurun_out/r4/b1.json 2> gpurun_out/r4/b1.err || { echo BENCH_FAIL; tail -30 gpurun_out/r4/b1.err; exit 1; }
python -c "
import json; r=json.load(open('gpurun_out/r4/b1.json')); print(r['value'], r['roofline']['frac'], r['kernels_ms']); print(json.dumps(r['cpu_baseline'])[:900])"
