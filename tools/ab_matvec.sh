# A/B probe for matvec kernel changes: hot-path GPU tests, two bench --no-pcg runs, the shard probe at N = 8/4/2, config E
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_nfft.py tests/test_gpu_dist.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pt.log; exit 1; }
tail -2 gpurun_out/pt.log
for r in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic --no-pcg --steps 500 > gpurun_out/b$r.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }; python -c "import json;d=json.load(open('gpurun_out/b$r.json'));print(round(d['ms_per_step']*1e3,2), {k:round(x*1e3,2) for k,x in d['kernels_ms'].items()})"; done
for N in 8 4 2; do timeout -k 10 300 python tools/shard_probe.py --ranks $N 2>/dev/null | tail -1 || exit 1; done
timeout -k 10 300 python3 tools/config_e.py --reps 5 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('config E', d['matvecs_per_s'], d['kernels_ms'])"
