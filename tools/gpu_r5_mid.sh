# Round 5 mid-round evidence: GPU suite, a no-PCG bench line, per-rank shard probes, config E, SQ counters.
set -o pipefail
mkdir -p gpurun_out/mid
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/mid/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/mid/pytest.log; exit 1; }
tail -1 gpurun_out/mid/pytest.log
timeout -k 10 400 python bench.py --no-cpu-baseline --no-traffic --no-pcg --steps 500 > gpurun_out/mid/bench_nopcg.json 2> gpurun_out/mid/bench_nopcg.err || { echo BENCH_FAIL; tail -20 gpurun_out/mid/bench_nopcg.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/mid/bench_nopcg.json'));print('matvec', round(d['ms_per_step']*1e3,2), {k:round(x*1e3,2) for k,x in d['kernels_ms'].items()}, 'frac', round(d['roofline']['frac'],3))"
timeout -k 10 120 python tools/shard_probe.py --ranks 8 > gpurun_out/mid/shard_rows8.json 2>/dev/null || { echo SHARD_FAIL; exit 1; }
timeout -k 10 120 python tools/shard_probe.py --ranks 8 --partition components > gpurun_out/mid/shard_components8.json 2>/dev/null || { echo SHARD_FAIL; exit 1; }
cat gpurun_out/mid/shard_rows8.json gpurun_out/mid/shard_components8.json
timeout -k 10 600 python tools/config_e.py > gpurun_out/mid/config_e.json 2> gpurun_out/mid/config_e.err || { echo CONFIG_E_FAIL; tail -20 gpurun_out/mid/config_e.err; exit 1; }
cat gpurun_out/mid/config_e.json
timeout -k 10 600 python tools/pmc_sq.py --out gpurun_out/mid/pmc_sq.csv > gpurun_out/mid/pmc_sq.log 2>&1 || { echo PMC_FAIL; tail -20 gpurun_out/mid/pmc_sq.log; exit 1; }
grep -E "k_spread|k_interp" gpurun_out/mid/pmc_sq.csv | head -40
