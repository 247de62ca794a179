# Round 5: two-vector interpolation threads at config E (loss probe pairs), component shard after the grouping rule,
# and bench.py's own rank launcher on a one-GPU box (gloo rehearsal: n_gpus 2; RCCL: refused).
set -o pipefail
mkdir -p gpurun_out/b
for rep in 1 2; do
  for t in 1024 512; do
    NFFT4GP_AMD_INTERP2_THREADS=$t timeout -k 10 600 python tools/config_e.py --reps 10 > gpurun_out/b/config_e_$t.json 2>/dev/null || { echo CONFIG_E_FAIL; exit 1; }
    tail -1 gpurun_out/b/config_e_$t.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('interp2 $t rep $rep', round(d['matvecs_per_s'],1), 'loss', round(d['loss_s'],3), round(d['loss_dcgs2_s'],3))"
  done
done
timeout -k 10 120 python tools/shard_probe.py --ranks 8 --partition components > gpurun_out/b/shard_components8.json 2>/dev/null || { echo SHARD_FAIL; exit 1; }
cat gpurun_out/b/shard_components8.json
NFFT4GP_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --no-pcg --no-cpu-baseline --no-traffic --steps 50 > gpurun_out/b/bench_gloo2.json 2> gpurun_out/b/bench_gloo2.err || { echo GLOO2_FAIL; tail -20 gpurun_out/b/bench_gloo2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b/bench_gloo2.json'));print('gloo2 n_gpus', d['n_gpus'], 'comm_ranks', d['comm_ranks'], 'rccl_ranks', d['rccl_ranks'], d['per_rank'])"
timeout -k 10 300 python bench.py --gpus 2 --no-pcg --no-cpu-baseline --no-traffic --steps 50 > gpurun_out/b/bench_rccl2.json 2> gpurun_out/b/bench_rccl2.err
echo "rccl --gpus 2 on one GPU: exit $?"; tail -2 gpurun_out/b/bench_rccl2.err
