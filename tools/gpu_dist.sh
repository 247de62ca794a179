# distributed path on one GPU: the gloo/RCCL GPU tests and a two-rank bench rehearsal (gloo, one GPU)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_dist.log; exit 1; }
tail -15 gpurun_out/pytest_dist.log
NFFT4GP_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || { echo BENCH2_FAIL; tail -40 gpurun_out/bench_gloo2.err; exit 1; }
cat gpurun_out/bench_gloo2.json
