#!/bin/bash
# batched predictive std: the krylov tests that cover predict, then the batch-size probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_krylov.py -x -v --timeout 200 --timeout-method thread -k predict > gpurun_out/predict_tests.log 2>&1 || { tail -30 gpurun_out/predict_tests.log; exit 1; }
tail -6 gpurun_out/predict_tests.log
timeout -k 10 400 python tools/predict_probe.py --n 20000 --npred 64 > gpurun_out/predict_probe.txt 2>&1 || { tail -20 gpurun_out/predict_probe.txt; exit 1; }
timeout -k 10 300 python tools/predict_probe.py --n 200000 --npred 32 --d 16 --batches 1,16,32 >> gpurun_out/predict_probe.txt 2>&1 || { tail -20 gpurun_out/predict_probe.txt; exit 1; }
grep '^{' gpurun_out/predict_probe.txt
