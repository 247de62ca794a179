#!/bin/bash
# KNN tiled screen: in-tree (A) against gpurun_ab (B) on tools/knn_probe.py (variant 4) and the config-C AFN setup
set -o pipefail
mkdir -p gpurun_out
LIB=preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd/libnfft4gp_amd.so
cp $LIB gpurun_out/lib_a.so || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_knn.py > gpurun_out/knn_tests.log 2>&1 || { echo KNN_TESTS_FAIL; tail -20 gpurun_out/knn_tests.log; exit 1; }
tail -1 gpurun_out/knn_tests.log
for rep in 1 2; do
  for v in a b; do
    if [ $v = a ]; then cp gpurun_out/lib_a.so $LIB; else cp gpurun_ab/libnfft4gp_amd.so $LIB; fi
    echo -n "lib $v rep $rep knn "; timeout -k 10 120 python -u tools/knn_probe.py --variants 4,4 2>/dev/null | tail -1 || exit 1
    echo -n "lib $v rep $rep "; timeout -k 10 120 python -u tools/afn_config_c_probe.py 2>/dev/null | tail -1 || exit 1
  done
done
cp gpurun_out/lib_a.so $LIB
