# GPU-box jobs, one script for all of them (run through gpurun from the repo root; outputs under gpurun_out/):
#   bash tools/gpu_job.sh tests [pytest args]   GPU tests in one pytest process (default: the whole suite)
#   bash tools/gpu_job.sh driver                the driver's round-end commands in its order: GPU suite, smoke(),
#                                               the default bench line (gpurun_out/driver_*)
#   bash tools/gpu_job.sh evidence [--gloo2]    driver, then a rocprofv3 kernel trace of the headline bench with
#                                               tools/prof_summary.py over its timed loops, the SQ / LDS counter
#                                               passes (tools/pmc_sq.py) and optionally a 2-rank gloo rehearsal
#   bash tools/gpu_job.sh bitwise "ENV_A" "ENV_B" [interp_check configs separated by ';']
#                                               one matvec under two settings (commas join variables), compared
#                                               bit for bit (tools/interp_check.py)
#   bash tools/gpu_job.sh config-e [ENV=V ...]  config E's operator + loss (tools/config_e.py) under rocprofv3,
#                                               top kernels by total time
# Every GPU step runs under its own time limit, and the first failure ends the job.
set -o pipefail
mkdir -p gpurun_out
mode="$1"; shift

run_tests() {
  if [ $# -eq 0 ]; then set -- tests; fi
  timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -5; tail -60 gpurun_out/pytest_gpu.log; return 1; }
  tail -3 gpurun_out/pytest_gpu.log
}

run_driver() {
  timeout -k 10 1100 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/driver_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/driver_pytest.log; return 1; }
  tail -3 gpurun_out/driver_pytest.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/driver_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/driver_smoke.log; return 1; }
  tail -2 gpurun_out/driver_smoke.log
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driver_bench.json 2> gpurun_out/driver_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/driver_bench.err; return 1; }
  tail -c 600 gpurun_out/driver_bench.json; echo
}

run_evidence() {
  run_driver || return 1
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || return 1
  rm -rf gpurun_out/prof gpurun_out/oracle_native
  # config C only (--no-config-e), so the trace's last timed loops are the headline's
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-traffic --no-pcg --no-config-e > gpurun_out/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_bench.log; return 1; }
  python tools/prof_summary.py $(find gpurun_out/prof -name "*kernel_trace.csv" | head -1) --steps 200 --out gpurun_out/prof_summary.json
  cp $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1) gpurun_out/prof_kernel_stats.csv
  rm -rf gpurun_out/prof  # the full trace is > 64 MiB: gpurun would not copy gpurun_out/ back
  head -c 1200 gpurun_out/prof_summary.json; echo
  timeout -k 10 600 python tools/pmc_sq.py --out gpurun_out/pmc_sq.csv > gpurun_out/pmc_sq.log 2>&1 || { echo PMC_SQ_FAIL; tail -20 gpurun_out/pmc_sq.log; return 1; }
  tail -2 gpurun_out/pmc_sq.log
  rm -rf gpurun_out/pmc_sq
  if [ "$1" = "--gloo2" ]; then
    # the N > 1 path with 2 gloo ranks on the one GPU (host all-reduce through the callback communicator)
    NFFT4GP_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || { echo GLOO2_FAIL; tail -30 gpurun_out/bench_gloo2.err; return 1; }
    tail -c 400 gpurun_out/bench_gloo2.json; echo
  fi
}

run_bitwise() {
  local a="$1" b="$2" cfgs="${3:---n 1000000 --d 32;--n 10000000 --d 64 --precision 32;--n 10000000 --d 64}"
  local IFS_OLD="$IFS"; IFS=';'; set -- $cfgs; IFS="$IFS_OLD"
  for cfg in "$@"; do
    env $(echo "$a" | tr ',' ' ') timeout -k 10 120 python tools/interp_check.py $cfg --out gpurun_out/y_a.npy > /dev/null 2> gpurun_out/bw_a.err || { echo CHECK_A_FAIL; tail gpurun_out/bw_a.err; return 1; }
    env $(echo "$b" | tr ',' ' ') timeout -k 10 120 python tools/interp_check.py $cfg --out gpurun_out/y_b.npy > /dev/null 2> gpurun_out/bw_b.err || { echo CHECK_B_FAIL; tail gpurun_out/bw_b.err; return 1; }
    python -c "import numpy as np;a=np.load('gpurun_out/y_a.npy');b=np.load('gpurun_out/y_b.npy');print('[$cfg] bitwise', np.array_equal(a,b), 'max rel', float(np.abs(a-b).max()/np.abs(a).max()))"
  done
  rm -f gpurun_out/y_a.npy gpurun_out/y_b.npy  # 80 MB each at n = 1e7: keep gpurun_out/ under 64 MiB
}

run_config_e() {
  mkdir -p gpurun_out/prof_e
  export TMPDIR=/tmp
  env "$@" timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_e -o e -- python3 tools/config_e.py --reps 5 > gpurun_out/config_e.json 2> gpurun_out/config_e.err || { echo CONFIG_E_FAIL; tail -30 gpurun_out/config_e.err; return 1; }
  tail -1 gpurun_out/config_e.json
  cp "$(find gpurun_out/prof_e -name "*kernel_stats.csv" | head -1)" gpurun_out/config_e_kernel_stats.csv
  rm -rf gpurun_out/prof_e
  python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/config_e_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.2f} us  {r["Name"][:90]}')
PY
}

case "$mode" in
  tests) run_tests "$@" ;;
  driver) run_driver ;;
  evidence) run_evidence "$@" ;;
  bitwise) run_bitwise "$@" ;;
  config-e) run_config_e "$@" ;;
  *) echo "usage: bash tools/gpu_job.sh tests|driver|evidence|bitwise|config-e ..."; exit 2 ;;
esac
