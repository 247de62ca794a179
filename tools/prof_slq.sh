# kernel trace of the config E loss with 2 SLQ workers; overlap of kernels across streams
set -o pipefail
mkdir -p gpurun_out/prof_slq
export TMPDIR=/tmp
export NFFT4GP_AMD_SLQ_STREAMS=${1:-2}
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_slq -o s -- python3 tools/config_e.py --reps 1 > gpurun_out/slq.json 2> gpurun_out/slq.err || { echo FAIL; tail -30 gpurun_out/slq.err; exit 1; }
f=$(find gpurun_out/prof_slq -name "*kernel_trace.csv" | head -1)
head -1 "$f"
python3 tools/overlap.py "$f"
