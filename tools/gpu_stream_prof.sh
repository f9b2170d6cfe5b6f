# Development GPU pass for the streaming receiver: gpu parity tests, then the
# config-4 stream bench under rocprofv3 --kernel-trace --stats.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stream -o run -- python3 tools/stream_bench.py --reps 3 ${STREAM_ARGS} > gpurun_out/stream_prof.log 2>&1 || exit 1
grep workload gpurun_out/stream_prof.log
python3 - <<'PY'
import csv
for x in csv.DictReader(open('gpurun_out/prof_stream/run_kernel_stats.csv')):
    if 'ofdm' in x['Name']:
        print(x['Name'][:64], x['Calls'], round(float(x['AverageNs']) / 1000, 1), 'us')
PY
