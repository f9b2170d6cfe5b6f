#!/bin/bash
# Stream development pass: stream parity tests (walk vs the oracle's
# sequential walk, decode vs the oracle chain), the config-4 stream bench
# (f64 + int16), then its kernel stats under rocprofv3. Output: gpurun_out/si_*
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-si}
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_stream_full.py tests/test_gpu_stream_shard.py tests/test_gpu_sync.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python tools/stream_bench.py --reps 10 > gpurun_out/${TAG}_stream.json 2> gpurun_out/${TAG}_stream.err || exit 1
timeout -k 10 200 python tools/stream_bench.py --reps 10 --i16 >> gpurun_out/${TAG}_stream.json 2>> gpurun_out/${TAG}_stream.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 tools/stream_bench.py --reps 5 > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python3 - "$TAG" <<'PY'
import csv, json, sys
tag = sys.argv[1]
for l in open(f'gpurun_out/{tag}_stream.json'):
    d = json.loads(l)
    print(d.get('workload'), d.get('G_stream_samples_per_s'), d.get('ms'))
for x in csv.DictReader(open(f'gpurun_out/{tag}_prof/run_kernel_stats.csv')):
    if 'ofdm' in x['Name']:
        print(x['Name'][:64], x['Calls'], round(float(x['AverageNs']) / 1000, 1), 'us')
PY
