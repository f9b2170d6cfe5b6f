#!/bin/bash
# Stream-path GPU check: the stream parity tests, then tools/stream_bench.py
# f64 and int16 (two runs each). Output: gpurun_out/${TAG}_*
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-sc}
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_stream_full.py tests/test_gpu_stream_shard.py tests/test_gpu_sync.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log; grep "stream: {\|shards: {" gpurun_out/${TAG}_tests.log
: > gpurun_out/${TAG}_bench.txt
for i16 in "" "--i16" "" "--i16"; do
  timeout -k 10 200 python tools/stream_bench.py --reps 10 $i16 > gpurun_out/${TAG}_sb.json 2> gpurun_out/${TAG}_sb.err || { tail gpurun_out/${TAG}_sb.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_sb.json').read().splitlines()[-1]);print('$i16', d['ms'], d['G_stream_samples_per_s'], d['roofline']['frac'], d['frames_found'])" | tee -a gpurun_out/${TAG}_bench.txt
done
