#!/bin/bash
# round-4 check: stream (ring mode) + sync + drop-in + parity tests, then the default bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r04b}
rm -f gpurun_out/stream_full_summary.jsonl
timeout -k 10 1000 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_stream_shard.py tests/test_dropin_gpu.py tests/test_gpu_sync.py tests/test_gpu_parity.py tests/test_gpu_stream_full.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/${TAG}_bench.json'))
print('value', d['value']/1e9, 'ms', d['ms_per_step'], 'rx frac', d['roofline']['frac'], 'rx ms', d['roofline']['avg_launch_ms'], 'tx ms', d['tx_avg_launch_ms'])
for k in ('stream','stream_int16'):
    s=d[k]; print(k, s['value']/1e9, s['ms_per_call'], s['roofline']['frac'], s['frames_found'], s['frames_error_free'], s['rewalks_per_call'], s.get('pipelined',{}).get('value',0)/1e9)
"
