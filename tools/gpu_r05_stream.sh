export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_stream_full.py tests/test_gpu_stream_shard.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05a_stream_tests.log 2>&1 || { tail -80 gpurun_out/r05a_stream_tests.log; exit 1; }
tail -3 gpurun_out/r05a_stream_tests.log
timeout -k 10 400 python bench.py --no-config3 --stream-b-frames 4096 --no-cpu-baseline > gpurun_out/r05a_bench.json 2> gpurun_out/r05a_bench.err || { tail gpurun_out/r05a_bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/r05a_bench.json'))
print('value', d['value']/1e9, 'rx frac', d['roofline']['frac'])
for k in ('stream','stream_int16','stream_B'):
    s=d[k]; print(k, s['value']/1e9, s['ms_per_call'], s['roofline']['frac'], s['frames_found'], s['frames_error_free'], s['rewalks_per_call'])
"
