# Scratch slot for one-off GPU commands (`gpurun -- bash tools/gpu_adhoc.sh`);
# its content changes with the experiment at hand and is not part of any flow.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_stream.py -k "defaults" > gpurun_out/t.log 2>&1; tail -1 gpurun_out/t.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config3 > gpurun_out/hb.json 2> gpurun_out/hb.err || { tail gpurun_out/hb.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/hb.json'))
print(*[(k, round(d[k]['value']/1e9,1), round(d[k]['roofline']['avg_call_ms'],3), d[k]['rewalks_per_call']) for k in ('stream','stream_int16')])"
