#!/bin/bash
# kernel trace of stream_bench.py-style back-to-back calls on two contexts
# (bench.py's pipelined leg, f64 stream only): walker / decode overlap
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
D=$R/gpurun_out/ov_prof; rm -rf $D
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 bench.py --no-cpu-baseline --no-config3 --stream-b-frames 0 --no-ingest --stream-pipeline 2 --steps 5 --warmup 5 > gpurun_out/ov_bench.json 2> gpurun_out/ov_bench.err || { tail gpurun_out/ov_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ov_bench.json'))
for k in ('stream','stream_int16'):
    s=d[k]; print(k, 'serial', round(s['value']/1e9,1), 'G', round(s['ms_per_call'],3), 'ms; pipelined', round(s['pipelined']['value']/1e9,1), 'G', round(s['pipelined']['ms_per_call'],3), 'ms')"
python3 tools/stream_overlap.py $D/run_kernel_trace.csv 20 > gpurun_out/stream_overlap.json && cat gpurun_out/stream_overlap.json
