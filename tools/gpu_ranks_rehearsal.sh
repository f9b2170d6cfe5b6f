#!/bin/bash
# multi-rank rehearsal on one GPU (gloo: ranks share the card): 2 and 4 ranks,
# the stream legs' report exchange per call (exchange_ms_per_call)
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 2 4; do
  timeout -k 10 900 python bench.py --gpus $n --backend gloo --no-cpu-baseline --no-config3 --stream-b-frames 0 > gpurun_out/ranks$n.json 2> gpurun_out/ranks$n.err || { tail -20 gpurun_out/ranks$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ranks$n.json'))
print('ranks $n', 'n_gpus', d['n_gpus'], round(d['value']/1e9,2), 'G', 'ms/step', round(d['ms_per_step'],3))
for k in ('stream','stream_int16'):
    s=d[k]; print('  ', k, round(s['value']/1e9,2), 'G', 'ms/call', round(s['ms_per_call'],3), 'exchange ms/call', round(s['exchange_ms_per_call'],3), 'rewalks', s['rewalks_per_call'], 'found', s['frames_found'], 'ok', s['frames_error_free'])
"
done
