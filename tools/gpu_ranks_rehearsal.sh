#!/bin/bash
# multi-rank rehearsal on one GPU (gloo: ranks share the card): 2 and 4 ranks,
# the stream legs' report exchange per call (exchange_ms_per_call); RANKS="8"
# with SMALL=1 runs every leg at reduced sizes (the 8-rank code path)
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in ${RANKS:-2 4}; do
  extra="--no-config3 --stream-b-frames 0"
  [ -n "$SMALL" ] && extra="--frames 1024 --stream-frames 2048 --stream-b-frames 512 --config3-frames 512 --stream-warmup 5 --config3-warmup 5"
  timeout -k 10 900 python bench.py --gpus $n --backend gloo --no-cpu-baseline $extra > gpurun_out/ranks$n.json 2> gpurun_out/ranks$n.err || { tail -20 gpurun_out/ranks$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ranks$n.json'))
print('ranks $n', 'n_gpus', d['n_gpus'], round(d['value']/1e9,2), 'G', 'ms/step', round(d['ms_per_step'],3))
for k in ('stream','stream_int16','stream_B','config3'):
    s=d.get(k)
    if not s: continue
    if 'error' in s: print('  ', k, 'ERROR', s['error']); continue
    if k == 'config3': print('  ', k, round(s['value']/1e9,2), 'G'); continue
    if k == 'stream_B': print('  ', k, round(s['value']/1e9,2), 'G found', s['frames_found'], 'ok', s['frames_error_free'], 'staged', round(s['staged']['value']/1e9,2)); continue
    print('  ', k, round(s['value']/1e9,2), 'G', 'ms/call', round(s['ms_per_call'],3), 'exchange ms/call', round(s['exchange_ms_per_call'],3), 'rewalks', s['rewalks_per_call'], 'found', s['frames_found'], 'ok', s['frames_error_free'])
"
done
