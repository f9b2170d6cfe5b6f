#!/bin/bash
# scratch slot for one-off GPU commands (overwritten per experiment)
# current: multi-rank launch rehearsals on the final tree (one MI355X): torch.distributed.run with one
# RCCL rank, and the self-launcher with 2 gloo ranks sharing the card
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --no-cpu-baseline > gpurun_out/rccl1.json 2> gpurun_out/rccl1.err || { tail -20 gpurun_out/rccl1.err; exit 1; }
timeout -k 10 500 python bench.py --gpus 2 --backend gloo --no-cpu-baseline > gpurun_out/gloo2.json 2> gpurun_out/gloo2.err || { tail -20 gpurun_out/gloo2.err; exit 1; }
python3 -c "
import json
for f in ('gpurun_out/rccl1.json','gpurun_out/gloo2.json'):
    d=json.load(open(f)); c=d['config']
    print(f, d['n_gpus'], c.get('backend'), round(d['value']/1e9,1), round(d['ms_per_step'],4), round(d['roofline']['frac'],3), round(d['stream']['value']/1e9,1), d['stream'].get('exchange_ms_per_call'), round(d['stream_int16']['value']/1e9,1), round(d['config3']['value']/1e9,1))
"
