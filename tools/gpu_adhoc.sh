#!/bin/bash
# scratch slot for one-off GPU commands (overwritten per experiment)
# current: the profiling pass on the round's last tree
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_profile_round.sh || { echo profile_round failed; exit 1; }
python3 -c "
import json
print(json.dumps(json.load(open('gpurun_out/trace_timed.json'))))
for f in ('gpurun_out/pmc_rx.json','gpurun_out/pmc_tx.json'):
    d=json.load(open(f)); print(f, d['traffic_over_algorithmic'])
d=json.load(open('gpurun_out/bench.json'))
print('bench', d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['tx_avg_launch_ms'])
"
