#!/bin/bash
# scratch slot for one-off GPU commands (overwritten per experiment)
# current: the round's final profiling pass on HEAD (headline profile + PMC, stream PMC f64/int16)
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_profile_round.sh || { echo profile_round failed; exit 1; }
bash tools/pmc_stream.sh || { echo pmc_stream failed; exit 1; }
SUF=_i16 bash tools/pmc_stream.sh --i16 || { echo pmc_stream i16 failed; exit 1; }
python3 -c "
import json
for f in ('gpurun_out/trace_timed.json','gpurun_out/pmc_rx.json','gpurun_out/pmc_tx.json','gpurun_out/pmc_stream.json','gpurun_out/pmc_stream_i16.json'):
    print(f, json.dumps(json.load(open(f)))[:600])
d=json.load(open('gpurun_out/bench.json'))
print('bench', d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['tx_avg_launch_ms'], d['stream']['value']/1e9, d['stream_int16']['value']/1e9, d['config3']['value']/1e9)
"
