#!/bin/bash
# scratch slot for one-off GPU commands (overwritten per experiment)
# current: the round-6 profiling pass (headline trace + PMC, stream kernel
# means + PMC, SQ counters of the stream kernels, the two-context overlap trace)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
bash tools/gpu_profile_round.sh || { echo profile_round failed; exit 1; }
python3 -c "
import json
print(json.dumps(json.load(open('gpurun_out/trace_timed.json'))))
for f in ('gpurun_out/pmc_rx.json','gpurun_out/pmc_tx.json'):
    d=json.load(open(f)); print(f, d['traffic_over_algorithmic'])
d=json.load(open('gpurun_out/bench.json'))
print('bench', d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['tx_avg_launch_ms'])
"
bash tools/gpu_stream_trace.sh > gpurun_out/r06_stream_trace.log 2>&1 || { tail gpurun_out/r06_stream_trace.log; exit 1; }
tail -40 gpurun_out/r06_stream_trace.log
TAG=r06 bash tools/gpu_profile_stream.sh || exit 1
bash tools/sq_stream.sh --frames 16384 --i16 && cp gpurun_out/sq_stream.txt gpurun_out/r06_sq_stream_Di16.txt && \
bash tools/sq_stream.sh --frames 16384 && cp gpurun_out/sq_stream.txt gpurun_out/r06_sq_stream_D.txt || exit 1
bash tools/gpu_stream_overlap.sh
