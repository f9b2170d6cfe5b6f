#!/bin/bash
# round 4, last tree: the profiling pass (rx/tx kernel trace + PMC traffic and
# the bench line, tools/gpu_profile_round.sh), the stream PMC traffic (D f64,
# D int16, config-B wide decode) and the drop-in rx.cpp timing
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_profile_round.sh && echo "profile round ok" && \
bash tools/pmc_stream.sh --frames 16384 && cp gpurun_out/pmc_stream.json gpurun_out/r04z_pmc_stream.json && \
SUF=_i16 bash tools/pmc_stream.sh --frames 16384 --i16 && cp gpurun_out/pmc_stream_i16.json gpurun_out/r04z_pmc_stream_i16.json && \
SUF=_B bash tools/pmc_stream.sh --config B --frames 4096 && cp gpurun_out/pmc_stream_B.json gpurun_out/r04z_pmc_stream_B.json && \
echo "pmc stream ok" && \
timeout -k 10 300 python tools/dropin_rx_timing.py --frames 200 > gpurun_out/r04z_dropin_rx_timing.json 2> gpurun_out/r04z_dropin.err && echo "dropin ok"
