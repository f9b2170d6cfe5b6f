#!/bin/bash
# round-4 profiling pass: rx/tx kernel trace + PMC (gpu_profile_round.sh),
# stream PMC traffic (D f64 / int16, config-B wide decode), SQ counters of the
# config-B stream, the drop-in rx.cpp timing
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_profile_round.sh && echo "profile round ok" && \
bash tools/pmc_stream.sh --frames 16384 && cp gpurun_out/pmc_stream.json gpurun_out/r04k_pmc_stream.json && \
SUF=_i16 bash tools/pmc_stream.sh --frames 16384 --i16 && cp gpurun_out/pmc_stream_i16.json gpurun_out/r04k_pmc_stream_i16.json && \
SUF=_B bash tools/pmc_stream.sh --config B --frames 4096 && cp gpurun_out/pmc_stream_B.json gpurun_out/r04k_pmc_stream_B.json && \
echo "pmc stream ok" && \
bash tools/sq_stream.sh --config B --frames 4096 && cp gpurun_out/sq_stream.txt gpurun_out/r04k_sq_stream_B.txt && echo "sq ok" && \
timeout -k 10 300 python tools/dropin_rx_timing.py --frames 200 > gpurun_out/r04k_dropin_rx_timing.json 2> gpurun_out/r04k_dropin.err && echo "dropin ok"
