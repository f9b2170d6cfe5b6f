#!/bin/bash
# SQ counters of the config-B stream (wide fused decode), then the D stream
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/sq_stream.sh --config B --frames 4096 && cp gpurun_out/sq_stream.txt gpurun_out/r04j_sq_stream_B.txt && cat gpurun_out/r04j_sq_stream_B.txt
