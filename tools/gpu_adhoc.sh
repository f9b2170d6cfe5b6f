#!/bin/bash
# scratch slot for one-off GPU commands (overwritten per experiment)
# current: walker FP32 tier of the FFT preamble search: stream parity, same-box
# A/B against the previous build, walker phase clocks
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
TAG=${1:-r06f}
timeout -k 10 900 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_stream_full.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
TAG=$TAG LIBS="product abtest/libofdm_head.so" bash tools/stream_ab.sh || exit 1
TUNINGS=chunks_per_slot=1 bash tools/gpu_walk_prof.sh
