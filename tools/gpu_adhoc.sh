#!/bin/bash
# scratch slot for one-off GPU commands (overwritten per experiment)
# current: FP32 preamble-search screen in the stream walker: the stream parity
# tests, then a same-box A/B against HEAD's build (abtest/libofdm_head.so)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_stream_full.py tests/test_gpu_stream_shard.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s32_tests.log 2>&1 || { tail -30 gpurun_out/s32_tests.log; exit 1; }
tail -2 gpurun_out/s32_tests.log
LIBS="abtest/libofdm_head.so product" TAG=s32 timeout -k 10 700 bash tools/stream_ab.sh || exit 1
cat gpurun_out/s32_stream_ab.txt
