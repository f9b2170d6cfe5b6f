#!/bin/bash
# scratch slot for one-off GPU commands (overwritten per experiment)
# current: stream-call ordering across streams (per-call completion event): stream tests + stream bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_stream_shard.py tests/test_bench_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/evc_tests.log 2>&1 || { tail -30 gpurun_out/evc_tests.log; exit 1; }
tail -2 gpurun_out/evc_tests.log
timeout -k 10 200 python tools/stream_bench.py --reps 10 > gpurun_out/evc_sb.log 2>&1 && timeout -k 10 200 python tools/stream_bench.py --reps 10 --i16 >> gpurun_out/evc_sb.log 2>&1; grep "^{" gpurun_out/evc_sb.log
