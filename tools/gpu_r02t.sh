#!/bin/bash
# A/B of the stream call's event placement (one marker between the stream
# kernels instead of two): stream parity tests on the new build, then the
# config-4 stream bench alternating HEAD (abtest/libofdm_head.so) and new on
# the same box, f64 and int16, and a kernel trace of the new build.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_stream_shard.py tests/test_gpu_threads.py tests/test_bench_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/stream_tests.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in head new; do
    if [ $v = head ]; then export OFDM_MI355X_LIB=abtest/libofdm_head.so; else unset OFDM_MI355X_LIB; fi
    timeout -k 10 120 python tools/stream_bench.py 2>/dev/null | sed "s/^/$v /" >> gpurun_out/stream_ab.txt || exit 1
    timeout -k 10 120 python tools/stream_bench.py --i16 2>/dev/null | sed "s/^/$v /" >> gpurun_out/stream_ab.txt || exit 1
  done
done
unset OFDM_MI355X_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sprof_t -o run -- python3 tools/stream_bench.py --reps 10 > gpurun_out/sprof_t.log 2>&1
