#!/bin/bash
# A/B of where the one stream-call marker sits: before the compaction (markpre,
# abtest build) or after it (the product build).
# config-4 stream bench alternating the two on the same box, f64 and int16,
# and a kernel trace of the markpre build.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/stream_tests_u.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in markpre new; do
    if [ $v = markpre ]; then export OFDM_MI355X_LIB=abtest/libofdm_markpre.so; else unset OFDM_MI355X_LIB; fi
    timeout -k 10 120 python tools/stream_bench.py 2>/dev/null | sed "s/^/$v /" >> gpurun_out/stream_ab_u.txt || exit 1
    timeout -k 10 120 python tools/stream_bench.py --i16 2>/dev/null | sed "s/^/$v /" >> gpurun_out/stream_ab_u.txt || exit 1
  done
done
export OFDM_MI355X_LIB=abtest/libofdm_markpre.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sprof_u -o run -- python3 tools/stream_bench.py --reps 10 > gpurun_out/sprof_u.log 2>&1
