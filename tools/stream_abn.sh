#!/bin/bash
# stream tests, then the stream bench (f64 and int16) and a kernel-stats
# profile for each library variant: VARIANTS="name:lib name2: ..." (empty lib
# = the product build). Output: gpurun_out/stream_abn.txt, gpurun_out/abn_<name>/
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_sync.py -x -q --timeout 120 --timeout-method thread > gpurun_out/stream_tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in $VARIANTS; do
    n=${v%%:*}; l=${v#*:}
    if [ -n "$l" ]; then export OFDM_MI355X_LIB=$l; else unset OFDM_MI355X_LIB; fi
    timeout -k 10 120 python tools/stream_bench.py 2>/dev/null | sed "s/^/$n /" >> gpurun_out/stream_abn.txt || exit 1
    timeout -k 10 120 python tools/stream_bench.py --i16 2>/dev/null | sed "s/^/$n /" >> gpurun_out/stream_abn.txt || exit 1
    if [ $r = 1 ]; then
      timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abn_$n -o run -- python3 tools/stream_bench.py --reps 3 > /dev/null 2>&1 || exit 1
    fi
  done
done
unset OFDM_MI355X_LIB
