#!/bin/bash
# round-4: walker debug on the exact-zero capture, kernel traces of the config-B
# stream (fused wide decode vs staged), then the pipelined A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r04e}
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -k "wide or config_b" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_wide_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_wide_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_wide_tests.log
timeout -k 10 300 python tools/walk_debug.py > gpurun_out/${TAG}_walk_debug.log 2>&1 || { cat gpurun_out/${TAG}_walk_debug.log; exit 1; }
cat gpurun_out/${TAG}_walk_debug.log
for mode in fused staged; do
  tun=""; [ $mode = staged ] && tun="--walk-tuning staged_decode=1"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_B_$mode -o run -- python3 tools/stream_bench.py --config B --frames 4096 --reps 5 $tun > gpurun_out/${TAG}_prof_B_$mode.json 2> gpurun_out/${TAG}_prof_B_$mode.err || { tail gpurun_out/${TAG}_prof_B_$mode.err; exit 1; }
  f=$(find gpurun_out/${TAG}_prof_B_$mode -name "*kernel_stats.csv" | head -1)
  echo "== $mode"; cut -d, -f1-8 "$f" | head -12
done
bash tools/pipelined_ab.sh ${TAG}
