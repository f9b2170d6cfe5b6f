#!/bin/bash
# round-4 check: the wide fused stream decode (B/C) first, its A/B against the
# staged kernels, then the stream/sync/drop-in/parity suites and the bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r04d}
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -k "wide or config_b or walk_tuning" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_wide_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_wide_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_wide_tests.log
for cfg in B C; do
  for tun in "" "--walk-tuning staged_decode=1"; do
    timeout -k 10 200 python tools/stream_bench.py --config $cfg --frames 4096 --reps 5 $tun >> gpurun_out/${TAG}_stream_wide_ab.jsonl 2>> gpurun_out/${TAG}_stream_wide_ab.err || { tail gpurun_out/${TAG}_stream_wide_ab.err; exit 1; }
  done
done
timeout -k 10 200 python tools/stream_bench.py --config B --frames 4096 --reps 5 --i16 >> gpurun_out/${TAG}_stream_wide_ab.jsonl 2>> gpurun_out/${TAG}_stream_wide_ab.err || exit 1
cat gpurun_out/${TAG}_stream_wide_ab.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['workload'], d['ms'], d['G_stream_samples_per_s'], d['frames_found'], d['frames_error_free'], d['roofline']['frac'])"
bash tools/gpu_r04b.sh ${TAG}
