#!/bin/bash
# same-box A/B: abtest/libofdm_base.so (before the cache touches) vs the product
# build, stream_bench D f64 / int16 and config B, kernel traces; then the stream
# parity tests on the product build
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/r04l_touch_ab.txt
: > $OUT
for round in 1 2; do
  for lib in abtest/libofdm_base.so product; do
    for args in "--frames 16384" "--frames 16384 --i16" "--config B --frames 4096"; do
      if [ "$lib" = product ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=$R/$lib; fi
      D=$R/gpurun_out/ab_prof; rm -rf $D
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/stream_bench.py --reps 5 $args > gpurun_out/ab_sb.log 2>&1 || { tail gpurun_out/ab_sb.log; exit 1; }
      python3 - "$lib" "$args" "$D/run_kernel_stats.csv" gpurun_out/ab_sb.log >> $OUT <<'PY'
import csv, json, sys
lib, args, stats, log = sys.argv[1:5]
k = {}
for x in csv.DictReader(open(stats)):
    for key in ("stream_walk_kernel", "stream_decode_wide_kernel", "stream_decode_kernel"):
        if key in x["Name"]:
            k[key] = round(float(x["AverageNs"]) / 1000, 1)
d = json.loads([l for l in open(log) if l.startswith("{")][-1])
print(f"{lib:26s} {args:26s} walk {k.get('stream_walk_kernel')} decode {k.get('stream_decode_kernel') or k.get('stream_decode_wide_kernel')} us | call {d['ms']} ms {d['G_stream_samples_per_s']} G ok {d['frames_error_free']}/{d['frames_found']}")
PY
    done
  done
done
unset OFDM_MI355X_LIB
cat $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_stream_full.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04l_tests.log 2>&1; tail -3 gpurun_out/r04l_tests.log
