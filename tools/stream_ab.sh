#!/bin/bash
# Same-box A/B of library builds on the config-4 stream: for each library in
# $LIBS (paths; "product" = c-ofdm_amd/lib), alternately, tools/stream_bench.py
# (f64 and --i16) under rocprofv3 --kernel-trace --stats; prints per-kernel
# average durations (walker, compaction, decode) and the call time.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
OUT=$R/gpurun_out/${TAG:-ab}_stream_ab.txt
: > $OUT
for round in 1 2; do
  for lib in $LIBS; do
    for mode in "" "--i16"; do
      if [ "$lib" = product ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=$R/$lib; fi
      D=$R/gpurun_out/ab_prof
      rm -rf $D
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/stream_bench.py --reps 5 $mode > $R/gpurun_out/ab_sb.log 2>&1 || { tail $R/gpurun_out/ab_sb.log; exit 1; }
      python3 - "$lib" "$mode" "$D/run_kernel_stats.csv" "$R/gpurun_out/ab_sb.log" >> $OUT <<'PY'
import csv, json, sys
lib, mode, stats, log = sys.argv[1:5]
k = {}
for x in csv.DictReader(open(stats)):
    for key in ("stream_walk_kernel", "compact_kernel", "resolve_kernel", "stream_decode_kernel"):
        if key in x["Name"]:
            k[key] = round(float(x["AverageNs"]) / 1000, 1)
line = [l for l in open(log) if l.startswith("{")][-1]
d = json.loads(line)
print(f"{lib:28s} {mode or 'f64':6s} walk {k.get('stream_walk_kernel')} compact {k.get('compact_kernel')} "
      f"resolve {k.get('resolve_kernel')} decode {k.get('stream_decode_kernel')} us | call {d['ms']} ms {d['G_stream_samples_per_s']} G")
PY
    done
  done
done
unset OFDM_MI355X_LIB
cat $OUT
