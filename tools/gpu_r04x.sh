#!/bin/bash
# round 4 (x): wide decode variants (V=name: abtest/libofdm_$V.so) against the
# product build, same box (x: CP sums on every wave; y: opaque per-symbol index, no spills)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=${V:-cp}
for v in $V; do
  OFDM_MI355X_LIB=$R/abtest/libofdm_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -k "wide or config_b" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04x_tests.log 2>&1 || { tail -30 gpurun_out/r04x_tests.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/r04x_tests.log)"
done
OUT=gpurun_out/r04x_wide_ab.txt; : > $OUT
for round in 1 2 3; do
  for v in base $V; do
    if [ $v = base ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=$R/abtest/libofdm_$v.so; fi
    for args in "--config B --frames 4096" "--config B --frames 4096 --i16"; do
      D=$R/gpurun_out/ab_prof; rm -rf $D
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/stream_bench.py --reps 5 $args > gpurun_out/ab_sb.log 2>&1 || { tail gpurun_out/ab_sb.log; exit 1; }
      python3 - "$v" "$args" "$D/run_kernel_stats.csv" gpurun_out/ab_sb.log >> $OUT <<'PY'
import csv, json, sys
v, args, stats, log = sys.argv[1:5]
k = []
for x in csv.DictReader(open(stats)):
    if "stream_decode" in x["Name"]:
        k.append((x["Name"].split("(")[0].replace("void ofdm::", ""), round(float(x["AverageNs"]) / 1000, 1)))
d = json.loads([l for l in open(log) if l.startswith("{")][-1])
print(f"{v:5s} {args:32s} {k} | call {d['ms']} ms {d['G_stream_samples_per_s']} G ok {d['frames_error_free']}/{d['frames_found']}")
PY
    done
  done
done
unset OFDM_MI355X_LIB
cat $OUT
