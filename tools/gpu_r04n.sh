#!/bin/bash
# wide decode: fused (one kernel) vs split (sync kernel + rx kernel), same box
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
OFDM_WIDE_SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -k "wide or config_b" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04n_tests.log 2>&1; tail -2 gpurun_out/r04n_tests.log
OUT=gpurun_out/r04n_split_ab.txt; : > $OUT
for round in 1 2; do
  for mode in fused split; do
    for args in "--config B --frames 4096" "--config B --frames 4096 --i16" "--config C --frames 2048"; do
      if [ $mode = split ]; then export OFDM_WIDE_SPLIT=1; else unset OFDM_WIDE_SPLIT; fi
      D=$R/gpurun_out/ab_prof; rm -rf $D
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/stream_bench.py --reps 5 $args > gpurun_out/ab_sb.log 2>&1 || { tail gpurun_out/ab_sb.log; exit 1; }
      python3 - "$mode" "$args" "$D/run_kernel_stats.csv" gpurun_out/ab_sb.log >> $OUT <<'PY'
import csv, json, sys
mode, args, stats, log = sys.argv[1:5]
k = []
for x in csv.DictReader(open(stats)):
    if "stream_decode_wide" in x["Name"] or "stream_walk" in x["Name"]:
        k.append((x["Name"].split("(")[0].replace("void ofdm::", ""), round(float(x["AverageNs"]) / 1000, 1)))
d = json.loads([l for l in open(log) if l.startswith("{")][-1])
print(f"{mode:6s} {args:32s} {k} | call {d['ms']} ms {d['G_stream_samples_per_s']} G ok {d['frames_error_free']}/{d['frames_found']}")
PY
    done
  done
done
unset OFDM_WIDE_SPLIT
cat $OUT
