#!/bin/bash
# the look-back walk (device-side stitching, no walk-in halo) against
# the round-4 halo walk with host stitching (walk tuning lookback=0), same box:
# per-kernel mean times from rocprofv3 --kernel-trace --stats of stream_bench.py
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "config3_bench" -x -v --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_config3_test.log 2>&1; tail -3 gpurun_out/r05_config3_test.log
OUT=gpurun_out/r05_lookback_ab.txt; : > $OUT
for round in 1 2; do
  for lb in 0 1; do
    for args in "--frames 16384" "--frames 16384 --i16" "--config B --frames 4096"; do
      D=$R/gpurun_out/ab_prof; rm -rf $D
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/stream_bench.py --reps 10 --walk-tuning lookback=$lb $args > gpurun_out/ab_sb.log 2>&1 || { tail gpurun_out/ab_sb.log; exit 1; }
      python3 - "lb=$lb" "$args" "$D/run_kernel_stats.csv" gpurun_out/ab_sb.log >> $OUT <<'PY'
import csv, json, sys
v, args, stats, log = sys.argv[1:5]
k = []
for x in csv.DictReader(open(stats)):
    if any(s in x["Name"] for s in ("stream_decode", "stream_walk", "resolve", "compact")):
        k.append((x["Name"].split("(")[0].replace("void ofdm::", "").split("<")[0], round(float(x["AverageNs"]) / 1000, 1), int(x["Calls"])))
d = json.loads([l for l in open(log) if l.startswith("{")][-1])
print(f"{v:5s} {args:28s} {k} | call {d['ms']} ms {d['G_stream_samples_per_s']} G found {d['frames_found']} ok {d['frames_error_free']}")
PY
    done
  done
done
cat $OUT
