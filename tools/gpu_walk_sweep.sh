#!/bin/bash
# look-back walker tuning sweep (chunks per walker slot x walk-in
# halo) on stream_bench.py, per-kernel means from rocprofv3 --stats; the
# stream parity tests first
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05b_stream_tests.log 2>&1 || { tail -40 gpurun_out/r05b_stream_tests.log; exit 1; }
tail -1 gpurun_out/r05b_stream_tests.log
OUT=gpurun_out/r05b_walk_sweep.txt; : > $OUT
for tun in "lookback=0" "chunks_per_slot=1" "chunks_per_slot=2" "chunks_per_slot=3" "chunks_per_slot=4" "chunks_per_slot=1,halo_milli=100" "chunks_per_slot=2,halo_milli=100"; do
    for args in "--frames 16384" "--frames 16384 --i16" "--config B --frames 4096"; do
      D=$R/gpurun_out/ab_prof; rm -rf $D
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/stream_bench.py --reps 10 --walk-tuning $tun $args > gpurun_out/ab_sb.log 2>&1 || { tail gpurun_out/ab_sb.log; exit 1; }
      python3 - "$tun" "$args" "$D/run_kernel_stats.csv" gpurun_out/ab_sb.log >> $OUT <<'PY'
import csv, json, sys
v, args, stats, log = sys.argv[1:5]
k = []
for x in csv.DictReader(open(stats)):
    if any(s in x["Name"] for s in ("stream_decode", "stream_walk", "resolve", "compact")):
        k.append((x["Name"].split("(")[0].replace("void ofdm::", "").replace("ofdm::", "").split("<")[0], round(float(x["AverageNs"]) / 1000, 1)))
d = json.loads([l for l in open(log) if l.startswith("{")][-1])
print(f"{v:34s} {args:26s} {k} | call {d['ms']} ms {d['G_stream_samples_per_s']} G found {d['frames_found']} ok {d['frames_error_free']}")
PY
    done
done
cat $OUT
