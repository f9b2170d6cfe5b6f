#!/bin/bash
# round 4 (q): the served demod's fused compare+clamp (drop-in MAC stage), and
# three wide-decode variants against the product build, same box:
#   v2  = the rx stage's next-symbol samples fetched after each transform, the
#         first symbol's during the sync tail;  v2b = the in-loop fetch only;
#   v3  = no wave priority in the wide kernel
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/dropin_rx_timing.py --frames 200 > gpurun_out/r04q_dropin.json 2> gpurun_out/r04q_dropin.err || { tail gpurun_out/r04q_dropin.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04q_dropin.json')); print('dropin', d['median_us'], d['stage_median_us'], d['frames_payload_exact'], d['frames_written'])"
for v in v2 v2b; do
  OFDM_MI355X_LIB=$R/abtest/libofdm_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -k "wide or config_b" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04q_tests_$v.log 2>&1 || { tail -30 gpurun_out/r04q_tests_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/r04q_tests_$v.log)"
done
OUT=gpurun_out/r04q_wide_ab.txt; : > $OUT
for round in 1 2; do
  for v in base v2 v2b v3; do
    if [ $v = base ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=$R/abtest/libofdm_$v.so; fi
    for args in "--config B --frames 4096" "--config B --frames 4096 --i16"; do
      D=$R/gpurun_out/ab_prof; rm -rf $D
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/stream_bench.py --reps 5 $args > gpurun_out/ab_sb.log 2>&1 || { tail gpurun_out/ab_sb.log; exit 1; }
      python3 - "$v" "$args" "$D/run_kernel_stats.csv" gpurun_out/ab_sb.log >> $OUT <<'PY'
import csv, json, sys
v, args, stats, log = sys.argv[1:5]
k = []
for x in csv.DictReader(open(stats)):
    if "stream_decode_wide" in x["Name"] or "stream_walk" in x["Name"]:
        k.append((x["Name"].split("(")[0].replace("void ofdm::", ""), round(float(x["AverageNs"]) / 1000, 1)))
d = json.loads([l for l in open(log) if l.startswith("{")][-1])
print(f"{v:5s} {args:32s} {k} | call {d['ms']} ms {d['G_stream_samples_per_s']} G ok {d['frames_error_free']}/{d['frames_found']}")
PY
    done
  done
done
unset OFDM_MI355X_LIB
cat $OUT
