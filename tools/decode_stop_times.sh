#!/bin/bash
# Kernel time of the fused stream decode (stream_decode_kernel, N = 512)
# ended at each stop point (OFDM_DECODE_STOP=k, the diagnostics
# instantiation; 0 = the product kernel): how the decode's time accumulates
# over its segments (1 = pilot_freq_sinh, 2 = rest of the sync stage, 3 = the
# message transforms, 4 = channel line / phys / gains, 5 = emit). Args: extra
# stream_bench args (e.g. --i16).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
TAG=${TAG:-dst}
OUT=$R/gpurun_out/${TAG}_decode_stop_times.txt; : > $OUT
for k in 1 2 3 4 5 0; do
  D=$R/gpurun_out/${TAG}_t$k; rm -rf $D
  if [ $k = 0 ]; then unset OFDM_DECODE_STOP; else export OFDM_DECODE_STOP=$k; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/stream_bench.py --reps 5 "$@" > $D.log 2>&1 || { tail $D.log; exit 1; }
  python3 - "$k" "$D/run_kernel_stats.csv" >> $OUT <<'PY'
import csv, sys
k, stats = sys.argv[1:3]
for x in csv.DictReader(open(stats)):
    if "stream_decode_kernel" in x["Name"]:
        print(f"stop {k}: {x['Name'].split('(')[0].replace('void ofdm::', '')[:48]} calls {x['Calls']} mean {float(x['AverageNs'])/1000:.1f} us")
PY
done
unset OFDM_DECODE_STOP
cat $OUT
