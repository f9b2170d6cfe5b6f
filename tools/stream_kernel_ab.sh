#!/bin/bash
# Per-kernel times of the stream path for several library builds:
# rocprofv3 --kernel-trace --stats over tools/stream_bench.py per build.
# AB_LIBS="name:path ..." (path "-" = in-tree library)
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in $AB_LIBS; do
  name=${spec%%:*}; path=${spec#*:}
  if [ "$path" = "-" ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=$path; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sk_$name -o run -- python3 tools/stream_bench.py --reps 3 > gpurun_out/sk_$name.log 2>&1 || exit 1
  python3 - "$name" <<'PY' >> gpurun_out/stream_kernel_ab.txt
import csv, sys
name = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/sk_{name}/run_kernel_stats.csv")):
    if "ofdm" in r["Name"]:
        print(name, r["Name"].split("(")[0].replace("void ofdm::", ""), r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
