#!/bin/bash
# the headline's dependence on warmup (driver: --steps 20 --warmup 5), same box:
# "first" = the headline alone (as the first GPU work of the process, cold
# clocks); "last" = bench.py's order (the sub-records' GPU work first)
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/r05_warmup.txt; : > $OUT
for r in 1 2; do
  for w in 5 10 50; do
    for order in first last; do
      extra="--no-stream --no-config3"
      [ $order = last ] && extra=""
      timeout -k 10 400 python bench.py --steps 20 --warmup $w --no-cpu-baseline $extra > gpurun_out/wu.json 2> gpurun_out/wu.err || { tail gpurun_out/wu.err; exit 1; }
      python3 -c "
import json; d=json.load(open('gpurun_out/wu.json'))
print('warmup $w headline $order', round(d['value']/1e9,2), 'G', 'ms/step', round(d['ms_per_step'],4), 'rx', round(d['roofline']['avg_launch_ms'],4), 'frac', round(d['roofline']['frac'],4), 'tx', round(d['tx_avg_launch_ms'],4))" >> $OUT
    done
  done
done
cat $OUT
