#!/bin/bash
# per-step device times of the headline over 60 timed steps after 5 warmup
# steps: alone (cold start) and in bench.py's order (sub-records first)
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/r05_ramp.txt; : > $OUT
for order in first last; do
  extra="--no-stream --no-config3"
  [ $order = last ] && extra=""
  timeout -k 10 400 python bench.py --steps 60 --warmup 5 --no-cpu-baseline $extra > gpurun_out/ramp_$order.json 2> gpurun_out/ramp.err || { tail gpurun_out/ramp.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ramp_$order.json'))
s=d['step_ms']
print('$order', round(d['value']/1e9,2), 'G; step ms in groups of 10:', [round(sum(s[i:i+10])/10,4) for i in range(0,len(s),10)])
print('   first 12:', s[:12])
c=d.get('config3')
if c: print('   config3 step ms:', c['step_ms'])" >> $OUT
done
cat $OUT
