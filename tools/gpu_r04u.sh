#!/bin/bash
# round 4 (u): one context vs two alternating contexts (tools/stream_bench.py
# --pipeline 2) after the per-format decode and walker kernels, same box
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/r04u_pipeline_ab.txt; : > $OUT
for round in 1 2 3; do
  for args in "--i16" "" "--config B --frames 4096 --i16"; do
    for p in 1 2; do
      timeout -k 10 200 python3 tools/stream_bench.py --reps 10 --pipeline $p $args > gpurun_out/ab_sb.log 2>&1 || { tail gpurun_out/ab_sb.log; exit 1; }
      python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/ab_sb.log') if l.startswith('{')][-1])
print(f\"pipeline $p {'$args':32s} {d['ms']} ms {d['G_stream_samples_per_s']} G ok {d['frames_error_free']}/{d['frames_found']}\")" >> $OUT
    done
  done
done
cat $OUT
