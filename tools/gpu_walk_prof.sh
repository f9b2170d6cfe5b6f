#!/bin/bash
# walker timelines (OFDM_WALK_PROF) of stream_bench.py calls, f64 / int16,
# look-back with 1 and 2 chunks per slot and the halo walk (TUNINGS=... to pick)
export TMPDIR=/tmp
mkdir -p gpurun_out
for tun in ${TUNINGS:-chunks_per_slot=1 chunks_per_slot=2 lookback=0}; do
  for args in "--frames 16384" "--frames 16384 --i16"; do
    tag=$(echo "$tun$args" | tr -c 'a-z0-9' '_')
    rm -f gpurun_out/wp_$tag.jsonl
    OFDM_WALK_PROF=gpurun_out/wp_$tag.jsonl timeout -k 10 200 python3 tools/stream_bench.py --reps 3 --walk-tuning $tun $args > gpurun_out/wp_sb.log 2>&1 || { tail gpurun_out/wp_sb.log; exit 1; }
    python3 tools/walk_prof_summary.py gpurun_out/wp_$tag.jsonl 2 > gpurun_out/wp_$tag.summary.json
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/wp_$tag.summary.json'))['calls'][-1]
print('$tun $args', 'span', d['kernel_span_us'], 'walker pct', d['walker_us_pct_0_10_50_90_99_100'], 'mean', d['walker_mean_us'], 'start pct', d['start_us_pct'], 'ext', d['ext_frames_hist'], 'waits', d['waits_total'], d['chunks_that_waited'])
print('   phases', d.get('phases'))
print('   tail', [(t['chunk'], t['start_us'], t['end_us'], t['core_us'], t['ext_frames'], t['waits'], t['nrec']) for t in d['tail_chunks'][:5]])
"
  done
done
