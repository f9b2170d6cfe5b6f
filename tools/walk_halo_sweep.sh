#!/bin/bash
# Walk-in halo sweep on the config-4 stream (ofdm_walk_tuning halo_milli, 1/1000 frames):
# stream time and re-walks per setting. Output: gpurun_out/halo_sweep.txt
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/halo_sweep.txt
for h in ${HALOS:-3000 2000 1700 1500 1200}; do
  OFDM_STREAM_DEBUG=1 timeout -k 10 120 python tools/stream_bench.py --reps 5 --walk-tuning halo_milli=$h > gpurun_out/hs.json 2> gpurun_out/hs.err || exit 1
  rw=$(grep -c "re-walk chunk" gpurun_out/hs.err || true)
  echo "halo=$h rewalk_lines=$rw $(python3 -c "import json;d=json.loads(open('gpurun_out/hs.json').read().splitlines()[-1]);print(d['G_stream_samples_per_s'], d['ms'])")" >> gpurun_out/halo_sweep.txt
done
cat gpurun_out/halo_sweep.txt
