#!/bin/bash
# Walker chunking sweep (chunks per walker slot x halo), config-4 stream bench;
# stream tests first. Output: gpurun_out/walk_q_sweep.txt
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/stream_tests.log 2>&1 || exit 1
export OFDM_STREAM_DEBUG=1
for cfg in ${SWEEP:-1:3000:2000 1:1500:2000 2:1500:2000}; do  # Q:halo:ext
  set -- ${cfg//:/ }
  for r in 1 2; do
    timeout -k 10 120 python tools/stream_bench.py --reps 5 --walk-tuning chunks_per_slot=$1,halo_milli=$2,ext_milli=$3 > gpurun_out/wq.json 2> gpurun_out/wq.err || exit 1
    echo "Q=$1 halo=$2 ext=$3 $(tail -1 gpurun_out/wq.err) $(python3 -c "import json;d=json.load(open('gpurun_out/wq.json'));print(d['ms'],d['G_stream_samples_per_s'])")" >> gpurun_out/walk_q_sweep.txt
  done
done
