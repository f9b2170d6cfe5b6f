#!/bin/bash
# round 4 (aa): the drop-in's pilot_freq_sinh answer written by the CFO kernel
# straight to a pinned word (no copy launch, no event wait): drop-in GPU tests
# and the rx.cpp stage timing
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dropin_gpu.py tests/test_gpu_sync.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04aa_tests.log 2>&1 || { tail -30 gpurun_out/r04aa_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r04aa_tests.log)"
for i in 1 2; do
  timeout -k 10 300 python3 -u tools/dropin_rx_timing.py --frames 200 > gpurun_out/r04aa_dropin_$i.json 2> gpurun_out/r04aa_dropin.err || { tail gpurun_out/r04aa_dropin.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r04aa_dropin_$i.json')); print('dropin', d['median_us'], d['stage_median_us'], d['frames_payload_exact'], d['frames_written'], d['frames_in_order'])"
done
