#!/bin/bash
# round 4 (ac): full GPU pass (tests, smoke, bench) and the drop-in timing after
# the CFO kernel's system fence was limited to ofdm_cfo_estimate's calls
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_full.sh r04ac && \
timeout -k 10 300 python3 -u tools/dropin_rx_timing.py --frames 200 > gpurun_out/r04ac_dropin.json 2> gpurun_out/r04ac_dropin.err && \
python3 -c "import json; d=json.load(open('gpurun_out/r04ac_dropin.json')); print('dropin', d['median_us'], d['stage_median_us'], d['frames_payload_exact'], d['frames_written'], d['frames_in_order'])"
