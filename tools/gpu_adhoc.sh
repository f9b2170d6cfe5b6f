#!/bin/bash
# scratch slot for one-off GPU commands (overwritten per experiment)
# current: stream parity tests + per-kernel stream means (walker A/B: packed FP32 T2 screen)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
TAG=${1:-r06b}
timeout -k 10 900 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_stream_full.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
ARGS=""
for spec in "config4_stream_D_frames_gaps0-4096_cfo0.004_awgn20dB:--frames 16384" "config4_stream_D_frames_gaps0-4096_cfo0.004_awgn20dB_int16:--frames 16384 --i16"; do
  w=${spec%%:*}; a=${spec#*:}
  D=$R/gpurun_out/sk_$w; rm -rf $D
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 tools/stream_bench.py --reps 10 $a > gpurun_out/sk_$w.log 2>&1 || { tail gpurun_out/sk_$w.log; exit 1; }
  tail -1 gpurun_out/sk_$w.log
  ARGS="$ARGS $w=$D/run_kernel_trace.csv"
done
python3 tools/stream_kernels.py gpurun_out/${TAG}_stream_kernels.json 10 $ARGS > /dev/null && cat gpurun_out/${TAG}_stream_kernels.json
TAG=${TAG}_dp bash tools/decode_phase_counts.sh --frames 16384 > gpurun_out/${TAG}_decode_phases.json && cat gpurun_out/${TAG}_decode_phases.json
