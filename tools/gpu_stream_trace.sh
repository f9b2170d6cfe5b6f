#!/bin/bash
# kernel trace of bench.py's stream legs (serial calls): per-call
# walker / resolve / decode times and the gaps between them; and per-workload
# kernel means of stream_bench.py (profiles/stream_kernels_*.json)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
D=$R/gpurun_out/st_prof; rm -rf $D
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 bench.py --no-cpu-baseline --no-config3 --stream-pipeline 1 --steps 5 --warmup 5 > gpurun_out/st_bench.json 2> gpurun_out/st_bench.err || { tail gpurun_out/st_bench.err; exit 1; }
python3 tools/stream_trace_calls.py $D/run_kernel_trace.csv 10 > gpurun_out/stream_calls.json && cat gpurun_out/stream_calls.json
ARGS=""
for spec in "config4_stream_D_frames_gaps0-4096_cfo0.004_awgn20dB:--frames 16384" "config4_stream_D_frames_gaps0-4096_cfo0.004_awgn20dB_int16:--frames 16384 --i16" "config4_stream_B_frames_gaps0-4096_cfo0.004_awgn20dB:--config B --frames 4096"; do
  w=${spec%%:*}; a=${spec#*:}
  D=$R/gpurun_out/sk_$w; rm -rf $D
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 tools/stream_bench.py --reps 10 $a > gpurun_out/sk_$w.log 2>&1 || { tail gpurun_out/sk_$w.log; exit 1; }
  tail -1 gpurun_out/sk_$w.log
  ARGS="$ARGS $w=$D/run_kernel_trace.csv"
done
python3 tools/stream_kernels.py gpurun_out/stream_kernels.json 10 $ARGS > /dev/null && cat gpurun_out/stream_kernels.json
