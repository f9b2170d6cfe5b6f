#!/bin/bash
# End-of-session GPU pass: parity tests, smoke(), the driver bench, and the
# config-4 stream bench (f64 + int16) with its kernel-stats profile.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stream -o run -- python3 tools/stream_bench.py --reps 5 > gpurun_out/stream_prof.json 2> gpurun_out/stream_prof.err || exit 1
timeout -k 10 300 python tools/stream_bench.py --cpu-seconds 12 > gpurun_out/stream_final.json 2> gpurun_out/stream_final.err || exit 1
timeout -k 10 200 python tools/stream_bench.py --i16 >> gpurun_out/stream_final.json 2>> gpurun_out/stream_final.err
