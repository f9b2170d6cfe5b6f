#!/bin/bash
# round 2: decision-boundary + drop-in file-contract tests, compat timing, bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_decision_boundary.py tests/test_dropin_gpu.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r02b_tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/dropin_rx_timing.py > gpurun_out/r02b_dropin_rx_timing.json 2> gpurun_out/r02b_dropin.err || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r02b_bench.json 2> gpurun_out/r02b_bench.err || exit 1
