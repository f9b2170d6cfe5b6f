#!/bin/bash
# round 2: sharded stream + multi-rank bench checks, full GPU suite, bench with stream legs
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream_shard.py tests/test_bench_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r02a_new_tests.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02a_gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r02a_bench.json 2> gpurun_out/r02a_bench.err || exit 1
