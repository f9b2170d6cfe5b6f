#!/bin/bash
# scratch slot for one-off GPU commands (overwritten per experiment)
# current: AWGN scale folded into FP32 + FMA emit (product build) vs HEAD (abtest/libofdm_head.so); tx parity tests
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/awgnfold.txt
: > $O
for rep in 1 2 3; do
  OFDM_MI355X_LIB=abtest/libofdm_head.so timeout -k 10 120 python tools/ab_step.py 2>/dev/null | sed "s/^/head /" >> $O || exit 1
  timeout -k 10 120 python tools/ab_step.py 2>/dev/null | sed "s/^/fold /" >> $O || exit 1
done
cat $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_gpu.py tests/test_gpu_config5.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/awgnfold_tests.log 2>&1; tail -3 gpurun_out/awgnfold_tests.log
