#!/bin/bash
# GPU tests, then bench.py (no CPU baseline) for each library variant, twice:
# VARIANTS="name:lib name2: ..." (empty lib = the product build).
# Output: gpurun_out/bench_ab.txt
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in $VARIANTS; do
    n=${v%%:*}; l=${v#*:}
    if [ -n "$l" ]; then export OFDM_MI355X_LIB=$l; else unset OFDM_MI355X_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | sed "s/^/$n /" >> gpurun_out/bench_ab.txt || exit 1
  done
done
unset OFDM_MI355X_LIB
