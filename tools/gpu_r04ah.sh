#!/bin/bash
# round 4 (ah): rx_kernel wave priority by phase (pa: symbol loop 1, epilogue
# 0; pb: the reverse) against the product build: bench.py's step per kernel
# (tools/ab_step.py), three interleaved rounds, same box
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/r04ah_rx_priority_ab.txt; : > $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "rx" > gpurun_out/r04ah_tests.log 2>&1 || { tail -20 gpurun_out/r04ah_tests.log; exit 1; }
for v in pa pb; do
  OFDM_MI355X_LIB=$R/abtest/libofdm_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "rx" > gpurun_out/r04ah_tests_$v.log 2>&1 || { tail -20 gpurun_out/r04ah_tests_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/r04ah_tests_$v.log)"
done
for round in 1 2 3; do
  for v in product pa pb; do
    if [ $v = product ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=$R/abtest/libofdm_$v.so; fi
    timeout -k 10 200 python3 tools/ab_step.py >> $OUT 2> gpurun_out/r04ah.err || { tail gpurun_out/r04ah.err; exit 1; }
  done
done
unset OFDM_MI355X_LIB
cat $OUT
