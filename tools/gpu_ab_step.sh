#!/bin/bash
# same-box A/B of library variants on bench.py's step (tools/ab_step.py,
# back-to-back steps): LIBS="abtest/libofdm_a.so abtest/libofdm_b.so", ROUNDS
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/ab_step.txt; : > $OUT
for r in $(seq 1 ${ROUNDS:-3}); do
  for lib in $LIBS; do
    OFDM_MI355X_LIB=$PWD/$lib timeout -k 10 120 python3 tools/ab_step.py >> $OUT 2> gpurun_out/ab_step.err || { tail gpurun_out/ab_step.err; exit 1; }
  done
done
cat $OUT
